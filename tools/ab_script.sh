#!/bin/bash
# Interleaved A/B of library builds (alpenglow_amd/_lib/<lib>.so, AG_RS_LIB_NAME) on any bench
# script that prints one JSON line with "value": for each round and lib one line into
# gpurun_out/ab_script.jsonl (fields lib, script, round added).  A failing run stops the session.
#   tools/ab_script.sh ROUNDS "LIB_A LIB_B ..." SCRIPT [ARGS...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rounds=$1; libs=$2; script=$3; shift 3
for r in $(seq 1 $rounds); do
  for lib in $libs; do
    AG_RS_LIB_NAME=$lib.so timeout -k 10 200 python3 $script "$@" > gpurun_out/abs_pt.json 2> gpurun_out/abs_pt.err
    rc=$?; [ $rc = 0 ] || { tail -3 gpurun_out/abs_pt.err; echo "STOP $lib $script exit $rc"; exit $rc; }
    python3 - "$lib" "$script $*" "$r" <<'PY'
import json, sys
lib, script, r = sys.argv[1:4]
d = json.loads(open("gpurun_out/abs_pt.json").read().strip().splitlines()[-1])
d.update(lib=lib, script=script, round=int(r))
open("gpurun_out/ab_script.jsonl", "a").write(json.dumps(d) + "\n")
print(r, script, lib, round(d["value"], 1), d.get("unit"), "verify", d.get("verify"))
PY
  done
done
exit 0
