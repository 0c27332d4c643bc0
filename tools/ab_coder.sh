#!/bin/bash
# Interleaved A/B of library builds (alpenglow_amd/_lib/<lib>.so, AG_RS_LIB_NAME) on the batched
# coder bench: for each round and lib, one bench_coder.py line per arrival shape into
# gpurun_out/ab_coder.jsonl (fields lib, shape, round added).  A failing run stops the session.
#   tools/ab_coder.sh ROUNDS "LIB_A LIB_B ..." ["SHAPE_ARGS" ...]   (default shape: --random-patterns)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rounds=$1; libs=$2; shift 2
[ $# -gt 0 ] || set -- "--random-patterns"
for r in $(seq 1 $rounds); do
  for shape in "$@"; do
    for lib in $libs; do
      AG_RS_LIB_NAME=$lib.so timeout -k 10 200 python3 bench_coder.py $shape --steps 5 --warmup 2 --no-cpu-baseline \
        > gpurun_out/abc_pt.json 2> gpurun_out/abc_pt.err
      rc=$?; [ $rc = 0 ] || { tail -3 gpurun_out/abc_pt.err; echo "STOP $lib $shape exit $rc"; exit $rc; }
      python3 - "$lib" "$shape" "$r" <<'PY'
import json, sys
lib, shape, r = sys.argv[1:4]
d = json.loads(open("gpurun_out/abc_pt.json").read().strip().splitlines()[-1])
d.update(lib=lib, shape=shape, round=int(r))
open("gpurun_out/ab_coder.jsonl", "a").write(json.dumps(d) + "\n")
print(r, shape, lib, round(d["value"] / 1e6, 3), "M slices/s", "verify", d.get("verify"))
PY
    done
  done
done
exit 0
