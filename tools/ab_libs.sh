#!/bin/bash
# Interleaved A/B of two builds of the library on one box (alpenglow_amd/_lib/<lib>, selected
# with AG_RS_LIB_NAME): for each round, each point, each lib one bench.py line into
# gpurun_out/ab.jsonl (fields lib, point, round added).  A failing run stops the session.
#   tools/ab_libs.sh ROUNDS "LIB_A LIB_B ..." "label:args" ["label:args" ...]   (args comma-separated)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rounds=$1; libs=$2; shift 2
for r in $(seq 1 $rounds); do
  for pt in "$@"; do
    label=${pt%%:*}; args=${pt#*:}; args=${args//,/ }
    for lib in $libs; do
      AG_RS_LIB_NAME=$lib timeout -k 10 200 python3 bench.py --steps 10 --warmup 10 --no-cpu-baseline $args \
        > gpurun_out/ab_pt.json 2> gpurun_out/ab_pt.err
      rc=$?; [ $rc = 0 ] || { tail -3 gpurun_out/ab_pt.err; echo "STOP $lib $label exit $rc"; exit $rc; }
      python3 - "$lib" "$label" "$r" <<'PY'
import json, sys
lib, label, r = sys.argv[1:4]
d = json.loads(open("gpurun_out/ab_pt.json").read().strip().splitlines()[-1])
d.update(lib=lib, point=label, round=int(r))
open("gpurun_out/ab.jsonl", "a").write(json.dumps(d) + "\n")
k = d["kernels"]
print(r, label, lib, {n: round(v["achieved_GBps"] / 1000, 3) for n, v in k.items()}, "verify", d["verify"]["all_ranks_ok"])
PY
    done
  done
done
exit 0
