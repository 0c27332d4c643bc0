#!/bin/bash
# Round 3 session O: intermittent-result hunt in the 64-point per-block-mask decode.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in libalpenglow_rs.so libll.so; do
  for cfg in "--n 9 --S 1024" "--n 64 --S 2048" "--n 33 --S 1024"; do
    AG_RS_LIB_NAME=$lib timeout -k 10 240 python3 tools/stress_xform64.py --variants 9,10 --iters 40 $cfg > gpurun_out/o.txt 2>&1
    rc=$?; echo "$lib $cfg exit $rc"; tail -4 gpurun_out/o.txt; [ $rc = 0 ] || exit $rc
  done
done
exit 0
