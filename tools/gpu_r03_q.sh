#!/bin/bash
# Round 3 session Q: xform_h8 mismatch map; DPP vs ds_swizzle quad exchange.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in libalpenglow_rs.so; do
  AG_RS_LIB_NAME=$lib timeout -k 10 240 python3 tools/stress_xform64.py --variants 9 --iters 30 --n 64 --S 2048 > gpurun_out/q_$lib.txt 2>&1
  rc=$?; echo "$lib exit $rc"; grep -A2 "iter" gpurun_out/q_$lib.txt | head -12; tail -n 1 gpurun_out/q_$lib.txt; [ $rc = 0 ] || exit $rc
done
exit 0
