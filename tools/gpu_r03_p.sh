#!/bin/bash
# Round 3 session P: which change removes xform_h8's intermittent reconstruct mismatches:
# no early retire, a barrier between IFFT and FFT, or workgroup barriers in the swaps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in libalpenglow_rs.so lib_noret.so lib_mid.so lib_nops.so; do
  AG_RS_LIB_NAME=$lib timeout -k 10 240 python3 tools/stress_xform64.py --variants 9 --iters 60 --n 64 --S 2048 > gpurun_out/p.txt 2>&1
  rc=$?; echo "$lib exit $rc"; tail -n 1 gpurun_out/p.txt; [ $rc = 0 ] || exit $rc
done
exit 0
