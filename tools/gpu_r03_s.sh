#!/bin/bash
# Round 3 session S: packed store predicates in every transform kernel -- stress, full GPU
# suite, A/B against the previous commit (libhead.so) on the headline and C4 shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "--n 64 --S 2048" "--n 33 --S 1024"; do
  timeout -k 10 240 python3 tools/stress_xform64.py --variants 0,9,10,7 --iters 40 $cfg > gpurun_out/s.txt 2>&1
  rc=$?; echo "stress $cfg exit $rc"; grep -A2 "iter" gpurun_out/s.txt | head -6; tail -n 1 gpurun_out/s.txt; [ $rc = 0 ] || exit $rc
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu exit $rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || exit $rc
LIBAB_CFGS="32:32:0 64:64:0 16:4:0 32:32:8" bash tools/gpu_libab.sh || exit 1
exit 0
