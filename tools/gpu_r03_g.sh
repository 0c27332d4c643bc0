#!/bin/bash
# Round 3 session G: full GPU parity + smoke + headline bench, then a kernel trace of the
# CodingOnly random-arrival coder batch (W = 128 per-lane windows).  Every GPU step
# time-limited; a failing step ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu exit $rc"; tail -5 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke exit $rc"; tail -2 gpurun_out/smoke.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench exit $rc"; cat gpurun_out/bench.json; [ $rc = 0 ] || { tail -5 gpurun_out/bench.err; exit $rc; }
rm -rf gpurun_out/kt_co
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_co -o kt --output-format csv -- \
  python3 bench_coder.py --coding-only --random-patterns --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/co.json 2> gpurun_out/kt_co.err
echo "kt exit $?"; tail -1 gpurun_out/co.json
find gpurun_out/kt_co -name "*kernel_stats.csv" -exec head -16 {} \;
exit 0
