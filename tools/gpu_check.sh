#!/bin/bash
# One GPU session: parity tests, smoke, bench, kernel-trace profile.  Every GPU step has
# its own time limit; a fault/abort/timeout ends the script (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
export TMPDIR=/tmp
stop_on_fatal() {  # $1 = exit code of a GPU step
  case "$1" in
    0|1) return 0 ;;                      # pass / ordinary test failure
    *) echo "FATAL step exit $1: stopping GPU work"; exit "$1" ;;
  esac
}
rocm-smi --showproductname > $OUT/rocm_smi.txt 2>&1 || true
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu exit $rc"; tail -5 $OUT/pytest_gpu.log; stop_on_fatal $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke exit $rc"; tail -3 $OUT/smoke.log; stop_on_fatal $rc
[ "${SKIP_BENCH:-0}" = 1 ] && exit 0
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench exit $rc"; cat $OUT/bench.json; tail -3 $OUT/bench.err; stop_on_fatal $rc
[ "${SKIP_PROF:-0}" = 1 ] && exit 0
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o kt --output-format csv -- \
  python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-verify > $OUT/prof_bench.json 2> $OUT/prof.err
rc=$?; echo "rocprof exit $rc"; stop_on_fatal $rc
find $OUT/prof -name "*stats*" | head
exit 0
