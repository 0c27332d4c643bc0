#!/bin/bash
# Round 3 session H: GPU parity (new CodingOnly device-pattern coder path), NT-load A/B on the
# non-headline kernels (libhead.so = previous commit), coder benches.  Every GPU step
# time-limited; a failing step ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu exit $rc"; tail -5 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || exit $rc
LIBAB_CFGS="32:32:0 64:64:0 16:4:0 32:32:8 32:32:16" bash tools/gpu_libab.sh || exit 1
: > gpurun_out/h.jsonl
for a in "--random-patterns" "--coding-only --random-patterns" "--coding-only"; do
  timeout -k 10 300 python3 bench_coder.py $a --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/h.json 2> gpurun_out/h.err
  rc=$?; echo "bench_coder '$a' exit $rc"; [ $rc = 0 ] || { tail -5 gpurun_out/h.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/h.json').read().strip().splitlines()[-1]); d['args']='$a'; print(json.dumps(d))" >> gpurun_out/h.jsonl
  python3 -c "import json; d=json.loads(open('gpurun_out/h.json').read().strip().splitlines()[-1]); print(round(d['value']/1e6,2), 'M slices/s', d['calls_ms'], d['verify'])"
done
rm -rf gpurun_out/kt_co
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_co -o kt --output-format csv -- \
  python3 bench_coder.py --coding-only --random-patterns --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2> gpurun_out/kt_co.err
echo "kt exit $?"
find gpurun_out/kt_co -name "*kernel_stats.csv" -exec head -12 {} \;
exit 0
