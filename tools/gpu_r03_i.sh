#!/bin/bash
# Round 3 session I: W = 128 per-lane passes on decode_h8 with the deferred output multiply
# (and the deferred multiply in decode_x16's passes): parity, coder benches, 64:64 lost-coding
# window-128 points, kernel trace.  Every GPU step time-limited; a failing step ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu exit $rc"; tail -5 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || exit $rc
: > gpurun_out/i.jsonl
for a in "--random-patterns" "--coding-only --random-patterns"; do
  timeout -k 10 300 python3 bench_coder.py $a --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/i.json 2> gpurun_out/i.err
  rc=$?; echo "bench_coder '$a' exit $rc"; [ $rc = 0 ] || { tail -5 gpurun_out/i.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/i.json').read().strip().splitlines()[-1]); d['args']='$a'; print(json.dumps(d))" >> gpurun_out/i.jsonl
  python3 -c "import json; d=json.loads(open('gpurun_out/i.json').read().strip().splitlines()[-1]); print(round(d['value']/1e6,2), 'M slices/s', d['calls_ms'], d['verify'])"
done
for a in "--k 64 --m 64 --erase 32 --lose-coding 8" "--k 64 --m 64 --erase 32 --lose-coding 16 --random-patterns"; do
  timeout -k 10 240 python bench.py $a --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/i.json 2> gpurun_out/i.err
  rc=$?; echo "bench '$a' exit $rc"; [ $rc = 0 ] || { tail -5 gpurun_out/i.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/i.json').read().strip().splitlines()[-1]); d['args']='$a'; print(json.dumps(d))" >> gpurun_out/i.jsonl
  python3 -c "import json; d=json.loads(open('gpurun_out/i.json').read().strip().splitlines()[-1]); k=d['kernels']; print('enc', round(k['encode']['achieved_GBps']), 'dec', round(k['reconstruct']['achieved_GBps']), d['verify'])"
done
rm -rf gpurun_out/kt_co
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_co -o kt --output-format csv -- \
  python3 bench_coder.py --coding-only --random-patterns --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2> gpurun_out/kt_co.err
echo "kt exit $?"
find gpurun_out/kt_co -name "*kernel_stats.csv" -exec head -8 {} \;
exit 0
