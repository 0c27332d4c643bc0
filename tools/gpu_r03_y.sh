#!/bin/bash
# Round 3 session Y: decode_h8 derivative handed over by epoch flags (AG_H8_PAIRDER=1, default)
# vs workgroup barriers (lib_bar.so): full GPU suite, repeated coder batches (every slice
# verified), A/B on the follower's and CodingOnly's random arrival.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu exit $rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || exit $rc
: > gpurun_out/y.jsonl
for lib in libalpenglow_rs.so lib_bar.so libalpenglow_rs.so lib_bar.so libalpenglow_rs.so; do
  for a in "--random-patterns" "--coding-only --random-patterns"; do
    AG_RS_LIB_NAME=$lib timeout -k 10 300 python3 bench_coder.py $a --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/y.json 2> gpurun_out/y.err
    rc=$?; echo "bench_coder $lib '$a' exit $rc"; [ $rc = 0 ] || { tail -5 gpurun_out/y.err; exit $rc; }
    python3 -c "import json; d=json.loads(open('gpurun_out/y.json').read().strip().splitlines()[-1]); d['args']='$lib $a'; print(json.dumps(d))" >> gpurun_out/y.jsonl
    python3 -c "import json; d=json.loads(open('gpurun_out/y.json').read().strip().splitlines()[-1]); print(round(d['value']/1e6,2), 'M slices/s', d['calls_ms'], d['verify'])"
  done
done
rm -rf gpurun_out/kt_y
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_y -o kt --output-format csv -- \
  python3 bench_coder.py --random-patterns --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2> gpurun_out/kt_y.err
echo "kt exit $?"
find gpurun_out/kt_y -name "*kernel_stats.csv" -exec head -3 {} \; | cut -c1-160
exit 0
