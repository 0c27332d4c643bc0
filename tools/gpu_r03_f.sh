#!/bin/bash
# Round 3 session F: decode_h8 (per-lane W = 64 on 32-column tiles, two workgroups per CU)
# parity first, then the coder benches with it and with decode_x16 (AG_RS_DX_H8=0), and a
# kernel trace.  Every GPU step time-limited; a failing step ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "per_lane_window64 or per_slice_random or coder_deshred or tail_chunk or lowrate" > gpurun_out/pytest_h8.log 2>&1
rc=$?; echo "pytest h8 exit $rc"; tail -15 gpurun_out/pytest_h8.log; [ $rc = 0 ] || exit $rc
: > gpurun_out/f.jsonl
for env in "AG_RS_DX_H8=1" "AG_RS_DX_H8=0"; do
  for a in "--random-patterns" "--coding-only --random-patterns"; do
    env $env timeout -k 10 300 python3 bench_coder.py $a --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/f.json 2> gpurun_out/f.err
    rc=$?; echo "bench_coder $env '$a' exit $rc"; [ $rc = 0 ] || { tail -5 gpurun_out/f.err; exit $rc; }
    python3 -c "import json; d=json.loads(open('gpurun_out/f.json').read().strip().splitlines()[-1]); d['args']='$env $a'; print(json.dumps(d))" >> gpurun_out/f.jsonl
    python3 -c "import json; d=json.loads(open('gpurun_out/f.json').read().strip().splitlines()[-1]); print(round(d['value']/1e6,2), 'M slices/s', d['calls_ms'], d['verify'])"
  done
done
rm -rf gpurun_out/kt_h8
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_h8 -o kt --output-format csv -- \
  python3 bench_coder.py --random-patterns --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2> gpurun_out/kt_h8.err
echo "kt exit $?"
find gpurun_out/kt_h8 -name "*kernel_stats.csv" -exec head -12 {} \;
exit 0
