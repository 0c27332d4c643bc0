#!/bin/bash
# Round 3 session N: lane-linear decode_h8 (libll.so) parity + coder A/B, then the round
# evidence and the C4 sweep (session M).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AG_RS_LIB_NAME=libll.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_ll.log 2>&1
rc=$?; echo "pytest ll exit $rc"; tail -3 gpurun_out/pytest_ll.log; [ $rc = 0 ] || exit $rc
: > gpurun_out/n.jsonl
for lib in libalpenglow_rs.so libll.so libalpenglow_rs.so libll.so; do
  for a in "--random-patterns" "--coding-only --random-patterns"; do
    AG_RS_LIB_NAME=$lib timeout -k 10 300 python3 bench_coder.py $a --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/n.json 2> gpurun_out/n.err
    rc=$?; echo "bench_coder $lib '$a' exit $rc"; [ $rc = 0 ] || { tail -5 gpurun_out/n.err; exit $rc; }
    python3 -c "import json; d=json.loads(open('gpurun_out/n.json').read().strip().splitlines()[-1]); d['args']='$lib $a'; print(json.dumps(d))" >> gpurun_out/n.jsonl
    python3 -c "import json; d=json.loads(open('gpurun_out/n.json').read().strip().splitlines()[-1]); print(round(d['value']/1e6,2), 'M slices/s', d['calls_ms'], d['verify'])"
  done
done
rm -rf gpurun_out/kt_ll
AG_RS_LIB_NAME=libll.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_ll -o kt --output-format csv -- \
  python3 bench_coder.py --random-patterns --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2> gpurun_out/kt_ll.err
echo "kt exit $?"
find gpurun_out/kt_ll -name "*kernel_stats.csv" -exec head -4 {} \;
bash tools/gpu_r03_m.sh
