#!/bin/bash
# Round 3 session E: parity suite on the coder's device-pattern path, the coder benches
# (random arrival, CodingOnly random arrival) and a HIP API trace of the CodingOnly deshred
# (where its host time goes).  Every GPU step time-limited; fatal exits end it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SKIP_BENCH=1 bash tools/gpu_check.sh; rc=$?; [ $rc = 0 ] || exit $rc
: > gpurun_out/e.jsonl
for a in "--random-patterns" "--random-patterns --exact" "--coding-only --random-patterns" ""; do
  timeout -k 10 300 python3 bench_coder.py $a --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/e.json 2> gpurun_out/e.err
  rc=$?; echo "bench_coder '$a' exit $rc"; [ $rc = 0 ] || { tail -5 gpurun_out/e.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/e.json').read().strip().splitlines()[-1]); d['args']='$a'; print(json.dumps(d))" >> gpurun_out/e.jsonl
  python3 -c "import json; d=json.loads(open('gpurun_out/e.json').read().strip().splitlines()[-1]); print(round(d['value']/1e6,2), 'M slices/s', d['calls_ms'], d['verify'])"
done
rm -rf gpurun_out/ht
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats -d gpurun_out/ht -o ht --output-format csv -- \
  python3 bench_coder.py --coding-only --random-patterns --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/ht.err
echo "hip trace exit $?"
find gpurun_out/ht -name "*hip_api_stats.csv" -exec head -15 {} \;
exit 0
