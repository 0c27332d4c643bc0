#!/bin/bash
# Round 3 session B: full GPU parity suite, the follower's random-arrival deshred
# (bench_coder.py --random-patterns, decode_x16<true> with Horner products) under a kernel
# trace, the tail sweep again, and the NT load/store A/B of the headline kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_dx16b -o kt --output-format csv -- \
  python3 bench_coder.py --random-patterns --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/dx16b_bench.json 2> gpurun_out/dx16b.err
rc=$?; echo "coder random exit $rc"; [ $rc = 0 ] || exit $rc
python3 -c "import json; d=json.load(open('gpurun_out/dx16b_bench.json')); print('random slices/s', round(d['value']/1e6,2), 'M', d['calls_ms'])"
find gpurun_out/kt_dx16b -name "*kernel_stats.csv" -exec head -8 {} \;
bash tools/gpu_r03_tail.sh > /dev/null 2>&1; rc=$?; echo "tail exit $rc"; [ $rc = 0 ] || exit $rc
python3 -c "
import json
for l in open('gpurun_out/sweep_tail_r03.jsonl'):
    d=json.loads(l); k=d['kernels']; print(d['label'], round(d['value'],1), {n: round(v['achieved_GBps']/1000,2) for n,v in k.items()})"
LIBS="libalpenglow_rs.so libntl.so libntls.so libnts.so" LIBAB_CFGS="32:32:0" bash tools/gpu_libab.sh > /dev/null 2>&1
rc=$?; echo "libab exit $rc"; cat gpurun_out/libab.txt
exit 0
