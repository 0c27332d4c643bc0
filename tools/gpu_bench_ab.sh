#!/bin/bash
# Whole-step A/B: bench.py under transform variants (AG_XFORM_VARIANT), interleaved, in
# separate processes.  BENCH_VARIANTS = space-separated variants (0 = default); BENCH_LIBS =
# space-separated library builds under alpenglow_amd/_lib (default: the shipped one).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/bench_ab.txt
for i in 1 2; do
  for lib in ${BENCH_LIBS:-libalpenglow_rs.so}; do
  for v in ${BENCH_VARIANTS:-0 3}; do
    AG_RS_LIB_NAME=$lib AG_XFORM_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bab.json 2> gpurun_out/bab.err
    rc=$?; [ $rc = 0 ] || { echo "bench variant $v exit $rc"; tail -3 gpurun_out/bab.err; exit $rc; }
    python -c "
import json; d=json.load(open('gpurun_out/bab.json'))
print('$lib variant $v run $i', round(d['value'],2), 'GiB/s', {k: round(r['ms'],4) for k, r in d['kernels'].items()}, 'frac', round(d['roofline']['frac'],4))" | tee -a gpurun_out/bench_ab.txt
  done
  done
done
