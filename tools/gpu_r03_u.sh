#!/bin/bash
# Round 3 session U: the reference bench's coder shape (deshred from the 32 coding shreds, 1 KiB
# shreds) with and without non-temporal shard accesses (lib_nont.so), kernel traces of both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "repeated or variants" > gpurun_out/pytest_u.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 gpurun_out/pytest_u.log; [ $rc = 0 ] || exit $rc
for lib in libalpenglow_rs.so lib_nont.so libalpenglow_rs.so lib_nont.so; do
  AG_RS_LIB_NAME=$lib timeout -k 10 300 python3 bench_coder.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/u.json 2> gpurun_out/u.err
  rc=$?; echo "$lib exit $rc"; [ $rc = 0 ] || { tail -5 gpurun_out/u.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/u.json').read().strip().splitlines()[-1]); print(round(d['value']/1e6,2), 'M slices/s', d['calls_ms'])"
done
for lib in libalpenglow_rs.so lib_nont.so; do
  rm -rf gpurun_out/kt_u_$lib
  AG_RS_LIB_NAME=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_u_$lib -o kt --output-format csv -- \
    python3 bench_coder.py --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2> gpurun_out/kt_u.err
  echo "kt $lib exit $?"
  find gpurun_out/kt_u_$lib -name "*kernel_stats.csv" -exec head -6 {} \; | cut -c1-160
done
exit 0
