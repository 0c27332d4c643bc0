#!/bin/bash
# Round 3 session J: xform_h8 (64-point transform on 32-column tiles) parity + A/B vs xform16.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "variants or 64_point or lowrate" > gpurun_out/pytest_j.log 2>&1
rc=$?; echo "pytest j exit $rc"; tail -5 gpurun_out/pytest_j.log; [ $rc = 0 ] || exit $rc
: > gpurun_out/ab_j.txt
for blk in 1048576 65536 4194304; do
  nb=$(( 4294967296 / blk )); [ $nb -gt 65536 ] && nb=65536
  timeout -k 10 300 python tools/ab_xform.py --k 64 --m 64 --variants 10,9 --rounds 5 --nblocks $nb --shard $((blk / 64)) > gpurun_out/ab_j.json 2> gpurun_out/ab_j.err
  rc=$?; echo "ab 64:64 block $blk exit $rc"; [ $rc = 0 ] || { tail -5 gpurun_out/ab_j.err; exit $rc; }
  echo "64:64 block $blk nblocks $nb" >> gpurun_out/ab_j.txt; cat gpurun_out/ab_j.json >> gpurun_out/ab_j.txt
done
cat gpurun_out/ab_j.txt
exit 0
