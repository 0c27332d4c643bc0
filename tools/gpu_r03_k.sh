#!/bin/bash
# Round 3 session K: xform_h8 parity + A/B vs xform16 (64:64), decode_syn with the recovery
# shards streamed first (16:4), full GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu exit $rc"; tail -5 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || exit $rc
: > gpurun_out/ab_k.txt
for blk in 1048576 65536 4194304; do
  nb=$(( 4294967296 / blk )); [ $nb -gt 65536 ] && nb=65536
  timeout -k 10 300 python tools/ab_xform.py --k 64 --m 64 --variants 10,9 --rounds 5 --nblocks $nb --shard $((blk / 64)) > gpurun_out/ab_k.json 2> gpurun_out/ab_k.err
  rc=$?; echo "ab 64:64 block $blk exit $rc"; [ $rc = 0 ] || { tail -5 gpurun_out/ab_k.err; exit $rc; }
  echo "64:64 block $blk nblocks $nb" >> gpurun_out/ab_k.txt; cat gpurun_out/ab_k.json >> gpurun_out/ab_k.txt
done
cat gpurun_out/ab_k.txt
SWEEP="16:4:1048576:4096 16:4:65536:65536 16:4:4194304:1024" SWEEP_STEPS=10 SWEEP_WARMUP=10 bash tools/gpu_sweep.sh || exit 1
python3 -c "
import json
for l in open('gpurun_out/sweep.jsonl'):
    d=json.loads(l); k=d['kernels']; c=d['config']
    print(c['data_shreds'], c['coding_shreds'], c['block_bytes'], 'enc', round(k['encode']['achieved_GBps']), 'dec', round(k['reconstruct']['achieved_GBps']), 'step', round(d['step_roofline_frac'],3))
"
exit 0
