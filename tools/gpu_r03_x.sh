#!/bin/bash
# Round 3 session X: xform_h8 half-pruned FFT for 64-point reconstructs with every erasure in
# shards 0..31: stress, full GPU suite, 64:64 sweep points (variant 5 = no pruning for A/B).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python3 tools/stress_xform64.py --variants 0,9,10 --iters 30 --n 64 --S 2048 > gpurun_out/x.txt 2>&1
rc=$?; echo "stress exit $rc"; tail -n 1 gpurun_out/x.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu exit $rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || exit $rc
: > gpurun_out/x.jsonl
for blk in 1048576 65536 4194304; do
  nb=$(( 4294967296 / blk )); [ $nb -gt 65536 ] && nb=65536
  timeout -k 10 300 python tools/ab_xform.py --k 64 --m 64 --variants 0,5 --rounds 5 --nblocks $nb --shard $((blk / 64)) > gpurun_out/x.json 2> gpurun_out/x.err
  rc=$?; echo "ab 64:64 block $blk exit $rc"; [ $rc = 0 ] || { tail -5 gpurun_out/x.err; exit $rc; }
  python3 -c "
import json; d=json.load(open('gpurun_out/x.json'))
print('64:64 block $blk', {v: (round(r['enc_GBps']), round(r['dec_GBps'])) for v, r in d.items()})
" | tee -a gpurun_out/x.jsonl
done
SWEEP="64:64:65536:65536 64:64:262144:16384 64:64:1048576:4096 64:64:4194304:1024" SWEEP_STEPS=10 SWEEP_WARMUP=30 bash tools/gpu_sweep.sh || exit 1
python3 -c "
import json
for l in open('gpurun_out/sweep.jsonl'):
    d=json.loads(l); k=d['kernels']; c=d['config']
    print(c['data_shreds'], c['coding_shreds'], c['block_bytes'], 'enc', round(k['encode']['achieved_GBps']), 'dec', round(k['reconstruct']['achieved_GBps']), 'step', round(d['step_roofline_frac'],3), 'value', round(d['value']))
"
exit 0
