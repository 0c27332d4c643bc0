#!/bin/bash
# Round 3 session M: round evidence (tests, smoke, headline bench, kernel trace, PMC traffic,
# call latency) then the full C4 geometry sweep with the round-3 kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_round_profile.sh || exit $?
SWEEP="32:32:65536:65536 32:32:262144:16384 32:32:1048576:4096 32:32:4194304:1024 64:64:65536:65536 64:64:262144:16384 64:64:1048576:4096 64:64:4194304:1024 16:4:65536:65536 16:4:262144:16384 16:4:1048576:4096 16:4:4194304:1024" \
  SWEEP_STEPS=10 SWEEP_WARMUP=30 bash tools/gpu_sweep.sh || exit 1
python3 -c "
import json
for l in open('gpurun_out/sweep.jsonl'):
    d=json.loads(l); k=d['kernels']; c=d['config']
    print(c['data_shreds'], c['coding_shreds'], c['block_bytes'], 'enc', round(k['encode']['achieved_GBps']), 'dec', round(k['reconstruct']['achieved_GBps']), 'step', round(d['step_roofline_frac'],3), 'value', round(d['value']))
"
exit 0
