#!/bin/bash
# Geometry sweep (BASELINE config C4): bench.py per k:m and block size, one JSON line each
# into gpurun_out/sweep.jsonl.  SWEEP="k:m:block_bytes:nblocks ..." overrides the list.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/sweep.jsonl
SWEEP=${SWEEP:-"32:32:1048576:4096 64:64:1048576:4096 16:4:1048576:4096"}
for cfg in $SWEEP; do
  IFS=: read -r k m bb nb <<< "$cfg"
  timeout -k 10 ${SWEEP_TIMEOUT:-240} python bench.py --k $k --m $m --block-bytes $bb --nblocks $nb \
    --steps ${SWEEP_STEPS:-10} --warmup ${SWEEP_WARMUP:-30} --no-cpu-baseline ${SWEEP_ARGS:-} >> gpurun_out/sweep.jsonl 2> gpurun_out/sweep_${k}_${m}_${bb}.err
  rc=$?
  echo "sweep $cfg exit $rc"
  case $rc in 0) ;; *) tail -5 gpurun_out/sweep_${k}_${m}_${bb}.err; exit $rc ;; esac
done
exit 0
