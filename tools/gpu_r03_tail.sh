#!/bin/bash
# Tail chunks in place (round 3): parity tests for tails and unaligned buffers, then the tail
# sweep points (S mod 64 != 0) into gpurun_out/sweep_tail_r03.jsonl.  Every GPU step has its
# own limit; a fatal exit ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/sweep_tail_r03.jsonl
: > $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -p no:cacheprovider --timeout 120 \
  --timeout-method thread -k "tail or unaligned or coder or golden" > gpurun_out/pytest_tail.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_tail.log; [ $rc = 0 ] || exit $rc
run() {
  label=$1; shift
  timeout -k 10 300 python bench.py --steps 10 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/sw.json 2> gpurun_out/sw.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "$label exit $rc"; tail -3 gpurun_out/sw.err; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1]); d['label']='$label'; print(json.dumps(d))" >> $OUT
  python3 -c "import json; d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$label', round(d['value'],1), 'GiB/s', {n: round(v['achieved_GBps']/1000,2) for n,v in k.items()}, 'TB/s')"
}
run tail_32x32_S1000 --block-bytes 32000 --nblocks 131072
run tail_32x32_S1022 --block-bytes 32704 --nblocks 131072
run tail_16x4_S1000 --k 16 --m 4 --block-bytes 16000 --nblocks 262144
run tail_32x32_S1000_random --block-bytes 32000 --nblocks 131072 --random-patterns --lose-coding 4
run tail_32x32_S62 --block-bytes 1984 --nblocks 1048576
exit 0
