#!/bin/bash
# Round 3 session AD: per-lane pattern trimming without a popcount per dropped bit -- parity, host enqueue times, random-pattern points.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu exit $rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || exit $rc
timeout -k 10 240 python tools/host_enqueue.py > gpurun_out/host_enqueue_ad.txt 2>&1
rc=$?; cat gpurun_out/host_enqueue_ad.txt | grep -v amdgpu.ids; [ $rc = 0 ] || exit $rc
OUT=gpurun_out/ad.jsonl
: > $OUT
run() {
  label=$1; shift
  timeout -k 10 300 python bench.py --steps 10 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/sw.json 2> gpurun_out/sw.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "$label exit $rc"; tail -3 gpurun_out/sw.err; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1]); d['label']='$label'; print(json.dumps(d))" >> $OUT
  python3 -c "import json; d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$label', round(d['value'],1), 'GiB/s', round(d['ms_per_step'],2), 'ms', {n: round(v['achieved_GBps']/1000,2) for n,v in k.items()}, 'TB/s', d['verify'])"
}
run tail_32x32_S1000_random_lose4 --block-bytes 32000 --nblocks 131072 --random-patterns --lose-coding 4
run x32_S1024_random_lose4 --block-bytes 32768 --nblocks 131072 --random-patterns --lose-coding 4
exit 0
