#!/bin/bash
# Round 3 session AB: LDS-staged tail unpack -- tail/unaligned parity first, full GPU suite, A/B tail points.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "tail or unaligned or coder" > gpurun_out/pytest_ab_tail.log 2>&1
rc=$?; echo "pytest tail exit $rc"; tail -2 gpurun_out/pytest_ab_tail.log; [ $rc = 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu exit $rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || exit $rc
OUT=gpurun_out/ab.jsonl
: > $OUT
run() {
  label=$1; shift
  timeout -k 10 300 python bench.py --steps 10 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/sw.json 2> gpurun_out/sw.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "$label exit $rc"; tail -3 gpurun_out/sw.err; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1]); d['label']='$label'; print(json.dumps(d))" >> $OUT
  python3 -c "import json; d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$label', round(d['value'],1), 'GiB/s', {n: round(v['achieved_GBps']/1000,2) for n,v in k.items()}, 'TB/s', d['verify'])"
}
for v in 0 1 0 1; do
  export AG_RS_TAIL_PIECES=$v
  run tail_32x32_S1000_pieces$v --block-bytes 32000 --nblocks 131072
  run tail_32x32_S1022_pieces$v --block-bytes 32704 --nblocks 131072
  run tail_16x4_S1000_pieces$v --k 16 --m 4 --block-bytes 16000 --nblocks 262144
  run tail_32x32_S62_pieces$v --block-bytes 1984 --nblocks 1048576
done
exit 0
