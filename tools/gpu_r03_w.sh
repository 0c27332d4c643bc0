#!/bin/bash
# Round 3 session W: decode_h8 UNI (one pattern per 32-column tile, lane-linear I/O, per-half
# uniform products) -- full GPU suite, then lost-coding decodes: decode_c vs h8 UNI
# (AG_RS_NO_CORR=1) vs decode_x16 (AG_RS_NO_CORR=1 AG_RS_H8U=0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AG_RS_H8U=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu exit $rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || exit $rc
: > gpurun_out/w.jsonl
run() {
  label=$1; shift
  timeout -k 10 300 "$@" --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/sw.json 2> gpurun_out/sw.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "$label exit $rc"; tail -3 gpurun_out/sw.err; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1]); d['label']='$label'; print(json.dumps(d))" >> gpurun_out/w.jsonl
  python3 -c "import json; d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$label', {n: round(v['achieved_GBps']/1000,2) for n,v in k.items()}, 'TB/s', d['verify'])"
}
for lc in 4 8 12 16; do
  run "decode_c_lose${lc}_random" python bench.py --lose-coding $lc --random-patterns
  AG_RS_H8U=1 AG_RS_NO_CORR=1 run "h8u_lose${lc}_random" python bench.py --lose-coding $lc --random-patterns
done
AG_RS_NO_CORR=1 run "x16_lose16_random" python bench.py --lose-coding 16 --random-patterns
run "decode_c_lose8" python bench.py --lose-coding 8
AG_RS_H8U=1 AG_RS_NO_CORR=1 run "h8u_lose8" python bench.py --lose-coding 8
run "decode_c_lose16" python bench.py --lose-coding 16
AG_RS_H8U=1 AG_RS_NO_CORR=1 run "h8u_lose16" python bench.py --lose-coding 16
run "lowrate_co_mixed" python bench.py --k 32 --m 64 --erase 16 --lose-coding 40 --random-patterns
exit 0
