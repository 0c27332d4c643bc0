#!/bin/bash
# Round 3 session V: uniform-pattern coder deshred fast path; decode_x16 one-pattern tiles
# with scalar-branch (uniform) products vs decode_c for lost coding shreds; W = 128 points.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu exit $rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || exit $rc
for a in "" "--random-patterns" ""; do
  timeout -k 10 300 python3 bench_coder.py $a --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/v.json 2> gpurun_out/v.err
  rc=$?; echo "bench_coder '$a' exit $rc"; [ $rc = 0 ] || { tail -5 gpurun_out/v.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/v.json').read().strip().splitlines()[-1]); print(round(d['value']/1e6,2), 'M slices/s', d['calls_ms'])"
done
: > gpurun_out/v.jsonl
run() {
  label=$1; shift
  timeout -k 10 300 "$@" --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/sw.json 2> gpurun_out/sw.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "$label exit $rc"; tail -3 gpurun_out/sw.err; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1]); d['label']='$label'; print(json.dumps(d))" >> gpurun_out/v.jsonl
  python3 -c "import json; d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$label', {n: round(v['achieved_GBps']/1000,2) for n,v in k.items()}, 'TB/s', d['verify'])"
}
for lc in 4 8 16; do
  run "decode_c_lose${lc}_random" python bench.py --lose-coding $lc --random-patterns
  AG_RS_NO_CORR=1 run "x16u_lose${lc}_random" python bench.py --lose-coding $lc --random-patterns
done
run "decode_c_lose8" python bench.py --lose-coding 8
AG_RS_NO_CORR=1 run "x16u_lose8" python bench.py --lose-coding 8
run w128_64x64_lose8 python bench.py --k 64 --m 64 --erase 32 --lose-coding 8
run w128_64x64_lose16_random python bench.py --k 64 --m 64 --erase 32 --lose-coding 16 --random-patterns
exit 0
