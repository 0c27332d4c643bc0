#!/bin/bash
# Round 3 session T (round evidence with the final kernels): session M (tests, smoke, headline
# bench, kernel trace, PMC traffic, call latency, C4 sweep), then the coder and shredder
# benches, the tail and lost-coding points.  Every GPU step time-limited; a failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r03_m.sh || exit $?
: > gpurun_out/t_coder.jsonl
for a in "" "--random-patterns" "--coding-only" "--coding-only --random-patterns"; do
  timeout -k 10 300 python3 bench_coder.py $a --steps 5 --warmup 2 $( [ -z "$a" ] || echo --no-cpu-baseline ) > gpurun_out/t.json 2> gpurun_out/t.err
  rc=$?; echo "bench_coder '$a' exit $rc"; [ $rc = 0 ] || { tail -5 gpurun_out/t.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/t.json').read().strip().splitlines()[-1]); d['args']='$a'; print(json.dumps(d))" >> gpurun_out/t_coder.jsonl
  python3 -c "import json; d=json.loads(open('gpurun_out/t.json').read().strip().splitlines()[-1]); print(round(d['value']/1e6,2), 'M slices/s', d['calls_ms'], d['verify'])"
done
timeout -k 10 400 python3 bench_shredder.py > gpurun_out/t_shredder.json 2> gpurun_out/t_shredder.err
rc=$?; echo "bench_shredder exit $rc"; tail -c 600 gpurun_out/t_shredder.json; [ $rc = 0 ] || exit $rc
OUT=gpurun_out/t_points.jsonl
: > $OUT
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
run random16_full_recovery --random-patterns
run lose4 --lose-coding 4
run lose8_random --lose-coding 8 --random-patterns
run lose16_random --lose-coding 16 --random-patterns
run w128_64x64_lose8 --k 64 --m 64 --erase 32 --lose-coding 8
run w128_64x64_lose16_random --k 64 --m 64 --erase 32 --lose-coding 16 --random-patterns
run pcie_headline --pcie --pcie-blocks 4096
exit 0
