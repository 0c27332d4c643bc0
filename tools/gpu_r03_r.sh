#!/bin/bash
# Round 3 session R: xform_h8 with store predicates packed before the stores (stress + full
# GPU suite), decode_h8 lane-linear A/B (AG_RS_H8_LL=0/1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "--n 64 --S 2048" "--n 33 --S 1024" "--n 9 --S 1024"; do
  timeout -k 10 240 python3 tools/stress_xform64.py --variants 9,10 --iters 60 $cfg > gpurun_out/r.txt 2>&1
  rc=$?; echo "stress $cfg exit $rc"; grep -A2 "iter" gpurun_out/r.txt | head -6; tail -n 1 gpurun_out/r.txt; [ $rc = 0 ] || exit $rc
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu exit $rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || exit $rc
: > gpurun_out/r.jsonl
for ll in 0 1 0 1; do
  for a in "--random-patterns" "--coding-only --random-patterns"; do
    AG_RS_H8_LL=$ll timeout -k 10 300 python3 bench_coder.py $a --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r.json 2> gpurun_out/r.err
    rc=$?; echo "bench_coder LL=$ll '$a' exit $rc"; [ $rc = 0 ] || { tail -5 gpurun_out/r.err; exit $rc; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r.json').read().strip().splitlines()[-1]); d['args']='AG_RS_H8_LL=$ll $a'; print(json.dumps(d))" >> gpurun_out/r.jsonl
    python3 -c "import json; d=json.loads(open('gpurun_out/r.json').read().strip().splitlines()[-1]); print(round(d['value']/1e6,2), 'M slices/s', d['calls_ms'], d['verify'])"
  done
done
exit 0
