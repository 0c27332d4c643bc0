#!/bin/bash
# decode_c bring-up: parity tests for the decoders, then decode-only bench points.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/dc
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "${TESTK:-correction or general_decode or decode_per_block or deshred or c4 or per_slice}" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -5 $OUT/pytest.log
case $rc in 0) ;; *) exit $rc;; esac
i=0
IFS=';' read -ra CFGS <<< "${CONFIGS:---only decode --lose-coding 4;--only decode --random-patterns --lose-coding 8;--only decode --lose-coding 16}"
for cfg in "${CFGS[@]}"; do
  i=$((i+1))
  timeout -k 10 240 python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline $cfg > $OUT/b$i.json 2> $OUT/b$i.err
  rc=$?; echo "bench $i ($cfg) exit $rc"
  python3 -c "import json,sys; d=json.load(open('$OUT/b$i.json')); k=d['kernels']; print({n: round(v['achieved_GBps']) for n,v in k.items()}, d['verify'])" || true
  case $rc in 0) ;; *) exit $rc;; esac
done
exit 0
