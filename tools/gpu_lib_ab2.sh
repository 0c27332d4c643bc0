#!/bin/bash
# GPU parity tests against each library in LIBS, then in-process transform A/B
# (tools/ab_xform.py, variants AB_VARIANTS) per library.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ab2.txt
for lib in ${LIBS:-libalpenglow_rs.so}; do
  if [ "${SKIP_TESTS:-0}" != 1 ]; then
    AG_RS_LIB_NAME=$lib timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
      --timeout-method thread > gpurun_out/pytest_$lib.log 2>&1
    rc=$?; echo "$lib pytest exit $rc: $(tail -1 gpurun_out/pytest_$lib.log)" | tee -a gpurun_out/ab2.txt
    [ $rc = 0 ] || { tail -30 gpurun_out/pytest_$lib.log; exit $rc; }
  fi
  AG_RS_LIB_NAME=$lib timeout -k 10 240 python tools/ab_xform.py --variants ${AB_VARIANTS:-0} --rounds ${AB_ROUNDS:-4} \
    ${AB_ARGS:-} > gpurun_out/ab_$lib.json 2> gpurun_out/ab_$lib.err
  rc=$?
  [ $rc = 0 ] || { echo "$lib ab exit $rc"; tail -5 gpurun_out/ab_$lib.err; exit $rc; }
  python3 -c "
import json; d = json.load(open('gpurun_out/ab_$lib.json'))
for v, r in d.items(): print('$lib', 'variant', v, 'enc %.4f ms %d GB/s  dec %.4f ms %d GB/s' % (r['enc_ms'], r['enc_GBps'], r['dec_ms'], r['dec_GBps']))
" | tee -a gpurun_out/ab2.txt
done
