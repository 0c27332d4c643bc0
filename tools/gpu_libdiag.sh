#!/bin/bash
# Kernel ms of diagnostic library builds (wrong output allowed) next to the default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/libdiag.txt
for lib in ${LIBS:-libalpenglow_rs.so}; do
  AG_RS_LIB_NAME=$lib timeout -k 10 180 python bench.py ${DIAG_ARGS:-} --steps 5 --warmup 2 --no-cpu-baseline --no-verify \
    > gpurun_out/ld.json 2> gpurun_out/ld.err
  rc=$?
  [ $rc = 0 ] || { echo "$lib exit $rc"; tail -3 gpurun_out/ld.err; exit $rc; }
  python3 -c "import json;d=json.load(open('gpurun_out/ld.json'));k=d['kernels'];print('$lib enc', round(k['encode']['ms'],4), round(k['encode']['achieved_GBps']), 'dec', round(k['reconstruct']['ms'],4), round(k['reconstruct']['achieved_GBps']))" >> gpurun_out/libdiag.txt
done
cat gpurun_out/libdiag.txt
