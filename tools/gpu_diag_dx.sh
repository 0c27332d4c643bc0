#!/bin/bash
# decode_x time attribution: the same decode bench against diagnostic library builds
# (libdiag<v>.so, built with -DAG_DX_DIAG=<v>; wrong output, timing only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/diag_dx.txt
for lib in libalpenglow_rs.so ${DIAG_LIBS:-libdiag1.so libdiag3.so libdiag4.so}; do
  for cfg in ${DIAG_CFGS:-"16:4:0" "32:32:4"}; do
    IFS=: read -r k m lc <<< "$cfg"
    AG_RS_LIB_NAME=$lib timeout -k 10 180 python bench.py --k $k --m $m --lose-coding $lc --only decode \
      --steps 5 --warmup 2 --no-cpu-baseline --no-verify > gpurun_out/dx.json 2> gpurun_out/dx.err
    rc=$?
    [ $rc = 0 ] || { echo "$lib $cfg exit $rc"; tail -3 gpurun_out/dx.err; exit $rc; }
    python3 -c "import json;d=json.load(open('gpurun_out/dx.json'));print('$lib', '$cfg', round(d['kernels']['reconstruct']['ms'],3), 'ms', round(d['kernels']['reconstruct']['achieved_GBps']), 'GB/s')" >> gpurun_out/diag_dx.txt
  done
done
cat gpurun_out/diag_dx.txt
