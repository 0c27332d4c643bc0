#!/bin/bash
# Same benches against two library builds (LIBS, default: the in-tree build and
# libhead.so = the previous commit), interleaved, kernel ms from bench.py's HIP events.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/libab.txt
for r in 1 2; do
  for lib in ${LIBS:-libalpenglow_rs.so libhead.so}; do
    for cfg in ${LIBAB_CFGS:-"32:32:0" "64:64:0" "16:4:0" "32:32:4"}; do
      IFS=: read -r k m lc <<< "$cfg"
      AG_RS_LIB_NAME=$lib timeout -k 10 180 python bench.py --k $k --m $m --lose-coding $lc \
        --steps 5 --warmup 2 --no-cpu-baseline --no-verify > gpurun_out/lab.json 2> gpurun_out/lab.err
      rc=$?
      [ $rc = 0 ] || { echo "$lib $cfg exit $rc"; tail -3 gpurun_out/lab.err; exit $rc; }
      python3 -c "import json;d=json.load(open('gpurun_out/lab.json'));k=d['kernels'];print('$r $lib $cfg enc', round(k['encode']['achieved_GBps']), 'dec', round(k['reconstruct']['achieved_GBps']))" >> gpurun_out/libab.txt
    done
  done
done
cat gpurun_out/libab.txt
