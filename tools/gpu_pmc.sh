#!/bin/bash
# rocprofv3 PMC passes (counters only with --kernel-trace; never with sys/hip traces).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${PMC_OUT:-gpurun_out/pmc}
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="${PMC_CMD:-python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-verify ${PMC_BENCH_ARGS:-}}"
if [ "${PMC_LIST:-0}" = 1 ]; then
  timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1; echo "list exit $?"
fi
i=0
IFS=';' read -ra PASSES <<< "${PMC_PASSES:-FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU}"
for p in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $p -d $OUT/p$i -o pmc --output-format csv -- $BENCH > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($p) exit $rc"
  case $rc in 0|1) ;; *) echo "stopping"; exit $rc;; esac
done
exit 0
