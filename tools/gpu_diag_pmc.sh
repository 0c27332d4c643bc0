#!/bin/bash
# Diagnostic PMC passes over several bench configurations (one rocprofv3 run per pass and
# configuration; counters only with --kernel-trace).  CONFIGS: ';'-separated bench args.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/diag
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${PMC_LIST:-0}" = 1 ]; then
  timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1; echo "list exit $?"
fi
IFS=';' read -ra CFGS <<< "${CONFIGS}"
IFS=';' read -ra PASSES <<< "${PMC_PASSES}"
c=0
for cfg in "${CFGS[@]}"; do
  c=$((c+1)); i=0
  for p in "${PASSES[@]}"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $p -d $OUT/c${c}p$i -o pmc --output-format csv -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-verify --no-settle $cfg > $OUT/c${c}p$i.log 2>&1
    rc=$?; echo "cfg $c ($cfg) pass $i ($p) exit $rc"
    case $rc in 0|1) ;; *) echo "stopping"; exit $rc;; esac
  done
done
exit 0
