#!/bin/bash
# Round-end evidence in one GPU session: parity tests, smoke, headline bench (JSON line),
# rocprofv3 kernel-trace stats of the same bench, PMC traffic passes (FETCH_SIZE and
# WRITE_SIZE in separate runs) summarised into gpurun_out/pmc_summary.json and
# gpurun_out/pmc_traffic.json.  Every GPU step has its own limit; a fatal exit ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 0|1) return 0 ;; *) echo "FATAL step exit $1"; exit "$1" ;; esac; }
BENCH_ARGS="--steps 20 --warmup 5" SKIP_PROF=1 bash tools/gpu_check.sh; rc=$?; fatal $rc; [ $rc = 0 ] || exit $rc
# the driver's command under the kernel trace (its settle steps are traced too)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o kt --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-verify > $OUT/prof_bench.json 2> $OUT/prof.err
rc=$?; echo "rocprof kernel-trace exit $rc"; fatal $rc
rm -rf $OUT/pmc
PMC_PASSES="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU;SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
  bash tools/gpu_pmc.sh; rc=$?; fatal $rc
python3 tools/pmc_summary.py --shape 4096,32,32,32768 --out $OUT/pmc_traffic.json > $OUT/pmc_summary.json
echo "pmc summary exit $?"
timeout -k 10 120 python3 tools/bench_latency.py > $OUT/latency.json 2> $OUT/latency.err
rc=$?; echo "latency exit $rc"; cat $OUT/latency.json; fatal $rc
exit 0
