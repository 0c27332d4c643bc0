#!/bin/bash
# Round-3 diagnosis: PMC passes for the per-lane window decoder (decode_x16<true>, the
# follower's random-arrival deshred: bench_coder.py --random-patterns) and the headline
# reconstruct (xform8<0,32,true>: bench.py --only decode).  One rocprofv3 run per pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
PMC_OUT=gpurun_out/pmc_dx16 PMC_CMD="python3 bench_coder.py --random-patterns --steps 3 --warmup 1 --slices 65536 --no-cpu-baseline" \
  PMC_PASSES="$P1;$P2;FETCH_SIZE;WRITE_SIZE" bash tools/gpu_pmc.sh; rc=$?; [ $rc = 0 ] || exit $rc
python3 tools/pmc_summary.py --dir gpurun_out/pmc_dx16 > gpurun_out/pmc_dx16_summary.json; echo "summary $?"
PMC_OUT=gpurun_out/pmc_rec PMC_CMD="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-verify --only decode" \
  PMC_PASSES="$P1;$P2" bash tools/gpu_pmc.sh; rc=$?; [ $rc = 0 ] || exit $rc
python3 tools/pmc_summary.py --dir gpurun_out/pmc_rec > gpurun_out/pmc_rec_summary.json; echo "summary $?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_dx16 -o kt --output-format csv -- \
  python3 bench_coder.py --random-patterns --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/dx16_bench.json 2> gpurun_out/dx16_bench.err
echo "kt exit $?"
exit 0
