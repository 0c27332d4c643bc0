#!/bin/bash
# Round 3 session C: lost-coding decoders (decode_c vs decode_x16 with Horner products,
# AG_RS_NO_CORR=1) over random per-block patterns, W = 128 windows (64:64 lost coding,
# CodingOnly random arrival), PMC of the per-lane decode.  One JSON line per point into
# gpurun_out/sweep_c.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/sweep_c.jsonl
: > $OUT
run() {
  label=$1; shift
  timeout -k 10 300 "$@" > gpurun_out/sc.json 2> gpurun_out/sc.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "$label exit $rc"; tail -3 gpurun_out/sc.err; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/sc.json').read().strip().splitlines()[-1]); d['label']='$label'; print(json.dumps(d))" >> $OUT
  python3 -c "
import json; d=json.loads(open('gpurun_out/sc.json').read().strip().splitlines()[-1])
k=d.get('kernels'); print('$label', round(d['value'],2), {n: round(v['achieved_GBps']/1000,2) for n,v in k.items()} if k else d.get('calls_ms'))"
}
B="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline"
for lc in 4 8 16; do
  run corr_lc$lc $B --random-patterns --lose-coding $lc --only decode
  AG_RS_NO_CORR=1 run x16_lc$lc $B --random-patterns --lose-coding $lc --only decode
done
run w128_64x64_lc8 $B --k 64 --m 64 --lose-coding 8 --only decode
run w128_64x64_lc16_random $B --k 64 --m 64 --lose-coding 16 --random-patterns --only decode
run coder_coding_only_random python3 bench_coder.py --coding-only --random-patterns --steps 5 --warmup 2 --no-cpu-baseline
run coder_random python3 bench_coder.py --random-patterns --steps 5 --warmup 2 --no-cpu-baseline
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_c -o kt --output-format csv -- \
  python3 bench_coder.py --coding-only --random-patterns --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/ktc.err
echo "kt exit $?"
find gpurun_out/kt_c -name "*kernel_stats.csv" -exec head -8 {} \;
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
PMC_OUT=gpurun_out/pmc_dx16h PMC_CMD="python3 bench_coder.py --random-patterns --steps 3 --warmup 1 --slices 65536 --no-cpu-baseline" \
  PMC_PASSES="$P1;$P2;FETCH_SIZE;WRITE_SIZE" bash tools/gpu_pmc.sh; rc=$?; [ $rc = 0 ] || exit $rc
python3 tools/pmc_summary.py --dir gpurun_out/pmc_dx16h > gpurun_out/pmc_dx16h_summary.json; echo "summary $?"
exit 0
