#!/bin/bash
# Round 3 session L: PMC passes (counters only with --kernel-trace) on the kernels below the
# bar: xform16 (64:64 encode / reconstruct), decode_h8 (per-lane W = 64, coder random
# arrival), decode_c (32:32 with 8 lost coding shards, random pattern per block).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
run() {  # name, command
  for i in 1 2; do
    eval "PP=\$P$i"
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $PP -d gpurun_out/pmc_$1/p$i -o pmc --output-format csv -- $2 > gpurun_out/pmc_$1_p$i.log 2>&1
    rc=$?; echo "$1 pass $i exit $rc"
    case $rc in 0|1) ;; *) echo "stopping"; exit $rc;; esac
  done
  python3 tools/pmc_summary.py --dir gpurun_out/pmc_$1 > gpurun_out/pmc_$1.json
}
run x16 "python3 bench.py --k 64 --m 64 --steps 3 --warmup 1 --no-cpu-baseline --no-verify"
run h8 "python3 bench_coder.py --random-patterns --steps 2 --warmup 1 --no-cpu-baseline"
run dc "python3 bench.py --lose-coding 8 --random-patterns --steps 3 --warmup 1 --no-cpu-baseline --no-verify"
for f in x16 h8 dc; do
  python3 - $f <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/pmc_{sys.argv[1]}.json"))
for k, v in d.items():
    if any(s in k for s in ("xform16", "decode_h8", "decode_c", "reconstruct", "encode")):
        wc = v.get("SQ_WAVE_CYCLES", 0) or 1
        print(sys.argv[1], k[:50], "waves", v.get("SQ_WAVES"), "wait_any %.2f" % (v.get("SQ_WAIT_ANY", 0) / wc),
              "wait_inst %.2f" % (v.get("SQ_WAIT_INST_ANY", 0) / wc), "active %.2f" % (v.get("SQ_ACTIVE_INST_ANY", 0) / wc),
              "valu/wave %.0f" % (v.get("SQ_INSTS_VALU", 0) / max(1, v.get("SQ_WAVES", 1))),
              "lds/wave %.0f" % (v.get("SQ_INSTS_LDS", 0) / max(1, v.get("SQ_WAVES", 1))),
              "salu/wave %.0f" % (v.get("SQ_INSTS_SALU", 0) / max(1, v.get("SQ_WAVES", 1))),
              "wait_lds %.2f" % (v.get("SQ_WAIT_INST_LDS", 0) / wc), "bankc", v.get("SQ_LDS_BANK_CONFLICT"))
PY
done
exit 0
