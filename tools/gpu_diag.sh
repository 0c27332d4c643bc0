#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools/ab_xform.py --variants 0 --rounds 3 > gpurun_out/diag_base.json 2>&1; rc=$?; echo "base $rc"; cat gpurun_out/diag_base.json | tail -12
case $rc in 0|1) ;; *) exit $rc;; esac
AG_RS_LIB_NAME=libalpenglow_rs_diag1role.so timeout -k 10 200 python tools/ab_xform.py --variants 0 --rounds 3 --no-check > gpurun_out/diag_1role.json 2>&1; rc=$?; echo "1role $rc"; tail -12 gpurun_out/diag_1role.json
case $rc in 0|1) ;; *) exit $rc;; esac
OUT=gpurun_out/pmc2; mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD -d $OUT/p1 -o pmc --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-verify > $OUT/p1.log 2>&1
echo "pmc $?"
