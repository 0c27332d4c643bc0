#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_xform.py ${AB_ARGS:-} > gpurun_out/ab.json 2> gpurun_out/ab.err
rc=$?; echo "ab exit $rc"; cat gpurun_out/ab.json; tail -3 gpurun_out/ab.err
case $rc in 0|1) ;; *) exit $rc;; esac
