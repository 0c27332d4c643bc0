#!/bin/bash
# Round 3 session D: parity suite + smoke + the driver's bench command with kernel trace and
# PMC traffic (tools/gpu_round_profile.sh), then session C's decoder sweep, then the
# s_setprio A/B of the headline reconstruct.  Every GPU step time-limited; fatal exits end it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_round_profile.sh > gpurun_out/round.log 2>&1; rc=$?; echo "round profile exit $rc"; tail -25 gpurun_out/round.log
[ $rc = 0 ] || exit $rc
bash tools/gpu_r03_c.sh > gpurun_out/c.log 2>&1; rc=$?; echo "session C exit $rc"; cat gpurun_out/c.log | grep -v "^\"" | tail -30
[ $rc = 0 ] || exit $rc
LIBS="libalpenglow_rs.so libprio.so" LIBAB_CFGS="32:32:0" bash tools/gpu_libab.sh > /dev/null 2>&1
rc=$?; echo "prio A/B exit $rc"; cat gpurun_out/libab.txt
exit 0
