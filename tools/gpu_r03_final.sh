#!/bin/bash
# Round 3 closing check: smoke, the driver's bench command, default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_final.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/smoke_final.log | tail -3; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err
rc=$?; echo "bench exit $rc"; [ $rc = 0 ] || { tail -5 gpurun_out/bench_final.err; exit $rc; }
tail -1 gpurun_out/bench_final.json | cut -c1-400
exit 0
