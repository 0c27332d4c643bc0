#!/bin/bash
# Round 3 session AA: kernel traces of the slow tail shapes (S = 62, random per-block S = 1000).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in "s62 --block-bytes 1984 --nblocks 1048576" "rnd --block-bytes 32000 --nblocks 131072 --random-patterns --lose-coding 4" "rnd0 --block-bytes 32000 --nblocks 131072 --random-patterns"; do
  set -- $c; label=$1; shift
  rm -rf gpurun_out/kt_$label
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_$label -o kt --output-format csv -- \
    python3 bench.py "$@" --steps 5 --warmup 2 --no-cpu-baseline --no-verify > gpurun_out/kt_$label.json 2> gpurun_out/kt_$label.err
  rc=$?; echo "$label exit $rc"; [ $rc = 0 ] || exit $rc
  tail -1 gpurun_out/kt_$label.json | cut -c1-300
  find gpurun_out/kt_$label -name "*kernel_stats.csv" -exec head -8 {} \; | cut -c1-170
done
exit 0
