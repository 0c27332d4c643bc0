#!/bin/bash
# One parametrised GPU session runner (replaces the per-session gpu_*.sh scripts).
#
#   tools/gpu_run.sh STEP [ARGS...] [+ STEP [ARGS...] ...]
#
# Steps (each GPU step has its own time limit; a fault, abort, time limit or failed step
# ends the session -- no retries, nothing further on the GPU):
#   tests [PYTEST ARGS]      pytest -m gpu (log: gpurun_out/pytest_gpu.log)
#   smoke                    __graft_entry__.smoke()
#   bench [BENCH ARGS]       bench.py (default: the driver's --steps 20 --warmup 5) -> bench.json
#   point LABEL [ARGS]       one bench.py line (10 timed steps, no CPU baseline) -> points.jsonl
#   points PRESET            a preset list of points: tail | lost | w128 | random | c4 | c4x64
#   coder [ARGS]             bench_coder.py over its four arrival shapes -> coder.jsonl
#   coder_short [ARGS]       bench_coder.py --random-patterns at four non-maximal payload lengths
#   shredder                 bench_shredder.py -> shredder.json
#   latency                  tools/bench_latency.py -> latency.json
#   kt NAME [CMD...]         rocprofv3 --kernel-trace --stats of CMD (default: the headline
#                            bench without the configs[4] stream, so every launch has the
#                            4096-block shape) into gpurun_out/kt_NAME
#   pmc NAME PASSES [CMD...] rocprofv3 --pmc, one run per ';'-separated counter pass, into
#                            gpurun_out/pmc_NAME/p<i>; then tools/pmc_summary.py
#   stress                   tools/stress_xform64.py (repeated per-block-mask reconstructs)
#   sh 'COMMAND'             any other command, under a 300 s limit
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
PY=python3

fail() { echo "STOP: $1 exit $2"; exit "$2"; }

jsonl_last() {  # $1 = json file, $2 = label, $3 = jsonl to append
  $PY - "$1" "$2" "$3" <<'EOF'
import json, sys
src, label, dst = sys.argv[1:4]
d = json.loads(open(src).read().strip().splitlines()[-1])
d["label"] = label
open(dst, "a").write(json.dumps(d) + "\n")
k = d.get("kernels") or {}
print(label, round(d["value"], 2) if isinstance(d.get("value"), (int, float)) else d.get("value"),
      d.get("unit"), {n: round(v["achieved_GBps"] / 1000, 2) for n, v in k.items() if v.get("achieved_GBps")},
      "TB/s", "verify", (d.get("verify") or {}).get("all_ranks_ok", d.get("verify")))
EOF
}

point() {
  local label=$1; shift
  timeout -k 10 300 $PY bench.py --steps 10 --warmup 5 --no-cpu-baseline "$@" > $OUT/pt.json 2> $OUT/pt.err
  local rc=$?
  [ $rc = 0 ] || { tail -5 $OUT/pt.err; fail "point $label" $rc; }
  jsonl_last $OUT/pt.json "$label" $OUT/points.jsonl
}

points() {
  case "$1" in
    tail)
      point tail_32x32_S1000 --block-bytes 32000 --nblocks 131072
      point tail_32x32_S1022 --block-bytes 32704 --nblocks 131072
      point tail_16x4_S1000 --k 16 --m 4 --block-bytes 16000 --nblocks 262144
      point tail_32x32_S1000_random_lose4 --block-bytes 32000 --nblocks 131072 --random-patterns --lose-coding 4
      point tail_32x32_S62 --block-bytes 1984 --nblocks 1048576 ;;
    lost)
      point lose4 --lose-coding 4
      point lose8_random --lose-coding 8 --random-patterns
      point lose16_random --lose-coding 16 --random-patterns ;;
    w128)
      point w128_64x64_lose8 --k 64 --m 64 --erase 32 --lose-coding 8
      point w128_64x64_lose16_random --k 64 --m 64 --erase 32 --lose-coding 16 --random-patterns ;;
    random)
      point random16_full_recovery --random-patterns ;;
    c4)
      for km in 16:4 32:32 64:64; do
        for bb in 65536 262144 1048576 4194304; do
          IFS=: read -r k m <<< "$km"
          nb=$(( (4 << 30) / bb ))
          timeout -k 10 300 $PY bench.py --k $k --m $m --block-bytes $bb --nblocks $nb --steps 10 --warmup 30 \
            --no-cpu-baseline > $OUT/pt.json 2> $OUT/pt.err
          rc=$?; [ $rc = 0 ] || { tail -5 $OUT/pt.err; fail "c4 $km $bb" $rc; }
          jsonl_last $OUT/pt.json "c4_${k}x${m}_${bb}" $OUT/points.jsonl
        done
      done ;;
    c4x64)
      for bb in 65536 262144 1048576 4194304; do
        nb=$(( (4 << 30) / bb ))
        point "c4_64x64_$bb" --k 64 --m 64 --block-bytes $bb --nblocks $nb --warmup 30
      done ;;
    *) echo "unknown preset $1"; exit 2 ;;
  esac
}

step() {
  local name=$1; shift
  case "$name" in
    tests)
      timeout -k 10 1000 $PY -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
        --timeout-method thread "$@" > $OUT/pytest_gpu.log 2>&1
      local rc=$?; echo "pytest gpu exit $rc"; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] || fail tests $rc ;;
    smoke)
      timeout -k 10 300 $PY -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
      local rc=$?; echo "smoke exit $rc"; tail -2 $OUT/smoke.log; [ $rc = 0 ] || fail smoke $rc ;;
    bench)
      [ $# -gt 0 ] || set -- --steps 20 --warmup 5
      timeout -k 10 600 $PY bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err
      local rc=$?; echo "bench exit $rc"; cat $OUT/bench.json; tail -3 $OUT/bench.err; [ $rc = 0 ] || fail bench $rc ;;
    point) point "$@" ;;
    points) points "$@" ;;
    coder)
      for a in "" "--random-patterns" "--coding-only" "--coding-only --random-patterns"; do
        timeout -k 10 300 $PY bench_coder.py $a --steps 5 --warmup 2 --no-cpu-baseline "$@" > $OUT/c.json 2> $OUT/c.err
        local rc=$?; [ $rc = 0 ] || { tail -5 $OUT/c.err; fail "coder '$a'" $rc; }
        jsonl_last $OUT/c.json "coder${a// /_}" $OUT/coder.jsonl
      done ;;
    coder_short)  # the follower's batches of non-maximal slices (whole-chunk and tail shred sizes)
      for L in 16383 4095 2047 31999; do
        timeout -k 10 300 $PY bench_coder.py --random-patterns --payload-len $L --steps 5 --warmup 2 --no-cpu-baseline "$@" \
          > $OUT/c.json 2> $OUT/c.err
        local rc=$?; [ $rc = 0 ] || { tail -5 $OUT/c.err; fail "coder_short $L" $rc; }
        jsonl_last $OUT/c.json "coder_random_L$L" $OUT/coder.jsonl
      done ;;
    shredder)
      timeout -k 10 400 $PY bench_shredder.py "$@" > $OUT/shredder.json 2> $OUT/shredder.err
      local rc=$?; echo "shredder exit $rc"; tail -c 600 $OUT/shredder.json; [ $rc = 0 ] || fail shredder $rc ;;
    latency)
      timeout -k 10 200 $PY tools/bench_latency.py "$@" > $OUT/latency.json 2> $OUT/latency.err
      local rc=$?; echo "latency exit $rc"; cat $OUT/latency.json; [ $rc = 0 ] || fail latency $rc ;;
    kt)
      local tag=$1; shift
      [ $# -gt 0 ] || set -- $PY bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-verify --strong-stream 0
      rm -rf $OUT/kt_$tag
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt_$tag -o kt --output-format csv -- "$@" \
        > $OUT/kt_$tag.log 2>&1
      local rc=$?; echo "kt $tag exit $rc"; [ $rc = 0 ] || { tail -5 $OUT/kt_$tag.log; fail "kt $tag" $rc; }
      find $OUT/kt_$tag -name "*kernel_stats.csv" -exec head -8 {} \; | cut -c1-200 ;;
    pmc)
      local tag=$1 passes=$2; shift 2
      [ $# -gt 0 ] || set -- $PY bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-verify --strong-stream 0
      rm -rf $OUT/pmc_$tag
      local i=0 p
      IFS=';' read -ra PS <<< "$passes"
      for p in "${PS[@]}"; do
        i=$((i+1))
        timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $p -d $OUT/pmc_$tag/p$i -o pmc --output-format csv -- "$@" \
          > $OUT/pmc_$tag.p$i.log 2>&1
        local rc=$?; echo "pmc $tag pass $i ($p) exit $rc"; [ $rc = 0 ] || fail "pmc $tag" $rc
      done
      $PY tools/pmc_summary.py --dir $OUT/pmc_$tag > $OUT/pmc_$tag.json; echo "pmc summary $tag exit $?" ;;
    stress)
      timeout -k 10 300 $PY tools/stress_xform64.py "$@" > $OUT/stress.log 2>&1
      local rc=$?; echo "stress exit $rc"; tail -5 $OUT/stress.log; [ $rc = 0 ] || fail stress $rc ;;
    sh)
      timeout -k 10 300 bash -c "$1"
      local rc=$?; echo "sh exit $rc"; [ $rc = 0 ] || fail sh $rc ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
}

args=()
for a in "$@" +; do
  if [ "$a" = "+" ]; then
    [ ${#args[@]} -gt 0 ] && step "${args[@]}"
    args=()
  else
    args+=("$a")
  fi
done
exit 0
