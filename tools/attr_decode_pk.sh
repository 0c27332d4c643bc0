set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in libalpenglow_rs libalpenglow_rs_noin libalpenglow_rs_noout libalpenglow_rs_noboth; do
  AG_RS_LIB_NAME=$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_$v -o kt --output-format csv -- python3 bench_coder.py --random-patterns --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/kt_$v.log 2>&1 || { echo "STOP $v"; exit 1; }
  echo "$v"; find gpurun_out/kt_$v -name "*kernel_stats.csv" -exec grep decode_pk {} \; | cut -c1-160
done
