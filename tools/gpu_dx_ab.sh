set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "general or decode" > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || exit $rc
for r in 1 2; do for lib in libalpenglow_rs.so libhead.so; do for args in "--lose-coding 4" "--random-patterns --lose-coding 8"; do
AG_RS_LIB_NAME=$lib timeout -k 10 200 python bench.py $args --only decode --steps 3 --warmup 1 --no-cpu-baseline --no-verify > gpurun_out/dx.json 2>/dev/null || exit 3
python3 -c "import json;d=json.load(open('gpurun_out/dx.json'));print('$lib', '$args', round(d['kernels']['reconstruct']['ms'],3), round(d['kernels']['reconstruct']['achieved_GBps']))"
done; done; done
