#!/bin/bash
# Round-2 measurement sweep: lost-coding decoders (decode_c; decode_x with AG_RS_NO_CORR=1
# for comparison), tail chunks, LowRate sub-window, PCIe.
# Every GPU step has its own limit; a fatal exit ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/r02_sweep.jsonl
: > $OUT
run() {  # label, bench args...
  local label=$1; shift
  timeout -k 10 240 python bench.py --no-cpu-baseline --steps 10 "$@" > gpurun_out/sw.json 2> gpurun_out/sw.err
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$label exit $rc"; tail -3 gpurun_out/sw.err; [ $rc -ge 124 ] && exit $rc; return 0; fi
  python -c "
import json,sys; d=json.load(open('gpurun_out/sw.json')); d['label']='$label'
print(json.dumps(d))" >> $OUT
  python -c "
import json; d=json.load(open('gpurun_out/sw.json')); k=d['kernels']
print('$label', round(d['value'],1), d['unit'], {n: (round(r['ms'],3), round(r['achieved_GBps'] or 0)) for n,r in k.items()}, d['verify'])"
}
run dc_lose4 --lose-coding 4 --only decode
run dc_lose8 --lose-coding 8 --only decode
run dc_lose16 --lose-coding 16 --only decode
run dc_rand_lose4 --random-patterns --lose-coding 4 --only decode
run dc_rand_lose8 --random-patterns --lose-coding 8 --only decode
run dc_rand_lose16 --random-patterns --lose-coding 16 --only decode
export AG_RS_NO_CORR=1  # the same patterns on decode_x (the round-1 decoder)
run dx_lose4 --lose-coding 4 --only decode
run dx_rand_lose8 --random-patterns --lose-coding 8 --only decode
unset AG_RS_NO_CORR
run tail_32x32_S1000 --block-bytes 32000 --nblocks 131072
run tail_32x32_S1022 --block-bytes 32704 --nblocks 131072
run tail_16x4_S1000 --k 16 --m 4 --block-bytes 16000 --nblocks 262144
run lr_32x64_S1024_mixed --m 64 --block-bytes 32768 --nblocks 65536 --random-patterns --lose-coding 16
run lr_32x33_S1024_mixed --m 33 --block-bytes 32768 --nblocks 65536 --random-patterns --erase 16 --lose-coding 8
run pcie_32x32 --pcie --steps 3 --nblocks 4096
exit 0
