"""Host-side cost of decode_batch calls with per-block patterns: the time a call takes to
return (enqueue: host bookkeeping + launches, no sync) against the synchronized time.
Run on the GPU box: python tools/host_enqueue.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from alpenglow_amd import rs  # noqa: E402
from alpenglow_amd.shard import RankPlan, erasure_patterns  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    ctx = rs.Context(0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    k = m = 32
    n = 131072
    for S, lc in ((960, 0), (960, 4), (1000, 0), (1000, 4), (1024, 4)):
        cw_stride = (k + m) * S
        cw = torch.empty((n, cw_stride), dtype=torch.uint8, device=dev)
        rs.fill_splitmix(ctx, cw, n, k * S, cw_stride, 7)
        d, p = cw.data_ptr(), cw.data_ptr() + k * S
        rs.encode_batch(ctx, k, m, S, n, d, cw_stride, p, cw_stride)
        plan = RankPlan(0, 1, n)
        o, r = erasure_patterns(plan, k, m, 16, lc, True)
        ob, rb = bytes(o), bytes(r)
        for _ in range(3):
            rs.decode_batch(ctx, k, m, S, n, d, cw_stride, p, cw_stride, ob, rb)
        torch.cuda.synchronize()
        enq, tot = [], []
        for _ in range(5):
            t0 = time.perf_counter()
            rs.decode_batch(ctx, k, m, S, n, d, cw_stride, p, cw_stride, ob, rb)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            enq.append(t1 - t0)
            tot.append(t2 - t0)
        print(f"S={S} lose_coding={lc}: enqueue {1e3 * min(enq):.2f} ms, synchronized {1e3 * min(tot):.2f} ms",
              flush=True)
        del cw
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
