#!/usr/bin/env python3
"""Repeat the 64-point transform decode with per-block store masks (test_transform64_geometries'
per-block case) many times in one process and report every mismatch (block, shard, first
differing chunk) -- an intermittent-result hunt, no faults.  AG_RS_LIB_NAME selects another
build of the library in alpenglow_amd/_lib (e.g. a diagnostic build of an older kernel).

Usage: python tools/stress_xform64.py [--iters 40] [--n 9] [--S 1024] [--seed 9]
"""
import argparse
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seed", type=int, default=9)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--n", type=int, default=9)
    ap.add_argument("--S", type=int, default=1024)
    args = ap.parse_args()
    import numpy as np
    import torch

    import ro_c
    import rs_oracle as o
    from alpenglow_amd import rs

    rs.load()
    dev = torch.device("cuda:0")
    ctx = rs.Context(0)
    st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(st)
    ctx.set_stream(st.cuda_stream)
    k, m, S, n = 64, 64, args.S, args.n
    blocks = np.stack([np.frombuffer(o.block_bytes(4100 + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    rec = ro_c.encode_blocks(blocks, m, threads=8)
    d_rec = torch.from_numpy(rec.reshape(n, m * S).copy()).to(dev)
    bad = {}
    for v in [args.seed]:
        rng = random.Random(v)
        bad[v] = 0
        for it in range(args.iters):
            op = []
            for b in range(n):
                lost = set(rng.sample(range(k), rng.randrange(1, 64)))
                op.append([0 if i in lost else 1 for i in range(k)])
            opa = np.array(op, np.uint8)
            damaged = blocks.copy()
            damaged[opa == 0] = 0x5A
            d_o = torch.from_numpy(damaged.reshape(n, k * S).copy()).to(dev)
            rs.decode_batch(ctx, k, m, S, n, d_o, k * S, d_rec, m * S, opa.reshape(-1), np.ones(n * m, np.uint8),
                            mode=rs.DECODE_ANY_K)
            got = d_o.cpu().numpy().reshape(n, k, S)
            if not np.array_equal(got, blocks):
                bad[v] += 1
                diff = np.argwhere(got != blocks)
                shards = sorted({(int(b), int(s)) for b, s, _ in diff})
                print(f"seed {v} iter {it}: {len(diff)} bytes differ in {len(shards)} shards, "
                      f"first {shards[:6]}, chunks {sorted({int(x) // 64 for _, _, x in diff})[:8]}, "
                      f"erased? {[bool(opa[b, s] == 0) for b, s in shards[:6]]}", flush=True)
                if bad[v] <= 3:  # (chunk, 16-byte quarter) map of the first bad shard: '#' differs
                    b0, s0 = shards[0]
                    d = (got[b0, s0] != blocks[b0, s0]).reshape(-1, 4, 16).any(axis=2)
                    print("   block", b0, "shard", s0, "quarters by chunk:",
                          " ".join("".join("#" if x else "." for x in row) for row in d), flush=True)
                    # what the bad pieces hold: the erasure fill (store missing), or another piece
                    pieces = {}
                    for bb in range(n):
                        for ss in range(k):
                            for pi, pc in enumerate(blocks[bb, ss].reshape(-1, 16)):
                                pieces.setdefault(pc.tobytes(), (bb, ss, pi // 4, pi % 4))
                    gp = got[b0, s0].reshape(-1, 16)
                    badp = [pi for pi in range(gp.shape[0]) if d.reshape(-1)[pi]]
                    fill = sum(bool((gp[pi] == 0x5A).all()) for pi in badp)
                    where = [pieces.get(gp[pi].tobytes()) for pi in badp[:6]]
                    print(f"   {len(badp)} bad pieces: {fill} hold the 0x5A fill; first as pieces of "
                          f"(block, shard, chunk, quarter): {where} (wanted chunk/quarter {[(pi // 4, pi % 4) for pi in badp[:6]]})",
                          flush=True)
    print({"mismatching_iterations": bad, "iters": args.iters, "n": n, "S": S})


if __name__ == "__main__":
    main()
