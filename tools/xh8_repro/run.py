#!/usr/bin/env python3
"""Drives tools/xh8_repro/_build/libxh8_repro.so (diagnostic only): 64:64 full-recovery
reconstructs with a random store mask per block, repeated, per MODE; counts the iterations
whose restored shards differ from the originals and prints the scanner's verdict for each
MODE's ISA (tools/scan_waitcnt.py).  Usage: run.py [--iters 40] [--modes 0,1,2] [--n 33]"""
import argparse
import ctypes
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]


class XformParams(ctypes.Structure):
    _fields_ = [("in_", ctypes.c_void_p), ("in_block_stride", ctypes.c_uint64), ("in_shard_stride", ctypes.c_uint64),
                ("out", ctypes.c_void_p), ("out_block_stride", ctypes.c_uint64), ("out_shard_stride", ctypes.c_uint64),
                ("out_mask", ctypes.c_void_p), ("pattern_per_block", ctypes.c_uint32), ("n_in", ctypes.c_uint32),
                ("n_out", ctypes.c_uint32), ("chunks_per_shard", ctypes.c_uint32), ("total_columns", ctypes.c_uint64),
                ("out_low_half", ctypes.c_uint32)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--modes", default="0,1,2")
    ap.add_argument("--n", type=int, default=33)
    ap.add_argument("--S", type=int, default=1024)
    args = ap.parse_args()
    import numpy as np
    import torch

    import ro_c
    import rs_oracle as o

    lib = ctypes.CDLL(os.path.join(HERE, "_build", "libxh8_repro.so"))
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    k, m, S, n = 64, 64, args.S, args.n
    blocks = np.stack([np.frombuffer(o.block_bytes(4100 + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    rec = ro_c.encode_blocks(blocks, m, threads=8)
    d_rec = torch.from_numpy(rec.reshape(n, m * S).copy()).to(dev)
    result = {}
    for mode in [int(x) for x in args.modes.split(",")]:
        rng = random.Random(1234)  # the same patterns for every mode
        bad = 0
        for it in range(args.iters):
            lost = [set(rng.sample(range(k), rng.randrange(1, 64))) for _ in range(n)]
            mask = np.array([sum(1 << i for i in ls) for ls in lost], dtype=np.uint64)
            damaged = blocks.copy()
            for b, ls in enumerate(lost):
                damaged[b, sorted(ls)] = 0x5A
            d_o = torch.from_numpy(damaged.reshape(n, k * S).copy()).to(dev)
            d_m = torch.from_numpy(mask.view(np.int64).copy()).to(dev)
            p = XformParams(d_rec.data_ptr(), m * S, S, d_o.data_ptr(), k * S, S, d_m.data_ptr(), 1, m, k, S // 64,
                            n * (S // 64), 0)
            with torch.cuda.stream(st):
                assert lib.xh8_repro_decode(mode, ctypes.byref(p), ctypes.c_void_p(st.cuda_stream)) == 0
            st.synchronize()
            got = d_o.cpu().numpy().reshape(n, k, S)
            if not np.array_equal(got, blocks):
                bad += 1
                diff = np.argwhere(got != blocks)
                b0, s0 = int(diff[0][0]), int(diff[0][1])
                fill = bool((got[b0, s0][diff[diff[:, 0] == b0][:, 2][:16]] == 0x5A).all())
                print(f"mode {mode} iter {it}: {len(diff)} bytes differ in "
                      f"{len({(int(b), int(s)) for b, s, _ in diff})} shards; first bad piece holds the fill: {fill}",
                      flush=True)
        result[mode] = bad
        print(f"mode {mode}: {bad} of {args.iters} iterations wrong", flush=True)
    print({"mismatching_iterations": result, "iters": args.iters, "n": n, "S": S})


if __name__ == "__main__":
    main()
