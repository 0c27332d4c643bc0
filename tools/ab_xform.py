"""Interleaved A/B of the bitsliced transform kernel variants in ONE process
(cdna_hip_programming.md section 5.4 rule 24).  Prints per-variant encode / reconstruct
times (HIP events on the launch stream) and algorithmic GB/s.

Usage: python tools/ab_xform.py [--variants 0,1] [--rounds 5] [--nblocks 4096]
"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,1")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--nblocks", type=int, default=4096)
    ap.add_argument("--shard", type=int, default=0, help="shard bytes (default: 1 MiB / k)")
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--m", type=int, default=32)
    ap.add_argument("--erase", type=int, default=-1, help="data shards erased (default k/2, at most m)")
    ap.add_argument("--lose-coding", type=int, default=0)
    ap.add_argument("--no-check", action="store_true", help="diagnostic builds with wrong output")
    args = ap.parse_args()
    import torch
    from alpenglow_amd import rs

    lib = rs.load()
    if hasattr(lib, "ag_rs_internal_set_xform_variant"):
        setv = lib.ag_rs_internal_set_xform_variant
        setv.argtypes = [ctypes.c_int]
    else:  # single-variant build: time the default kernel
        def setv(v):
            return 0
    dev = torch.device("cuda:0")
    ctx = rs.Context(0)
    st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(st)
    ctx.set_stream(st.cuda_stream)
    k, m = args.k, args.m
    S, n = args.shard or (1 << 20) // k, args.nblocks
    stride = (k + m) * S
    cw = torch.empty((n, stride), dtype=torch.uint8, device=dev)
    rs.fill_splitmix(ctx, cw, n, k * S, stride, 0x5EED_A19E_0000_0000)
    dp, pp = cw.data_ptr(), cw.data_ptr() + k * S
    e = args.erase if args.erase >= 0 else min(k // 2, m)
    op, rp = [0] * e + [1] * (k - e), [0] * args.lose_coding + [1] * (m - args.lose_coding)
    variants = [int(v) for v in args.variants.split(",")]
    res = {v: {"enc": [], "dec": []} for v in variants}
    ref = None
    for r in range(args.rounds):
        for v in variants:
            setv(v)
            rs.encode_batch(ctx, k, m, S, n, dp, stride, pp, stride)
            rs.decode_batch(ctx, k, m, S, n, dp, stride, pp, stride, op, rp)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            ev[0].record(st)
            for _ in range(args.reps):
                rs.encode_batch(ctx, k, m, S, n, dp, stride, pp, stride)
            ev[1].record(st)
            for _ in range(args.reps):
                rs.decode_batch(ctx, k, m, S, n, dp, stride, pp, stride, op, rp)
            ev[2].record(st)
            torch.cuda.synchronize()
            res[v]["enc"].append(ev[0].elapsed_time(ev[1]) / args.reps)
            res[v]["dec"].append(ev[1].elapsed_time(ev[2]) / args.reps)
            chk = cw.sum(dtype=torch.int64).item()
            if ref is None:
                ref = chk
            assert args.no_check or chk == ref, "variant changed the output"
    B = k * S
    ne = op.count(0)
    out = {}
    for v in variants:
        e = sorted(res[v]["enc"])[len(res[v]["enc"]) // 2]
        d = sorted(res[v]["dec"])[len(res[v]["dec"]) // 2]
        out[v] = {"enc_ms": e, "dec_ms": d, "enc_GBps": n * B * (1 + m / k) / e / 1e6,
                  "dec_GBps": n * B * (1 + ne / k) / d / 1e6,
                  "enc_min_ms": min(res[v]["enc"]), "dec_min_ms": min(res[v]["dec"])}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
