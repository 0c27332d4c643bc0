#!/usr/bin/env python3
"""bench_merkle.py -- slice Merkle trees on the device.

Workload: S-byte shreds, 64 per slice (TOTAL_SHREDS, shredder.rs:47; Regular shredder:
32 data + 32 coding shreds of <= 1 KiB), laid out like the RS codeword buffer (slice s =
64 contiguous shreds).  One step =
  build:  MerkleTree::new + get_root + create_proof for every shred of every slice
          (crypto/merkle.rs:281-370; shredder.rs:538-606 on the producer side)
  verify: check_proof for every shred against its slice root (merkle.rs:374-387; the
          receiver's per-shred check, shredder.rs:130-140)
Inputs are device-resident random shreds (splitmix64).  Prints one JSON line: slices/s of
build+verify, per-kernel HIP-event times, the HBM-read roofline of each kernel (each kernel
reads the shreds once; the work is SHA-256 on the VALU), and a CPU baseline (the oracle:
Python hashlib / OpenSSL SHA-256, one thread, bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
HBM_PEAK_GBPS = 8000.0


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--slices", type=int, default=65536)
    ap.add_argument("--shred-bytes", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    import torch

    from alpenglow_amd import rs

    dev = torch.device("cuda:0")
    ctx = rs.Context(0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    n, S, L = args.slices, args.shred_bytes, 64
    h = rs.merkle_height(L)
    shreds = torch.empty((n, L * S), dtype=torch.uint8, device=dev)
    rs.fill_splitmix(ctx, shreds, n, L * S, L * S, 0x3E2C1E00)
    roots = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    pstride = 32 * h * L
    proofs = torch.empty((n, pstride), dtype=torch.uint8, device=dev)
    index = torch.arange(n * L, dtype=torch.int64, device=dev).remainder(L).to(torch.int32)
    slice_of = torch.arange(n * L, device=dev) // L
    root_rep = None
    ok = torch.empty(n * L, dtype=torch.uint8, device=dev)

    def build():
        rs.merkle_build_batch(ctx, L, S, n, shreds, S, L * S, roots, None, 0, proofs, pstride)

    def verify():
        rs.merkle_verify_batch(ctx, n * L, S, shreds, S, index, root_rep, 32, proofs, 32 * h, h, ok)

    build()
    root_rep = roots[slice_of].contiguous()  # per shred: its slice's root (as received)
    for _ in range(args.warmup):
        build()
        verify()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        ev[s][0].record(stream)
        build()
        ev[s][1].record(stream)
        verify()
        ev[s][2].record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    b_ms = sum(e[0].elapsed_time(e[1]) for e in ev) / args.steps
    v_ms = sum(e[1].elapsed_time(e[2]) for e in ev) / args.steps
    all_ok = bool(ok.all().item())

    # spot check against the oracle (test infrastructure: the checker, not the product)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import merkle_oracle as mo
    host = shreds[:2].cpu().numpy().reshape(2, L, S)
    spot = all(roots[i].cpu().numpy().tobytes() == mo.MerkleTree([host[i, j].tobytes() for j in range(L)]).root()
               for i in range(2))

    read = n * L * S
    kern = {"build": {"ms": b_ms, "bytes_read": read, "achieved_GBps": read / (b_ms * 1e-3) / 1e9,
                      "sha256_blocks": n * (L * ((32 + S + 9 + 63) // 64) + 3 * (L - 1))},
            "verify": {"ms": v_ms, "bytes_read": read + n * L * 32 * (h + 1),
                       "achieved_GBps": (read + n * L * 32 * (h + 1)) / (v_ms * 1e-3) / 1e9,
                       "sha256_blocks": n * L * (((32 + S + 9 + 63) // 64) + 3 * h)}}
    for k in kern.values():
        k["sha256_blocks_per_s"] = k["sha256_blocks"] / (k["ms"] * 1e-3)
    line = {
        "metric": "slices/s slice Merkle trees (SHA-256): build roots+proofs and verify every shred",
        "value": n * args.steps / wall,
        "unit": "slices/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": wall * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32 (SHA-256)",
        "data": "synthetic (splitmix64 shreds, device-generated)",
        "config": {"workload": f"{n} slices x {L} shreds x {S} B", "slices": n, "shreds_per_slice": L,
                   "shred_bytes": S},
        "roofline": {"bound": "hbm", "kernel": "build", "achieved": kern["build"]["achieved_GBps"],
                     "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": kern["build"]["achieved_GBps"] / HBM_PEAK_GBPS, "traffic": None,
                     "note": "SHA-256 is VALU-bound; the HBM fraction shows the headroom, not the limit"},
        "kernels": kern,
        "verify": {"all_proofs_accepted": all_ok, "roots_match_oracle": spot},
    }
    if not args.no_cpu_baseline:
        t0, done = time.perf_counter(), 0
        hostall = shreds[:4096].cpu().numpy().reshape(-1, L, S)
        while time.perf_counter() - t0 < args.cpu_seconds and done < len(hostall):
            t = mo.MerkleTree([hostall[done, j].tobytes() for j in range(L)])
            for j in range(L):
                t.create_proof(j)
            done += 1
        bt = time.perf_counter() - t0
        line["cpu_baseline"] = {"value": done / bt, "unit": "slices/s (build + proofs)", "cores": 1,
                                "kind": "port",
                                "sample": f"{done} slices, oracle/merkle_oracle.py (hashlib SHA-256), one thread"}
    print(json.dumps(line), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
