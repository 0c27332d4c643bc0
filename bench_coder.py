#!/usr/bin/env python3
"""bench_coder.py -- the ReedSolomonCoder contract over batches of slices (SURVEY.md §8(f)
row 1), shaped like the reference's own benchmark (benches/shredder.rs:40-60): a maximum
slice (32 767-byte payload -> 32 data + 32 coding shreds of 1 KiB) is shredded, its 32
data shreds are dropped, and it is deshredded (restore, padding strip, re-encode of all
coding shreds; reed_solomon.rs:88-128, 140-208).

One step over n slices = ag_rs_coder_shred_batch (pad + encode, in place) then
ag_rs_coder_deshred_batch with every data shred absent (ANY_K by default; --exact for the
crate decoder).  Device-resident codewords (64 KiB per slice).  Prints one JSON line:
slices/s, payload GiB/s, per-call ms, and a CPU baseline (the C oracle: pad + encode,
decode + re-encode, 16 threads, bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
GIB = float(1 << 30)


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--slices", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--exact", action="store_true", help="crate decoder (EXACT) instead of ANY_K")
    ap.add_argument("--coding-only", action="store_true",
                    help="CodingOnlyShredder shape: 32:64, deshred from coding shreds 32..63 (the "
                         "reference bench drops the first 32 output shreds)")
    ap.add_argument("--random-patterns", action="store_true",
                    help="the follower's real deshred: per slice, the first 32 of its 64 shreds to arrive "
                         "in a seeded random order (slot_block_data.rs:331-370 deshreds at the 32nd), so data "
                         "and coding shreds are lost in arbitrary per-slice patterns")
    ap.add_argument("--payload-len", type=int, default=32767,
                    help="payload bytes per slice (default MAX_DATA_PER_SLICE = 32767: 1 KiB shreds); the "
                         "shred size is the padded length / 32 (reed_solomon.rs:94-95), e.g. 16383 -> 512 B")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    import numpy as np
    import torch

    from alpenglow_amd import rs

    dev = torch.device("cuda:0")
    ctx = rs.Context(0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    L = args.payload_len  # MAX_DATA_PER_SLICE by default: pads to S = 1024 (reed_solomon.rs:94-95)
    if not 0 <= L <= 32767:
        raise SystemExit("--payload-len must be in [0, 32767]")
    n, S, m = args.slices, (L + 64 - L % 64) // 32, (64 if args.coding_only else 32)
    stride = (32 + m) * S
    cw = torch.empty((n, stride), dtype=torch.uint8, device=dev)
    rs.fill_splitmix(ctx, cw, n, 32 * S, stride, 0xC0DE0000)  # payload bytes in the data regions
    lens = np.full(n, L, np.uint32)
    dpres, cpres = np.zeros(32 * n, np.uint8), np.ones(m * n, np.uint8)
    if args.coding_only:  # output shreds are the 64 coding shreds; the first 32 are dropped
        cpres = np.tile(np.array([0] * 32 + [1] * 32, np.uint8), n)
    if args.random_patterns:
        rng = np.random.default_rng(0xA221)
        arrived = np.argsort(rng.random((n, 64)), axis=1)[:, :32]  # first 32 arrivals per slice
        present = np.zeros((n, 64), np.uint8)
        np.put_along_axis(present, arrived, 1, axis=1)
        if args.coding_only:  # the 64 output shreds are the coding shreds (shredder.rs:362-395)
            dpres = np.zeros(32 * n, np.uint8)
            cpres = np.ascontiguousarray(present).reshape(-1)
        else:
            dpres = np.ascontiguousarray(present[:, :32]).reshape(-1)
            cpres = np.ascontiguousarray(present[:, 32:]).reshape(-1)
    mode = rs.DECODE_EXACT if args.exact else rs.DECODE_ANY_K

    def shred():
        rs.coder_shred_batch(ctx, m, n, S, None, 0, lens, cw, stride)

    def deshred():
        return rs.coder_deshred_batch(ctx, m, n, S, cw, stride, dpres, cpres, mode=mode, as_array=True)

    shred()
    for _ in range(args.warmup):
        shred()
        deshred()
    torch.cuda.synchronize()
    t_sh = t_de = 0.0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        a = time.perf_counter()
        shred()
        torch.cuda.synchronize()
        b = time.perf_counter()
        res = deshred()  # synchronous (payload lengths come back to the host)
        c = time.perf_counter()
        t_sh += b - a
        t_de += c - b
    wall = time.perf_counter() - t0
    ok = bool((res == L).all())
    if args.random_patterns:
        # zero every absent shred, deshred once more, compare with the original codewords
        want = cw.clone()
        pres = torch.from_numpy(np.concatenate([dpres.reshape(n, 32), cpres.reshape(n, m)], axis=1)).to(dev)
        view = cw.view(n, 32 + m, S)
        view.mul_(pres.unsqueeze(-1))
        res2 = deshred()
        ok = ok and bool((res2 == L).all()) and bool(torch.equal(cw, want))
        del want
    # spot check vs the oracle's ReedSolomonCoder (checker only)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import rs_oracle as o
    host = cw[:2].cpu().numpy()
    spot = True
    for i in range(2):
        raw = o.coder_shred(host[i, :L].tobytes(), m)
        spot &= host[i, :32 * S].tobytes() == b"".join(raw.data)
        spot &= host[i, 32 * S:].tobytes() == b"".join(raw.coding)
    size = "max slices" if L == 32767 else f"{L}-byte slices"
    line = {
        "metric": (f"slices/s ReedSolomonCoder shred + deshred (random 32 of 64 output shreds per slice), {size}"
                   if args.random_patterns else
                   f"slices/s ReedSolomonCoder shred + deshred (first 32 output shreds lost), {size}"),
        "value": n * args.steps / wall,
        "unit": "slices/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": wall * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8 (GF(2^16) symbols)",
        "data": "synthetic (splitmix64 payloads, device-generated)",
        "config": {"workload": f"{n} slices x {L} B payload, 32:{m} shreds of {S} B, deshred from "
                               + ("a random 32 of the 64 coding shreds per slice (CodingOnlyShredder)"
                      if args.coding_only and args.random_patterns else
                      "coding shreds 32..63 (CodingOnlyShredder)" if args.coding_only else
                                  "a random 32 of the 64 shreds per slice (RegularShredder)" if args.random_patterns
                                  else "the 32 coding shreds (RegularShredder)"),
                   "mode": "EXACT" if args.exact else "ANY_K"},
        "payload_GiBps": n * L * args.steps / wall / GIB,
        "calls_ms": {"shred_batch": t_sh * 1e3 / args.steps, "deshred_batch": t_de * 1e3 / args.steps},
        "verify": {"all_slices_restored": ok, "shreds_match_oracle": bool(spot)},
    }
    if not args.no_cpu_baseline and not args.coding_only and not args.random_patterns:
        import ro_c
        threads = max(1, min(16, len(os.sched_getaffinity(0))))
        ns = min(n, 2048)
        blocks = host_blocks = cw[:ns, :32 * S].cpu().numpy().reshape(ns, 32, S)
        t = time.perf_counter()
        par = ro_c.encode_blocks(host_blocks, m, threads=threads)  # shred: encode
        t1 = time.perf_counter()
        codewords = np.concatenate([np.zeros_like(blocks).reshape(ns, -1), par.reshape(ns, -1)], axis=1)
        restored = ro_c.decode_blocks(codewords.reshape(ns, 64, S), 32, [0] * 32, [1] * 32, threads=threads)
        ro_c.encode_blocks(np.ascontiguousarray(restored.reshape(ns, 32, S)), m, threads=threads)  # re-encode
        t2 = time.perf_counter()
        line["cpu_baseline"] = {"value": ns / (t2 - t), "unit": "slices/s (shred + deshred)", "cores": threads,
                                "kind": "port",
                                "sample": f"{ns} slices, C oracle encode / decode / re-encode, {threads} threads",
                                "shred_slices_per_s": ns / (t1 - t), "deshred_slices_per_s": ns / (t2 - t1)}
    print(json.dumps(line), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
