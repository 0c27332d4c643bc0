#!/usr/bin/env python3
"""bench_aon.py -- the AONT / PETS shredders' payload transforms on the device (SURVEY.md
§8(f) row 3): per maximum slice (32 751-byte payload + 16-byte key tail), AES-128-CTR over
the payload and (AONT) SHA-256 of the ciphertext (shredder.rs:414-418, 463-470, 509-528).

One step over n slices = ag_aon_encrypt_batch then ag_aon_decrypt_batch (in place).  Prints
one JSON line: payload GiB/s per scheme and kernel, and a CPU baseline (the oracle's pure
Python AES -- a lower bound for a CPU, labelled as such -- plus hashlib SHA-256, one thread).
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
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    args = ap.parse_args()
    import numpy as np
    import torch

    from alpenglow_amd import rs

    dev = torch.device("cuda:0")
    ctx = rs.Context(0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    n, L, stride = args.slices, 32767 - 16, 32768
    buf = torch.empty((n, stride), dtype=torch.uint8, device=dev)
    rs.fill_splitmix(ctx, buf, n, stride, stride, 0xA0E70000)
    keys = torch.randint(0, 256, (16 * n,), dtype=torch.uint8, device=dev)
    lens = np.full(n, L, np.uint32)
    lens_t = np.full(n, L + 16, np.uint32)
    res = {}
    for name, scheme in (("aont", rs.AON_AONT), ("pets", rs.AON_PETS)):
        for _ in range(args.warmup):
            rs.aon_encrypt_batch(ctx, scheme, n, keys, buf, stride, lens)
            rs.aon_decrypt_batch(ctx, scheme, n, buf, stride, lens_t)
        torch.cuda.synchronize()
        te = td = 0.0
        for _ in range(args.steps):
            a = time.perf_counter()
            rs.aon_encrypt_batch(ctx, scheme, n, keys, buf, stride, lens)
            torch.cuda.synchronize()
            b = time.perf_counter()
            out = rs.aon_decrypt_batch(ctx, scheme, n, buf, stride, lens_t)
            c = time.perf_counter()
            te += b - a
            td += c - b
        res[name] = {"encrypt_ms": te * 1e3 / args.steps, "decrypt_ms": td * 1e3 / args.steps,
                     "encrypt_GiBps": n * L * args.steps / te / GIB, "decrypt_GiBps": n * L * args.steps / td / GIB,
                     "ok": bool((out == L).all())}
    # keystream alone (the AES-CTR kernel) and SHA-256 alone
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    dig = torch.empty(32 * n, dtype=torch.uint8, device=dev)
    ev[0].record(stream)
    rs.cipher_apply_keystream_batch(ctx, n, keys, buf, stride, lens)
    ev[1].record(stream)
    rs.sha256_batch(ctx, n, buf, stride, lens, dig)
    ev[2].record(stream)
    torch.cuda.synchronize()
    ks_ms, sha_ms = ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])
    # oracle spot check (checker only) and a CPU baseline on a bounded sample
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cipher_oracle as co
    host = buf[:1].cpu().numpy()[0]
    k0 = keys[:16].cpu().numpy().tobytes()
    enc = co.aont_encrypt(host[:L].tobytes(), k0)
    rs.aon_encrypt_batch(ctx, rs.AON_AONT, 1, keys, buf, stride, [L])
    spot = buf[0, : L + 16].cpu().numpy().tobytes() == enc
    t = time.perf_counter()
    co.aont_encrypt(host[:4096].tobytes(), k0)
    cpu_aes = 4096 / (time.perf_counter() - t)
    t = time.perf_counter()
    for _ in range(200):
        co.sha256(host[:L].tobytes())
    cpu_sha = 200 * L / (time.perf_counter() - t)
    line = {
        "metric": "GiB/s AONT / PETS payload transforms (AES-128-CTR + SHA-256 key masking), max slices",
        "value": res["aont"]["encrypt_GiBps"],
        "unit": "GiB/s (AONT encrypt, payload bytes)",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8 / u32 (AES T-tables, SHA-256)",
        "data": "synthetic (splitmix64 payloads, device-generated; random keys)",
        "config": {"workload": f"{n} slices x {L} B payload + 16 B key tail"},
        "schemes": res,
        "kernels": {"aes_ctr_ms": ks_ms, "aes_ctr_GBps": n * L / (ks_ms * 1e-3) / 1e9,
                    "sha256_ms": sha_ms, "sha256_GBps": n * L / (sha_ms * 1e-3) / 1e9},
        "roofline": {"bound": "hbm", "kernel": "aes_ctr", "achieved": 2 * n * L / (ks_ms * 1e-3) / 1e9,
                     "peak": 8000.0, "unit": "GB/s", "frac": 2 * n * L / (ks_ms * 1e-3) / 1e9 / 8000.0,
                     "traffic": None, "note": "read + write of the payload; AES is LDS-lookup bound"},
        "verify": {"roundtrips": all(v["ok"] for v in res.values()), "aont_matches_oracle": bool(spot)},
        "cpu_baseline": {"value": cpu_aes / GIB, "unit": "GiB/s (AES-CTR, pure-Python oracle)", "cores": 1,
                         "kind": "port", "sample": "4096 bytes through oracle/cipher_oracle.py (pure-Python "
                                                   "AES: a lower bound, not a tuned CPU AES)",
                         "sha256_GiBps_hashlib": cpu_sha / GIB},
    }
    print(json.dumps(line), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
