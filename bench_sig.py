#!/usr/bin/env python3
"""bench_sig.py -- shred signatures on the device.

Workload: one leader key; S-byte shreds, 64 per slice, each carrying its Merkle path and the
leader's Ed25519 signature over the 49-byte SliceCommitment (shredder.rs:206-215, :540).
Timed kernels (device-resident inputs, HIP events on the launch stream):
  verify    Signature::verify_bytes over N commitments (ed25519-zebra ZIP-215 rules)
  validate  ValidatedShred::try_new for every shred of every slice with no cached
            commitment (derive root from the path + commitment + signature check: the
            receive path's worst case, validated_shred.rs:52-81)
  cached    the same with every shred's cached commitment matching (no signature work)
  sign      the shred side: SliceCommitment + sign per slice (shredder.rs:540)
  serialize / deserialize
            the Shred datagram (wincode layout, shredder.rs:113-186; network.rs:52-64)
            for every shred: columns -> packets and back (HBM-bound byte movement)
The headline is verifications per second.  The kernels are VALU-bound (field multiplies,
v_mad_i64_i32); the report gives the instruction-level estimate next to the rate.  CPU
baselines (one host thread): the oracle (oracle/ed25519_oracle.py, pure Python, kind
"port") and the kernels' own arithmetic compiled for the host
(tests/native/ed_host_check, "native_1thread") when that binary is present.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--sigs", type=int, default=262144)
    ap.add_argument("--slices", type=int, default=2048)
    ap.add_argument("--shred-bytes", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    import torch

    from alpenglow_amd import rs

    dev = torch.device("cuda:0")
    ctx = rs.Context(0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    N = args.sigs
    seed = torch.randint(0, 256, (32,), dtype=torch.uint8, device=dev, generator=g)
    pk = torch.zeros(32, dtype=torch.uint8, device=dev)
    rs.ed25519_public_key_batch(ctx, 1, seed, pk)
    msgs = torch.randint(0, 256, (N, 49), dtype=torch.uint8, device=dev, generator=g)
    sigs = torch.zeros((N, 64), dtype=torch.uint8, device=dev)
    rs.ed25519_sign_batch(ctx, N, seed, 0, pk, 0, msgs, 49, 49, sigs)
    ok = torch.zeros(N, dtype=torch.uint8, device=dev)

    # slices: random shreds -> Merkle roots + proofs on the device -> slice signatures
    n, S, L = args.slices, args.shred_bytes, 64
    h = rs.merkle_height(L)
    shreds = torch.empty((n, L * S), dtype=torch.uint8, device=dev)
    rs.fill_splitmix(ctx, shreds, n, L * S, L * S, 0x51C0FFEE)
    roots = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    proofs = torch.empty((n, 32 * h * L), dtype=torch.uint8, device=dev)
    rs.merkle_build_batch(ctx, L, S, n, shreds, S, L * S, roots, None, 0, proofs, 32 * h * L)
    # consecutive slices of consecutive slots (MAX_SLICES_PER_BLOCK = 1024 slices per slot)
    slots = 4242 + torch.arange(n, dtype=torch.int64, device=dev) // 1024
    slice_idx = torch.arange(n, dtype=torch.int64, device=dev) % 1024
    last = ((slice_idx == 1023) | (torch.arange(n, device=dev) == n - 1)).to(torch.uint8)
    ssig = torch.zeros((n, 64), dtype=torch.uint8, device=dev)
    commits = torch.zeros((n, 49), dtype=torch.uint8, device=dev)
    rs.slice_sign_batch(ctx, n, seed, pk, slots, slice_idx, last, roots, ssig, commits)
    # per shred: header, index, signature, cached commitment (the slice's)
    rep = torch.arange(n * L, device=dev) // L
    sh_idx = (torch.arange(n * L, device=dev) % L).to(torch.int32)
    sh_slot, sh_slice, sh_last = slots[rep].contiguous(), slice_idx[rep].contiguous(), last[rep].contiguous()
    sh_sig = ssig[rep].contiguous()
    sh_cached = commits[rep].contiguous()
    has_none = None
    has_all = torch.ones(n * L, dtype=torch.uint8, device=dev)
    status = torch.zeros(n * L, dtype=torch.uint8, device=dev)

    def k_verify():
        rs.ed25519_verify_batch(ctx, N, pk, 0, msgs, 49, sigs, 64, ok, msg_len=49)

    def k_validate(cached):
        rs.shred_validate_batch(ctx, n * L, shreds, S, S, sh_idx, proofs, 32 * h, h, sh_slot, sh_slice, sh_last,
                                sh_sig, 64, pk, status, cached=sh_cached if cached else None,
                                has_cached=has_all if cached else has_none)

    def k_sign():
        rs.slice_sign_batch(ctx, n, seed, pk, slots, slice_idx, last, roots, ssig)

    # wire format: the shreds as columns (data rows = the shreds themselves), packets back
    NS = n * L
    sh_kind = (sh_idx >= 32).to(torch.uint8)
    sh_dlen = torch.full((NS,), S, dtype=torch.int32, device=dev)
    sh_h = torch.full((NS,), h, dtype=torch.int32, device=dev)
    sh_proofs = proofs.view(NS, 32 * h)
    cols_in = rs.ShredColumns.of(sh_kind, sh_slot, sh_slice, sh_last, sh_idx, shreds, S, sh_dlen, sh_sig, sh_proofs,
                                 32 * h, sh_h)
    pstride = 1536
    packets = torch.zeros((NS, pstride), dtype=torch.uint8, device=dev)
    plens = torch.zeros(NS, dtype=torch.int32, device=dev)
    out = {k: torch.zeros_like(v) for k, v in dict(kind=sh_kind, slot=sh_slot, slice=sh_slice, last=sh_last,
                                                    idx=sh_idx, dlen=sh_dlen, h=sh_h).items()}
    o_data = torch.zeros((NS, S), dtype=torch.uint8, device=dev)
    o_sig = torch.zeros((NS, 64), dtype=torch.uint8, device=dev)
    o_proof = torch.zeros((NS, 32 * h), dtype=torch.uint8, device=dev)
    cols_out = rs.ShredColumns.of(out["kind"], out["slot"], out["slice"], out["last"], out["idx"], o_data, S,
                                  out["dlen"], o_sig, o_proof, 32 * h, out["h"])
    wstatus = torch.zeros(NS, dtype=torch.uint8, device=dev)

    def k_ser():
        rs.shred_serialize_batch(ctx, NS, cols_in, packets, pstride, plens)

    def k_deser():
        rs.shred_deserialize_batch(ctx, NS, packets, pstride, plens, cols_out, wstatus)

    phases = [("verify", k_verify), ("validate", lambda: k_validate(False)), ("cached", lambda: k_validate(True)),
              ("sign", k_sign), ("serialize", k_ser), ("deserialize", k_deser)]
    for _ in range(args.warmup):
        for _, f in phases:
            f()
    torch.cuda.synchronize()
    res = {}
    for name, f in phases:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.steps):
            f()
        e1.record(stream)
        torch.cuda.synchronize()
        res[name] = e0.elapsed_time(e1) / args.steps
    # correctness of what was timed
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    verify_ok = bool(ok.all().item())
    k_validate(False)
    torch.cuda.synchronize()
    validate_ok = bool((status == 0).all().item())
    wire_ok = bool((wstatus == 0).all().item()) and torch.equal(o_data, shreds.view(NS, S)) and \
        torch.equal(o_proof, sh_proofs) and torch.equal(out["idx"], sh_idx) and torch.equal(o_sig, sh_sig)
    import shred_wire_oracle as wo  # the checker (oracle/ is on sys.path)
    import ed25519_oracle as eo
    pkb = pk.cpu().numpy().tobytes()
    mh, sh = msgs[:4].cpu().numpy(), sigs[:4].cpu().numpy()
    oracle_ok = pkb == eo.secret_to_public(seed.cpu().numpy().tobytes()) and all(
        eo.verify(pkb, mh[i].tobytes(), sh[i].tobytes()) and
        sh[i].tobytes() == eo.sign(seed.cpu().numpy().tobytes(), mh[i].tobytes()) for i in range(4))

    rate = {"verify": N / (res["verify"] * 1e-3), "validate": n * L / (res["validate"] * 1e-3),
            "cached": n * L / (res["cached"] * 1e-3), "sign": n / (res["sign"] * 1e-3),
            "serialize": NS / (res["serialize"] * 1e-3), "deserialize": NS / (res["deserialize"] * 1e-3)}
    pkt0 = packets[0, :int(plens[0].item())].cpu().numpy().tobytes()
    wire_ok = wire_ok and wo.deserialize(pkt0) is not None and wo.serialize(*wo.deserialize(pkt0)) == pkt0
    wire_bytes = 2 * int(plens.to(torch.int64).sum().item())  # packet bytes once + column bytes once
    wire = {k: {"ms": res[k], "algorithmic_bytes": wire_bytes,
                "achieved_GBps": wire_bytes / (res[k] * 1e-3) / 1e9} for k in ("serialize", "deserialize")}
    line = {
        "metric": "Ed25519 shred signature verifications/s (ZIP-215, 49-byte slice commitments, one leader key)",
        "value": rate["verify"],
        "unit": "verifications/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": res["verify"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32 limbs / int64 products (GF(2^255-19))",
        "data": "synthetic (random seed, random commitments; slices of splitmix64 shreds)",
        "config": {"workload": f"{N} signatures; {n} slices x {L} shreds x {S} B", "sigs": N, "slices": n,
                   "shreds_per_slice": L, "shred_bytes": S},
        "roofline": {"bound": "valu", "kernel": "ed_verify_kernel", "achieved": None, "peak": None,
                     "unit": "verifications/s", "frac": None, "traffic": None,
                     "note": "compute-bound integer kernel: no HBM roofline applies (64 B of key/message/"
                             "signature per verification); see DESIGN.md §3.9 for the instruction estimate"},
        "kernels": {k: {"ms": res[k], "per_s": rate[k]} for k in res},
        "wire_roofline": {k: {**v, "peak_GBps": 8000.0, "frac": v["achieved_GBps"] / 8000.0} for k, v in wire.items()},
        "rates": {"verify_per_s": rate["verify"], "validate_shreds_per_s": rate["validate"],
                  "validate_cached_shreds_per_s": rate["cached"], "sign_slices_per_s": rate["sign"],
                  "serialize_shreds_per_s": rate["serialize"], "deserialize_shreds_per_s": rate["deserialize"]},
        "verify": {"all_signatures_accepted": verify_ok, "all_shreds_valid": validate_ok,
                   "wire_round_trip": wire_ok,
                   "oracle_spot_check": oracle_ok},
    }
    if not args.no_cpu_baseline:
        t0, done = time.perf_counter(), 0
        while time.perf_counter() - t0 < args.cpu_seconds:
            assert eo.verify(pkb, mh[done % 4].tobytes(), sh[done % 4].tobytes())
            done += 1
        bt = time.perf_counter() - t0
        line["cpu_baseline"] = {"value": done / bt, "unit": "verifications/s", "cores": 1, "kind": "port",
                                "sample": f"{done} verifications, oracle/ed25519_oracle.py (pure Python), one thread"}
        exe = os.path.join(ROOT, "tests", "native", "_build", "ed_host_check")
        if os.path.exists(exe):
            cmd = f"bench_verify {pkb.hex()} {mh[0].tobytes().hex()} {sh[0].tobytes().hex()} 2000\n"
            out = subprocess.run([exe], input=cmd, capture_output=True, text=True, timeout=120).stdout.split()
            line["cpu_baseline"]["native_1thread"] = {
                "value": float(out[0]) if out else None, "unit": "verifications/s",
                "sample": "2000 verifications, the kernels' ed25519_core.hpp compiled for the host (-O1), one thread"}
    print(json.dumps(line), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
