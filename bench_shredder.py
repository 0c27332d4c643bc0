#!/usr/bin/env python3
"""bench_shredder.py -- the composed RegularShredder on the device (SURVEY.md §8 a10 end to
end; VERDICT r01 "composed Shredder pipeline"): ag_shredder_shred_batch (Slice framing ->
ReedSolomonCoder::shred -> slice Merkle tree -> slice signature -> 64 Shred datagrams per
slice; shredder.rs:337-345, :533-560) and ag_shredder_deshred_batch (datagrams -> parse ->
ValidatedShred::try_new with the cached commitment -> ReedSolomonCoder::deshred ->
check_merkle_tree -> SlicePayload::try_from -> fill_missing_shreds; shredder.rs:282-311,
validated_shred.rs:52-81).

Workload: n maximum slices (32 758 data bytes + 9-byte header = 32 767-byte payload, 1 KiB
shreds).  Shred builds all 64 datagrams per slice; deshred receives, per slice, the first
32..64 datagrams of a seeded random arrival order (the follower deshreds once 32 arrived,
slot_block_data.rs:331-370) and fills in the rest.  Device-resident buffers; wall clock
around each (synchronous) call.  Prints one JSON line; the verify block checks the round
trip (every payload and datagram restored) and a spot check against the CPU composition of
the reference (oracle/shredder_oracle.py, checker only).
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
PKT = 1344  # datagram slot (1325 bytes for a 1 KiB shred, rounded to 64)
# name -> (AG_SHREDDER_*, coding shreds of its coder, key bytes appended to the payload)
NAMES = {"regular": "RegularShredder", "coding_only": "CodingOnlyShredder", "pets": "PetsShredder",
         "aont": "AontShredder"}
KINDS = {"regular": (0, 32, 0), "coding_only": (1, 64, 0), "pets": (2, 33, 16), "aont": (3, 32, 16)}


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--slices", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--arrived", type=int, default=32, help="datagrams received per slice before deshred (32..64)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--shred-bytes", type=int, default=1024,
                    help="shred size S (even, <= 1024): payloads of 32 S - 1 bytes; 1024 = maximum slices")
    ap.add_argument("--kind", choices=list(KINDS), default="regular",
                    help="the shredder (shredder.rs:336-500); the CPU baseline is timed for regular only")
    args = ap.parse_args()
    import numpy as np
    import torch

    from alpenglow_amd import rs

    dev = torch.device("cuda:0")
    torch.zeros(1, device=dev)
    ctx = rs.Context(0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    n, S = args.slices, args.shred_bytes
    assert S % 2 == 0 and 64 <= S <= 1024, "--shred-bytes: even, 64..1024"
    kind, m, extra = KINDS[args.kind]
    D = 32 * S - 1 - 9 - extra  # data bytes: framed payload (+ key) = MAX_DATA_PER_SLICE
    stride = (32 + m) * S
    data = torch.empty((n, 32 * S), dtype=torch.uint8, device=dev)
    rs.fill_splitmix(ctx, data, n, 32 * S, 32 * S, 0x5EED0000)
    g = torch.Generator(device="cpu").manual_seed(0xA221)
    slots = torch.randint(0, 1 << 40, (n,), generator=g, dtype=torch.int64).to(dev)
    sidx = torch.randint(0, 1024, (n,), generator=g, dtype=torch.int64).to(dev)
    last = (torch.arange(n) % 1024 == 1023).to(torch.uint8).to(dev)
    seed = torch.arange(32, dtype=torch.uint8).to(dev)
    pk = torch.empty(32, dtype=torch.uint8, device=dev)
    rs.ed25519_public_key_batch(ctx, 1, seed, pk)
    cw = torch.empty((n, stride), dtype=torch.uint8, device=dev)
    keys = torch.randint(0, 256, (n * 16,), generator=g, dtype=torch.uint8).to(dev)
    pkts = torch.zeros((n * 64, PKT), dtype=torch.uint8, device=dev)
    lens = torch.zeros(n * 64, dtype=torch.int32, device=dev)
    parents, dlens = [None] * n, np.full(n, D, np.uint32)
    # arrival: per slice the first `arrived` of a random order
    order = torch.argsort(torch.rand((n, 64), generator=g), dim=1)
    keep = torch.zeros((n, 64), dtype=torch.bool)
    keep.scatter_(1, order[:, :args.arrived], True)
    keep = keep.reshape(-1).to(dev)

    def shred():
        if kind == 0:
            rs.shredder_shred_batch(ctx, n, S, parents, data, 32 * S, dlens, slots, sidx, last, seed, pk, cw, pkts,
                                    PKT, lens)
        else:
            rs.shredder_shred_batch_kind(ctx, kind, n, S, parents, data, 32 * S, dlens, slots, sidx, last, seed, pk,
                                         keys, cw, stride, pkts, PKT, lens)

    def deshred():
        if kind == 0:
            return rs.shredder_deshred_batch(ctx, n, S, pkts, PKT, lens, pk, cw)
        return rs.shredder_deshred_batch_kind(ctx, kind, n, S, pkts, PKT, lens, pk, cw, stride)

    shred()
    torch.cuda.synchronize()
    full_lens = lens.clone()
    full_pkts = pkts[: 64 * 8].clone()
    for _ in range(args.warmup):
        lens.mul_(keep)
        deshred()
        shred()
    torch.cuda.synchronize()
    t_sh = t_de = 0.0
    for _ in range(args.steps):
        a = time.perf_counter()
        shred()
        torch.cuda.synchronize()
        b = time.perf_counter()
        lens.mul_(keep)  # the datagrams that did not arrive
        torch.cuda.synchronize()
        c = time.perf_counter()
        res = deshred()  # synchronous
        d = time.perf_counter()
        t_sh += b - a
        t_de += d - c
    ok = bool((res.status == 0).all()) and bool(torch.equal(lens, full_lens)) and \
        bool(torch.equal(pkts[: 64 * 8], full_pkts)) and bool((res.data_lens == D).all())
    off = res.data_offsets[:64].tolist()
    ok = ok and all(torch.equal(cw[b, off[b]:off[b] + D], data[b, :D]) for b in range(64))
    # spot check: two slices against the CPU composition of the reference (checker only)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import shredder_oracle as so
    hp, hl = pkts[:128].cpu().numpy(), lens[:128].cpu().numpy()
    hk = keys[:32].cpu().numpy().tobytes()
    sl, si, ls = slots[:2].cpu().tolist(), sidx[:2].cpu().tolist(), last[:2].cpu().tolist()
    spot = True
    for b in range(2):
        want, *_ = so.shred_kind(kind, None, data[b, :D].cpu().numpy().tobytes(), sl[b], si[b], bool(ls[b]),
                                 bytes(range(32)), hk[16 * b:16 * b + 16])
        spot &= all(hp[b * 64 + j, :hl[b * 64 + j]].tobytes() == want[j] for j in range(64))
    steps = args.steps
    line = {
        "metric": f"slices/s composed {NAMES[args.kind]} shred + deshred (datagrams in, datagrams out), "
                  + ("max slices" if S == 1024 else f"{S}-byte shreds"),
        "value": n * steps / (t_sh + t_de),
        "unit": "slices/s",
        "n_gpus": 1,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": (t_sh + t_de) * 1e3 / steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64 payloads, device-generated; one leader key)",
        "config": {"workload": f"{n} slices x {D + 9} B payload, 64 datagrams of {S + 301} B per slice; deshred from a "
                               f"random {args.arrived} of 64 datagrams per slice"},
        "payload_GiBps": n * (D + 9) * steps / (t_sh + t_de) / GIB,
        "calls_ms": {"shred_batch": t_sh * 1e3 / steps, "deshred_batch": t_de * 1e3 / steps},
        "shred_slices_per_s": n * steps / t_sh,
        "deshred_slices_per_s": n * steps / t_de,
        "verify": {"roundtrip_restores_everything": ok, "datagrams_match_oracle": bool(spot)},
    }
    if not args.no_cpu_baseline and kind == 0:
        line["cpu_baseline"] = _cpu_baseline(args, data, slots, sidx, last, cw, pkts, D, S)
    print(json.dumps(line), flush=True)
    ctx.close()


def _host_cpus():
    n = len(os.sched_getaffinity(0))
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def _cpu_baseline(args, data, slots, sidx, last, cw, pkts, D, S):
    """The composed RegularShredder on this host's CPU (oracle/shredder_cpu.c, a port: the
    crate's Avx2 RS engine restated, OpenSSL's SHA-256 and Ed25519), on a bounded sample of
    the same slices: shred (RS + Merkle tree + signature + proofs), the reference bench's
    deshred from the 32 coding shreds (RS decode + re-encode + Merkle check + parse + proofs;
    benches/shredder.rs:19-61) and the receive-side validation the device deshred also does
    (each shred's root from its path, one signature verified per slice).  1 thread and every
    host CPU; its coding shreds and signatures are compared with the device's."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np

    import ed25519_oracle as ed
    import shredder_cpu as sc

    seed = bytes(range(32))
    pk = ed.secret_to_public(seed)
    nall = _host_cpus()
    n = min(data.shape[0], max(64, nall * 64))
    framed = np.zeros((n, 32 * S), np.uint8)
    framed[:, 1:9] = np.frombuffer(int(D).to_bytes(8, "little"), np.uint8)
    framed[:, 9:9 + D] = data[:n, :D].cpu().numpy()
    lens = np.full(n, D + 9, np.uint32)
    sl, si, ls = slots[:n].cpu().numpy(), sidx[:n].cpu().numpy(), last[:n].cpu().numpy()

    def rate(what, threads, cnt):
        t = time.perf_counter()
        st, *_ = sc.run(what, threads, framed[:cnt], lens[:cnt], sl[:cnt], si[:cnt], ls[:cnt], seed, pk)
        dt = time.perf_counter() - t
        if st:
            raise RuntimeError(f"shredder_cpu failed ({st})")
        return cnt / dt

    out = {"unit": "slices/s", "kind": "port", "cores": nall, "cpu": _cpu_model()}
    # device comparison: the first 8 slices' coding shreds and slice signatures
    st, coding, _, sigs = sc.run(sc.SHRED, 1, framed[:8], lens[:8], sl[:8], si[:8], ls[:8], seed, pk, outputs=True)
    gc = cw[:8, 32 * S:64 * S].cpu().numpy().reshape(8, 32, S)
    gsig = pkts.view(-1, 64, pkts.shape[1])[:8, 0, 37 + S:37 + S + 64].cpu().numpy()
    out["gpu_matches_cpu"] = bool(st == 0 and np.array_equal(coding, gc) and np.array_equal(sigs, gsig))
    for threads in (1, nall):
        cnt = min(n, 64 * threads)
        r_sh = rate(sc.SHRED, threads, cnt)
        r_bench = rate(sc.SHRED | sc.DESHRED, threads, cnt)
        r_all = rate(sc.SHRED | sc.DESHRED | sc.RECEIVE, threads, cnt)
        t_sh, t_de, t_rx = 1 / r_sh, 1 / r_bench - 1 / r_sh, 1 / r_all - 1 / r_bench
        out[f"threads_{threads}"] = {
            "slices": cnt, "threads": threads,
            "shred_slices_per_s": r_sh, "deshred_slices_per_s": 1 / t_de,
            "receive_slices_per_s": 1 / t_rx,
            "reference_bench_roundtrip_slices_per_s": r_bench,
            "device_shape_roundtrip_slices_per_s": r_all,
        }
    out["value"] = out[f"threads_{nall}"]["device_shape_roundtrip_slices_per_s"]
    out["sample"] = (f"{n} of the same maximum slices (framed 32 767-byte payloads), shred + receive validation + "
                     f"deshred from the 32 coding shreds, one slice per task; RS by oracle/rs_cpu_avx2.c, SHA-256 "
                     f"and Ed25519 by OpenSSL libcrypto")
    return out


def _cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


if __name__ == "__main__":
    main()
