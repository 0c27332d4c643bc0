#!/usr/bin/env python3
"""Per-call latency of the crate-API path (INTEGRATION.md Route A): one slice per call, the
way the reference calls ReedSolomonCoder (reed_solomon.rs:88-128 shred, :140-208 deshred;
once per 32 KiB slice from block_producer.rs:339-345 / slot_block_data.rs:353).

Each call is H2D + kernel(s) + D2H through the C ABI (ctypes from Python, so a few us of
interpreter overhead per ctypes call are included and reported separately as the cost of
a no-op ABI call).  Prints one JSON line with median / p90 microseconds per call:
  shred    ReedSolomonCoder::shred(max payload)          -> 32 + 32 shreds of 1 KiB
  deshred  ReedSolomonCoder::deshred(first 32 lost)      -> payload + re-encoded coding
  deshred_random_32_of_64  the same from a random 32 of the 64 shreds (the follower's arrival)
  encoder  ReedSolomonEncoder: 32 x add_original_shard + encode + 32 recovery reads
"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from alpenglow_amd import rs

    ctx = rs.Context(0)
    coder = rs.ReedSolomonCoder(ctx, 32)
    payload = os.urandom(rs.MAX_DATA_PER_SLICE)
    raw = coder.shred(payload)
    shreds = [None] * 32 + [(False, c) for c in raw.coding]
    import random

    keep = set(random.Random(7).sample(range(64), 32))  # the follower's random 32 of 64
    shreds_r = [((j < 32), (raw.data + raw.coding)[j]) if j in keep else None for j in range(64)]
    enc = rs.ReedSolomonEncoder(ctx, 32, 32, 1024)

    def t_shred():
        coder.shred(payload)

    def t_deshred():
        got, _ = coder.deshred(shreds)
        assert got == payload

    def t_deshred_random():
        got, _ = coder.deshred(shreds_r)
        assert got == payload

    def t_encoder():
        enc.reset(32, 32, 1024)
        for d in raw.data:
            enc.add_original_shard(d)
        enc.encode()

    def t_noop():
        rs.load().ag_rs_abi_version()

    out = {"unit": "us per call", "slice": "32767-byte payload, 32:32 shreds of 1 KiB"}
    for name, f, reps in (("noop_abi_call", t_noop, 2000), ("shred", t_shred, 300), ("deshred", t_deshred, 300),
                          ("deshred_random_32_of_64", t_deshred_random, 300), ("encoder", t_encoder, 300)):
        for _ in range(20):
            f()
        ts = []
        for _ in range(reps):
            a = time.perf_counter()
            f()
            ts.append((time.perf_counter() - a) * 1e6)
        ts.sort()
        out[name] = {"median": statistics.median(ts), "p90": ts[int(0.9 * len(ts))], "min": ts[0]}
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
