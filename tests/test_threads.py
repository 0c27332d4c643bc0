"""Coders driven concurrently from several threads (SURVEY.md §8(b) Threading).

The reference builds its ReedSolomonCoders on one thread (ShredderPool::with_size inside
Alpenglow::new: block_producer.rs:91, blockstore.rs:131, consensus.rs:180-233) and then drives
them from separate tokio tasks (consensus.rs:257, 266).  Objects made with a private context
(ag_rs_*_new_on_device; ctx=None in rs.py) share no state, so that pattern is safe: here two
ReedSolomonCoders, one crate-API encoder and one decoder are created on this thread and then
run at the same time on four others (ctypes releases the GIL during each call), 120 calls
each, byte-exact against the C oracle (oracle/rs_oracle.c).
"""

import random
import threading

import numpy as np
import pytest

import ro_c
from alpenglow_amd import rs

pytestmark = pytest.mark.gpu

CALLS = 120


def _padded_shards(payload: bytes) -> np.ndarray:
    """ReedSolomonCoder::shred's padding and split (reed_solomon.rs:94-117)."""
    pad = 64 - len(payload) % 64
    buf = payload + b"\x80" + b"\x00" * (pad - 1)
    return np.frombuffer(buf, np.uint8).reshape(32, len(buf) // 32)


def _coder_cases(seed):
    rng = np.random.default_rng(seed)
    r = random.Random(seed)
    cases = []
    for _ in range(CALLS):
        payload = rng.bytes(int(rng.integers(0, rs.MAX_DATA_PER_SLICE + 1)))
        data = _padded_shards(payload)
        coding = ro_c.encode(data, 32)
        keep = set(r.sample(range(64), r.randint(32, 64)))
        cases.append((payload, data, coding, keep))
    return cases


def _run_coder(coder, cases, errors, tag):
    try:
        for i, (payload, data, coding, keep) in enumerate(cases):
            raw = coder.shred(payload)
            if raw.data != [bytes(x) for x in data] or raw.coding != [bytes(x) for x in coding]:
                errors.append(f"{tag} shred {i}")
                continue
            shreds = [(j < 32, (raw.data + raw.coding)[j]) if j in keep else None for j in range(64)]
            out, raw2 = coder.deshred(shreds)
            if out != payload or raw2.data != raw.data or raw2.coding != raw.coding:
                errors.append(f"{tag} deshred {i}")
    except Exception as e:  # noqa: BLE001 -- reported by the main thread
        errors.append(f"{tag}: {e!r}")


def _run_encoder(enc, cases, errors):
    try:
        for i, (k, m, data, want) in enumerate(cases):
            enc.reset(k, m, data.shape[1])
            for row in data:
                enc.add_original_shard(row.tobytes())
            if enc.encode() != [bytes(x) for x in want]:
                errors.append(f"encoder {i}")
    except Exception as e:  # noqa: BLE001
        errors.append(f"encoder: {e!r}")


def _run_decoder(dec, cases, errors):
    try:
        for i, (k, m, data, rec, lost, lost_r) in enumerate(cases):
            dec.reset(k, m, data.shape[1])
            for a in range(k):
                if a not in lost:
                    dec.add_original_shard(a, data[a].tobytes())
            for b in range(m):
                if b not in lost_r:
                    dec.add_recovery_shard(b, rec[b].tobytes())
            got = dec.decode()
            if got != {a: data[a].tobytes() for a in sorted(lost)}:
                errors.append(f"decoder {i}")
    except Exception as e:  # noqa: BLE001
        errors.append(f"decoder: {e!r}")


def test_concurrent_private_context_coders(ctx):  # ctx: torch initialises the device first
    coders = [rs.ReedSolomonCoder(None, 32) for _ in range(2)]  # created here, used elsewhere
    enc = rs.ReedSolomonEncoder(None, 32, 32, 1024)
    dec = rs.ReedSolomonDecoder(None, 32, 32, 1024)
    coder_cases = [_coder_cases(100 + t) for t in range(2)]
    rng = np.random.default_rng(7)
    r = random.Random(7)
    enc_cases, dec_cases = [], []
    for _ in range(CALLS):
        k, m = r.choice([(32, 32), (16, 4), (32, 64), (20, 30)])
        S = 2 * r.randint(1, 600)
        data = rng.integers(0, 256, (k, S), dtype=np.uint8)
        enc_cases.append((k, m, data, ro_c.encode(data, m)))
        k, m = r.choice([(32, 32), (16, 4), (20, 30)])
        S = 64 * r.randint(1, 16)
        data = rng.integers(0, 256, (k, S), dtype=np.uint8)
        rec = ro_c.encode(data, m)
        nlost = r.randint(1, min(k, m))
        lost = set(r.sample(range(k), nlost))
        lost_r = set(r.sample(range(m), r.randint(0, m - nlost)))
        dec_cases.append((k, m, data, rec, lost, lost_r))
    errors = []
    threads = [threading.Thread(target=_run_coder, args=(coders[t], coder_cases[t], errors, f"coder{t}"))
               for t in range(2)]
    threads.append(threading.Thread(target=_run_encoder, args=(enc, enc_cases, errors)))
    threads.append(threading.Thread(target=_run_decoder, args=(dec, dec_cases, errors)))
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=300)
        assert not th.is_alive(), "a worker thread did not finish"
    assert not errors, errors[:10]
