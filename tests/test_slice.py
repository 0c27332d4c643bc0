"""Slice payload framing: Slice::payload_bytes and
SlicePayload::try_from (/root/reference/src/types/slice.rs:73-84, :211-218).

CPU: the oracle restates the reference's own slice.rs tests (:267-332).  GPU: the device
framing feeds the batched coder (payload_bytes -> ReedSolomonCoder::shred, shredder.rs
337-345) and the device parser reads what the batched deshred leaves (shredder.rs:282-311),
both against the oracle, byte for byte.  wincode's byte rules are recalled (the crate is
not vendored): parity of the framing bytes is unpinned beyond the reference's tests and
its own comment (slice.rs:77).
"""

import random
import struct

import numpy as np
import pytest

import rs_oracle as o
import slice_oracle as so

GENESIS = (6, bytes(32))  # (Slot::new(6), GENESIS_BLOCK_HASH) as in slice.rs:283


# ----------------------------------------------------------------------- oracle (CPU)

def test_payload_roundtrip():                       # slice.rs:267-272
    b = so.payload_bytes(None, bytes([1, 2, 3, 4]))
    assert so.try_from(b) == (so.OK, None, bytes([1, 2, 3, 4]))


def test_payload_bytes_layout():                    # slice.rs:274-288 (both parents)
    assert so.payload_bytes(None, b"\x01\x02\x03\x04\x05") == b"\x00" + struct.pack("<Q", 5) + b"\x01\x02\x03\x04\x05"
    b = so.payload_bytes(GENESIS, b"abc")
    assert b == b"\x01" + struct.pack("<Q", 6) + bytes(32) + struct.pack("<Q", 3) + b"abc"
    assert so.try_from(b) == (so.OK, GENESIS, b"abc")
    assert so.header_len(None) == 9 and so.header_len(GENESIS) == 49


def test_trailing_bytes_are_rejected():             # slice.rs:290-299
    assert so.try_from(so.payload_bytes(None, bytes([1, 2, 3, 4])) + b"\xaa")[0] == so.BAD_ENCODING


def test_malformed_payload_returns_error():         # slice.rs:301-308
    assert so.try_from(b"\xff" * 4)[0] == so.BAD_ENCODING


def test_oversized_payload_returns_error():         # slice.rs:310-319
    assert so.try_from(bytes(so.MAX_DATA_PER_SLICE + 1))[0] == so.TOO_LARGE


def test_inflated_length_prefix_is_rejected():      # slice.rs:321-332
    b = bytearray(so.payload_bytes(None, b""))
    b[-8:] = struct.pack("<Q", 2**64 - 1)
    assert so.try_from(bytes(b))[0] == so.BAD_ENCODING


def malformed_payloads():
    """(bytes, expected status) covering every decode rule."""
    good = so.payload_bytes(GENESIS, b"hello world")
    cases = [(b"", so.BAD_ENCODING), (b"\x02" + good[1:], so.BAD_ENCODING), (good[:30], so.BAD_ENCODING),
             (good[:49], so.BAD_ENCODING), (good[:-1], so.BAD_ENCODING), (good + b"\x00", so.BAD_ENCODING),
             (b"\x00" + struct.pack("<Q", 40000) + bytes(10), so.BAD_ENCODING),
             (b"\x00" + struct.pack("<Q", 2**63 + 10) + bytes(10), so.BAD_ENCODING),
             (bytes(so.MAX_DATA_PER_SLICE + 1), so.TOO_LARGE),
             (b"\x00" + struct.pack("<Q", so.MAX_DATA_PER_SLICE - 9) + bytes(so.MAX_DATA_PER_SLICE - 9), so.OK),
             (b"\x00" + struct.pack("<Q", 0), so.OK)]
    return cases


def test_oracle_decode_rules():
    for b, want in malformed_payloads():
        assert so.try_from(b)[0] == want, b[:16]


# ------------------------------------------------------------------------- device (GPU)

def _framed_lens(rng, S, n, parent_bytes):
    """Data lengths whose framed payload maps to shred size S (reed_solomon.rs:94-95)."""
    lo = max(0, 32 * S - 64)
    return [rng.randrange(lo, 32 * S) - parent_bytes[b] for b in range(n)]


@pytest.mark.gpu
@pytest.mark.parametrize("S,n", [(1024, 37), (96, 20), (2, 3)])
def test_gpu_frame_shred_matches_oracle(ctx, S, n):
    """payload_bytes -> ReedSolomonCoder::shred on the device, against the oracle's
    coder_shred(payload_bytes(...)): data shreds (framing + padding) and coding shreds."""
    import torch
    from alpenglow_amd import rs
    dev = "cuda:0"
    rng = random.Random(S * 3 + n)
    parents = [None if rng.random() < 0.5 else (rng.getrandbits(64), rng.randbytes(32)) for _ in range(n)]
    hb = [so.header_len(p) for p in parents]
    lens = _framed_lens(rng, S, n, hb)
    if S == 2:  # 64-byte padded payloads only hold empty data with no parent
        parents, hb, lens = [None] * n, [9] * n, [0] * n
    datas = [rng.randbytes(max(L, 0)) for L in lens]
    stride_d = max(16, (max(lens) + 15) // 16 * 16)
    dbuf = np.zeros((n, stride_d), np.uint8)
    for b, d in enumerate(datas):
        dbuf[b, :len(d)] = np.frombuffer(d, np.uint8)
    m = 32
    stride = (32 + m) * S
    d_data = torch.from_numpy(dbuf).to(dev)
    d_cw = torch.full((n, stride), 0xEE, dtype=torch.uint8, device=dev)
    plens = rs.slice_frame_batch(ctx, n, S, parents, d_data, stride_d, [len(d) for d in datas], d_cw, stride)
    rs.coder_shred_batch(ctx, m, n, S, None, 0, plens, d_cw, stride)
    host = d_cw.cpu().numpy()
    for b in range(n):
        payload = so.payload_bytes(parents[b], datas[b])
        assert plens[b] == len(payload)
        raw = o.coder_shred(payload, m)
        assert host[b, :32 * S].tobytes() == b"".join(raw.data), b
        assert host[b, 32 * S:].tobytes() == b"".join(raw.coding), b


@pytest.mark.gpu
def test_gpu_frame_rejects_oversized(ctx):
    import torch
    from alpenglow_amd import rs
    d_cw = torch.zeros((2, 64 * 1024), dtype=torch.uint8, device="cuda:0")
    d_data = torch.zeros((2, 32768), dtype=torch.uint8, device="cuda:0")
    for S, lens, par in [(1024, [10, 32767 - 8], [None, None]), (1024, [10, 32767 - 48], [None, GENESIS]),
                         (64, [2000, 2048 - 9], [None, None])]:
        with pytest.raises(rs.RSError) as e:
            rs.slice_frame_batch(ctx, 2, S, par, d_data, 32768, lens, d_cw, 64 * 1024)
        assert e.value.kind == "TooMuchData"


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
def test_gpu_deshred_parse_matches_oracle(ctx, mode):
    """Shredder::deshred's tail: the batched deshred (random losses per slice) leaves the
    payload in the codeword; SlicePayload::try_from on the device gives the oracle's parent
    and data (in place), NoPayload for failed slices, and the oracle's verdicts on
    malformed payloads that are still validly padded and encoded."""
    import torch
    from alpenglow_amd import rs
    dev = "cuda:0"
    rng = random.Random(11 + mode)
    S, m, n = 1024, 32, 24
    stride = (32 + m) * S
    payloads = [b for b, _ in malformed_payloads() if len(b) <= so.MAX_DATA_PER_SLICE]
    while len(payloads) < n:
        par = None if len(payloads) % 2 else (rng.getrandbits(64), rng.randbytes(32))
        L = rng.randrange(32 * S - 64, 32 * S) - so.header_len(par)
        payloads.append(so.payload_bytes(par, rng.randbytes(L)))
    # the batch coder takes one shred size per call: group the slices by their S
    sizes = {b: -(-(len(p) + 64 - len(p) % 64) // 32) for b, p in enumerate(payloads)}
    keep = [b for b in range(n) if sizes[b] == S]
    short = [b for b in range(n) if sizes[b] != S]
    results = {}
    for group, Sg in [(keep, S)] + [([b], sizes[b]) for b in short]:
        ng = len(group)
        strideg = (32 + m) * Sg
        cw = np.zeros((ng, strideg), np.uint8)
        dp, cp = [], []
        for gi, b in enumerate(group):
            raw = o.coder_shred(payloads[b], m)
            cw[gi] = np.frombuffer(b"".join(raw.data) + b"".join(raw.coding), np.uint8)
            lost = set(rng.sample(range(64), 33 if gi % 5 == 4 else 32))  # every 5th: NotEnoughShreds
            dp += [0 if i in lost else 1 for i in range(32)]
            cp += [0 if 32 + j in lost else 1 for j in range(m)]
            for i in lost:
                cw[gi, i * Sg:(i + 1) * Sg] = 0
        d_cw = torch.from_numpy(cw).to(dev)
        plens = rs.coder_deshred_batch(ctx, m, ng, Sg, d_cw, strideg, dp, cp, mode=mode, as_array=True)
        st, parents, offs, dls = rs.slice_parse_batch(ctx, ng, d_cw, strideg, plens)
        host = d_cw.cpu().numpy()
        for gi, b in enumerate(group):
            results[b] = (plens[gi], st[gi], parents[gi], host[gi, offs[gi]:offs[gi] + dls[gi]].tobytes())
    for b in range(n):
        plen, st, par, data = results[b]
        if plen < 0:
            assert st == rs.SLICE_NO_PAYLOAD
            continue
        wst, wpar, wdata = so.try_from(payloads[b])
        assert st == wst, b
        if wst == so.OK:
            assert par == wpar and data == wdata, b


def test_parent_arrays_round_trip():
    """The binding's parent conversion (rs._parent_arrays / rs._parent_list): None entries stay
    None, set entries keep slot and hash, and any sequence type is accepted (host logic only)."""
    from alpenglow_amd import rs

    h1, h2 = bytes(range(32)), bytes(range(100, 132))
    parents = [None, (7, h1), None, None, ((1 << 64) - 1, h2)]
    for seq in (parents, tuple(parents), iter(parents)):
        flags, ids = rs._parent_arrays(seq, len(parents))
        assert flags.tolist() == [0, 1, 0, 0, 1]
        assert rs._parent_list(flags, ids) == parents
    flags, ids = rs._parent_arrays([None] * 4, 4)
    assert not flags.any() and not ids.any()
    assert rs._parent_list(flags, ids) == [None] * 4
    with pytest.raises(ValueError):
        rs._parent_arrays([None] * 3, 4)
