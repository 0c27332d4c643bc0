"""Shred wire format: the oracle's wincode layout (CPU) and the
device serialize / deserialize batches against it (GPU).  Parity unpinned against wincode
itself (no serialized Shred bytes in the reference; see oracle/shred_wire_oracle.py)."""

import random
import struct

import numpy as np
import pytest

import shred_wire_oracle as wo


def _shred(rng, S=1024, height=6, kind=None):
    return (rng.choice([wo.DATA, wo.CODING]) if kind is None else kind, rng.getrandbits(64),
            rng.randrange(wo.MAX_SLICES_PER_BLOCK), bool(rng.getrandbits(1)), rng.randrange(wo.TOTAL_SHREDS),
            bytes(rng.getrandbits(8) for _ in range(S)), bytes(rng.getrandbits(8) for _ in range(64)),
            [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(height)])


def test_oracle_layout_and_size():
    rng = random.Random(1)
    sh = _shred(rng)
    b = wo.serialize(*sh)
    assert len(b) == 4 + 8 + 8 + 1 + 8 + 8 + 1024 + 64 + 8 + 6 * 32 == 1325  # fits MTU_BYTES
    assert len(b) <= wo.MTU_BYTES
    assert struct.unpack_from("<I", b, 0)[0] == sh[0]
    assert wo.deserialize(b) == sh


def malformed_variants(b: bytes):
    """(bytes, expected) mutations of one valid encoding: each breaks one decode rule."""
    out = []
    def put(off, fmt, v):
        x = bytearray(b)
        struct.pack_into(fmt, x, off, v)
        return bytes(x)
    out.append(put(0, "<I", 2))                 # unknown variant
    out.append(put(12, "<Q", 1024))             # slice_index >= MAX_SLICES_PER_BLOCK
    out.append(put(20, "<B", 2))                # bool not 0/1
    out.append(put(21, "<Q", 64))               # shred_index >= TOTAL_SHREDS
    out.append(put(29, "<Q", 1501))             # data length over the preallocation cap
    out.append(put(29, "<Q", len(b)))           # data length past the end
    out.append(b + b"\x00")                     # trailing byte
    out.append(b[:-1])                          # truncated proof
    out.append(b[:20])                          # truncated header
    out.append(b"")
    return out


def huge_proof_len_variants(b: bytes):
    """Proof lengths whose 32x product wraps in u64 (2^59 + h: 32 * that = 32 * h mod 2^64),
    so an unguarded exact-length check would accept them; wincode's MTU cap rejects them."""
    dlen = struct.unpack_from("<Q", b, 29)[0]
    off = 37 + dlen + 64
    h = struct.unpack_from("<Q", b, off)[0]
    out = []
    for v in (2**59 + h, 2**59, 2**63 + h, 2**64 - 1):
        x = bytearray(b)
        struct.pack_into("<Q", x, off, v)
        out.append(bytes(x))
    return out


def test_oracle_rejects_malformed():
    rng = random.Random(2)
    b = wo.serialize(*_shred(rng))
    for bad in malformed_variants(b):
        assert wo.deserialize(bad) is None
    for height in (0, 1, 6):
        for bad in huge_proof_len_variants(wo.serialize(*_shred(rng, height=height))):
            assert wo.deserialize(bad) is None
    # empty data, empty proof, kind/slice/shred at their maxima are fine
    edge = (wo.CODING, 2**64 - 1, 1023, True, 63, b"", bytes(64), [])
    assert wo.deserialize(wo.serialize(*edge)) == edge


# ---- device --------------------------------------------------------------------------------

def _cols(torch, rs, n, S_cap, H_cap, dev):
    t = dict(kind=torch.zeros(n, dtype=torch.uint8, device=dev), slot=torch.zeros(n, dtype=torch.int64, device=dev),
             slice_index=torch.zeros(n, dtype=torch.int64, device=dev),
             is_last=torch.zeros(n, dtype=torch.uint8, device=dev),
             shred_index=torch.zeros(n, dtype=torch.int32, device=dev),
             data=torch.zeros((n, max(S_cap, 1)), dtype=torch.uint8, device=dev),
             data_len=torch.zeros(n, dtype=torch.int32, device=dev),
             sig=torch.zeros((n, 64), dtype=torch.uint8, device=dev),
             proof=torch.zeros((n, max(32 * H_cap, 32)), dtype=torch.uint8, device=dev),
             height=torch.zeros(n, dtype=torch.int32, device=dev))
    c = rs.ShredColumns.of(t["kind"], t["slot"], t["slice_index"], t["is_last"], t["shred_index"], t["data"], S_cap,
                           t["data_len"], t["sig"], t["proof"], 32 * H_cap, t["height"])
    return t, c


@pytest.mark.gpu
@pytest.mark.parametrize("stride", [1500, 1501])  # odd rows: every packet alignment for the word copies
def test_gpu_serialize_matches_oracle(ctx, stride):
    import torch
    from alpenglow_amd import rs
    rng = random.Random(3)
    dev = "cuda:0"
    shreds = [_shred(rng, S=rng.choice([0, 1, 62, 1024]), height=rng.choice([0, 1, 6])) for _ in range(200)]
    n = len(shreds)
    t, c = _cols(torch, rs, n, 1024, 6, dev)
    t["kind"].copy_(torch.tensor([s[0] for s in shreds], dtype=torch.uint8))
    t["slot"].copy_(torch.tensor(np.array([s[1] for s in shreds], dtype=np.uint64).view(np.int64)))
    t["slice_index"].copy_(torch.tensor([s[2] for s in shreds], dtype=torch.int64))
    t["is_last"].copy_(torch.tensor([s[3] for s in shreds], dtype=torch.uint8))
    t["shred_index"].copy_(torch.tensor([s[4] for s in shreds], dtype=torch.int32))
    t["data_len"].copy_(torch.tensor([len(s[5]) for s in shreds], dtype=torch.int32))
    t["height"].copy_(torch.tensor([len(s[7]) for s in shreds], dtype=torch.int32))
    data = np.zeros((n, 1024), np.uint8)
    proof = np.zeros((n, 192), np.uint8)
    for i, s in enumerate(shreds):
        data[i, :len(s[5])] = np.frombuffer(s[5], np.uint8)
        pb = b"".join(s[7])
        proof[i, :len(pb)] = np.frombuffer(pb, np.uint8)
    t["data"].copy_(torch.from_numpy(data))
    t["proof"].copy_(torch.from_numpy(proof))
    t["sig"].copy_(torch.from_numpy(np.frombuffer(b"".join(s[6] for s in shreds), np.uint8).reshape(n, 64).copy()))
    packets = torch.full((n, stride), 0xAB, dtype=torch.uint8, device=dev)
    lens = torch.zeros(n, dtype=torch.int32, device=dev)
    rs.shred_serialize_batch(ctx, n, c, packets, stride, lens)
    ctx.synchronize()
    ph, lh = packets.cpu().numpy(), lens.cpu().numpy()
    for i, s in enumerate(shreds):
        want = wo.serialize(*s)
        assert lh[i] == len(want)
        assert ph[i, :lh[i]].tobytes() == want
        assert (ph[i, lh[i]:] == 0xAB).all()
    # a shred that does not fit the packet row: length 0, packet untouched
    small = torch.full((n, 100), 0xCD, dtype=torch.uint8, device=dev)
    rs.shred_serialize_batch(ctx, n, c, small, 100, lens)
    ctx.synchronize()
    for i, s in enumerate(shreds):
        if len(wo.serialize(*s)) > 100:
            assert lens[i].item() == 0 and (small[i] == 0xCD).all().item()


@pytest.mark.gpu
@pytest.mark.parametrize("stride", [1600, 1603])
def test_gpu_deserialize_matches_oracle(ctx, stride):
    import torch
    from alpenglow_amd import rs
    rng = random.Random(4)
    dev = "cuda:0"
    pkts = []
    for _ in range(60):
        b = wo.serialize(*_shred(rng, S=rng.choice([0, 5, 1024]), height=rng.choice([0, 6])))
        pkts.append(b)
        pkts.extend(malformed_variants(b)[:: rng.choice([1, 2, 3])])
        pkts.extend(huge_proof_len_variants(b))  # u64 wrap of 32 * proof_len (always included)
    big = wo.serialize(*_shred(rng, S=1024, height=10))   # valid, but wider than the proof rows
    pkts.append(big)
    n = len(pkts)
    buf = np.zeros((n, stride), np.uint8)
    for i, b in enumerate(pkts):
        buf[i, :len(b)] = np.frombuffer(b, np.uint8)
    packets = torch.from_numpy(buf).to(dev)
    lens = torch.tensor([len(b) for b in pkts], dtype=torch.int32, device=dev)
    t, c = _cols(torch, rs, n, 1024, 6, dev)
    status = torch.full((n,), 9, dtype=torch.uint8, device=dev)
    rs.shred_deserialize_batch(ctx, n, packets, stride, lens, c, status)
    ctx.synchronize()
    st = status.cpu().numpy()
    h = {k: v.cpu().numpy() for k, v in t.items()}
    n_ok = 0
    for i, b in enumerate(pkts):
        want = wo.deserialize(b)
        if want is None:
            assert st[i] == rs.WIRE_MALFORMED, i
            continue
        if len(want[7]) > 6:
            assert st[i] == rs.WIRE_TOO_LARGE
            continue
        assert st[i] == rs.WIRE_OK
        n_ok += 1
        kind, slot, si, last, idx, data, sig, proof = want
        assert h["kind"][i] == kind and h["slot"][i].astype(np.uint64) == slot and h["slice_index"][i] == si
        assert bool(h["is_last"][i]) == last and h["shred_index"][i] == idx
        assert h["data_len"][i] == len(data) and h["data"][i, :len(data)].tobytes() == data
        assert h["sig"][i].tobytes() == sig
        assert h["height"][i] == len(proof) and h["proof"][i, :32 * len(proof)].tobytes() == b"".join(proof)
    assert n_ok >= 60
