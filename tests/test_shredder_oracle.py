"""CPU tests of the composed-shredder oracle (oracle/shredder_oracle.py), the checker of
ag_shredder_deshred_batch: the receive side + Shredder::deshred (shredder.rs:282-311) round
trip an honest slice, and on a leader-signed non-codeword held with surplus shreds the
crate's decoder over every kept shred (reed_solomon.rs:154-166) and a decoder over any 32 of
them reach different errors -- the case the device must resolve like the crate."""

import random

import rs_oracle as o
import shredder_oracle as so
import slice_oracle as sl
import ed25519_oracle as ed

SEED = bytes(range(7, 39))
S = 1024


def _slice(rng):
    parent = (rng.randrange(1 << 40), bytes(rng.randrange(256) for _ in range(32)))
    data = bytes(rng.randrange(256) for _ in range(32 * S - 64 - sl.header_len(parent)))
    return parent, data, rng.randrange(1 << 32), rng.randrange(1024), False


def test_receive_deshred_roundtrip():
    rng = random.Random(3)
    parent, data, slot, si, last = _slice(rng)
    pkts, raw, root, sig = so.shred(parent, data, slot, si, last, SEED)
    keep = set(rng.sample(range(64), 33))
    rows = [pkts[j] if j in keep else None for j in range(64)]
    kept = so.receive(rows, ed.secret_to_public(SEED), S)
    assert [j for j in range(64) if kept[j] is not None] == sorted(keep)
    st, res = so.deshred(kept)
    assert st == so.OK and res["data"] == data and res["parent"] == parent
    assert res["datagrams"] == pkts and res["header"] == (slot, si, last)
    # a datagram signed by another key is not kept
    other = so.datagrams(raw.data, raw.coding, slot, si, last, bytes(range(100, 132)))[0]
    rows[min(keep)] = other[min(keep)]
    kept = so.receive(rows, ed.secret_to_public(SEED), S)
    assert kept[min(keep)] is None and sum(x is not None for x in kept) == 32


def test_exact_and_any_k_disagree_on_non_codeword():
    rng = random.Random(9)
    parent, data, slot, si, last = _slice(rng)
    raw = o.coder_shred(sl.payload_bytes(parent, data), 32)
    shards = list(raw.data) + list(raw.coding)
    shards[62] = bytes(x ^ 0x5A for x in shards[62])  # the leader signs a non-codeword
    pkts = so.datagrams(shards[:32], shards[32:], slot, si, last, SEED)[0]
    keep = set(range(16)) | set(range(32, 64))  # holds the odd shred, data 16..31 missing
    kept = so.receive([pkts[j] if j in keep else None for j in range(64)], ed.secret_to_public(SEED), S)
    st, _ = so.deshred(kept)
    assert st == so.BAD_ENCODING  # the crate's decoder (all 48 kept shreds): garbage padding
    # any 32 survivors (data 0..15, coding 32..47) restore the honest bytes: the padding
    # passes and the Merkle check fails instead
    any32 = [kept[j] if j < 48 else None for j in range(64)]
    st, _ = so.deshred(any32)
    assert st == so.INVALID_MERKLE_TREE


import pytest  # noqa: E402

import cipher_oracle as ci  # noqa: E402


@pytest.mark.parametrize("kind", [so.CODING_ONLY, so.PETS, so.AONT])
def test_other_shredders_roundtrip(kind):
    """CodingOnlyShredder / PetsShredder / AontShredder (shredder.rs:361-500): the output layout
    (0 / 31 / 32 data shreds first), the payload transform (PETS: ciphertext || key; AONT:
    ciphertext || key ^ SHA-256(ciphertext)), and the receive + deshred round trip from a random
    32 of the 64 datagrams; a receiver with the Regular layout rejects the datagrams of a
    shredder with another one."""
    rng = random.Random(40 + kind)
    Sk = 64
    parent = (rng.randrange(1 << 40), bytes(rng.randrange(256) for _ in range(32))) if kind != so.AONT else None
    extra = 16 if kind in (so.PETS, so.AONT) else 0
    data = bytes(rng.randrange(256) for _ in range(32 * Sk - 40 - extra - sl.header_len(parent)))
    key = bytes(rng.randrange(256) for _ in range(16))
    pkts, raw, root, sig = so.shred_kind(kind, parent, data, 77, 5, True, SEED, key)
    assert len(raw.data) == so.DATA_OUT[kind] and len(raw.data) + len(raw.coding) == 64
    payload = sl.payload_bytes(parent, data)
    if kind == so.PETS:
        enc = ci.pets_encrypt(payload, key)
        assert enc[-16:] == key and enc[:-16] != payload
    elif kind == so.AONT:
        enc = ci.aont_encrypt(payload, key)
        assert bytes(a ^ b for a, b in zip(enc[-16:], ci.sha256(enc[:-16]))) == key
    else:
        enc = payload
    full = o.coder_shred(enc, so.CODING[kind])
    assert raw.coding == full.coding and raw.data == full.data[:so.DATA_OUT[kind]]
    keep = set(rng.sample(range(64), 32))
    rows = [pkts[j] if j in keep else None for j in range(64)]
    pkb = ed.secret_to_public(SEED)
    kept = so.receive(rows, pkb, Sk, so.DATA_OUT[kind])
    assert [j for j in range(64) if kept[j] is not None] == sorted(keep)
    st, res = so.deshred_kind(kept, kind)
    assert st == so.OK and res["data"] == data and res["parent"] == parent
    assert res["datagrams"] == pkts and res["header"] == (77, 5, True)
    # the Regular receiver's layout check drops the shreds whose kind does not fit its slots
    wrong = so.receive(rows, pkb, Sk)
    mism = [j for j in keep if (j < 32) != (j < so.DATA_OUT[kind])]
    assert all(wrong[j] is None for j in mism)


def test_pets_aont_too_much_data_and_short_buffer():
    """MAX_DATA_SIZE is 16 bytes less for PETS / AONT (shredder.rs:409, 457); decrypt_payload of a
    buffer shorter than the key is BadEncoding (:517-521)."""
    data = bytes(32767 - 9 - 16 + 1)  # framed + 16 = 32768 > MAX_DATA_PER_SLICE
    for kind in (so.PETS, so.AONT):
        with pytest.raises(o.RSError):
            so.shred_kind(kind, None, data, 1, 0, False, SEED, bytes(16))
    so.shred_kind(so.PETS, None, data[:-1], 1, 0, False, SEED, bytes(16))  # fits exactly
    assert ci.decrypt_payload(bytes(15), True) is None and ci.decrypt_payload(bytes(15), False) is None
