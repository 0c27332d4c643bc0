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
