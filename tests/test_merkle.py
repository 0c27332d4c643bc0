"""Slice Merkle trees: oracle pins, library SHA-256 on the host,
and device parity (roots, nodes, proofs, proof checks) against oracle/merkle_oracle.py.

Pins: the 32 EMPTY_ROOTS digests the reference holds (crypto/merkle.rs:62-157,
tests/golden/merkle_empty_roots.json); the reference's own tree tests
(merkle.rs:477-660) restated on the oracle.
"""

import json
import os
import random

import numpy as np
import pytest
import torch  # before the library: torch's HIP runtime must be the process's first

import merkle_oracle as mo
import rs_oracle as o
from alpenglow_amd import rs

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "merkle_empty_roots.json")


@pytest.fixture(scope="module")
def empty_roots():
    return [bytes.fromhex(h) for h in json.load(open(GOLDEN))["empty_roots"]]


# ------------------------------------------------------------------ oracle and host pins

def test_oracle_empty_roots_match_reference(empty_roots):
    assert mo.EMPTY_ROOTS == empty_roots


def test_library_sha256_reproduces_empty_roots(empty_roots):
    """The library's SHA-256 and labels (host build of the kernel code), no GPU needed."""
    assert [rs.merkle_empty_root(h) for h in range(32)] == empty_roots


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 31, 32, 33, 63, 64])
def test_height_and_node_count(n):
    t = mo.MerkleTree([b"x"] * n)
    assert rs.merkle_height(n) == t.height()
    assert rs.merkle_node_count(n) == len(t.nodes)


def test_reference_tree_cases():
    """merkle.rs tests basic, two_leaves, empty_trees, proofs, three_leaves, non_power_of_two."""
    data = [b"hello", b"world"]
    t = mo.MerkleTree(data)
    assert len(t.nodes) == 3
    assert t.root() == mo.hash_pair(mo.hash_leaf(data[0]), mo.hash_leaf(data[1]))
    assert mo.MerkleTree([b""]).root() != mo.MerkleTree([b"", b""]).root()
    data = [b"hello", b"world", b"data", b"test"]
    t = mo.MerkleTree(data)
    for i in range(4):
        assert mo.check_proof(data[i], i, t.root(), t.create_proof(i))
    assert mo.MerkleTree([b"a", b"b", b"c"]).root() == mo.MerkleTree([b"a", b"b", b"c", b""]).root()
    assert mo.MerkleTree([b"hello"] * 33).root() == mo.MerkleTree([b"hello"] * 33 + [b""] * 31).root()


def test_reference_proof_last_cases():
    """merkle.rs tests proof_last, proof_last_overlong_is_rejected, ..._non_canonical_..."""
    data = [b"hello"] * 33
    t = mo.MerkleTree(data)
    root = t.root()
    assert not mo.check_proof_last(data[31], 31, root, t.create_proof(31))
    p32 = t.create_proof(32)
    assert mo.check_proof_last(data[32], 32, root, p32)
    assert not mo.check_proof_last(data[32], 32, root, [bytes(32)] * 33)
    bad = list(p32)
    bad[0] = bytes(32)
    assert not mo.check_proof_last(data[32], 32, root, bad)


def test_reference_fuzzing_reduced():
    """merkle.rs fuzzing (10k iterations there; 300 here)."""
    rng = random.Random(5)
    for _ in range(300):
        n = rng.randint(1, 64)
        data = [rng.randbytes(rng.randint(0, 64)) for _ in range(n)]
        t = mo.MerkleTree(data)
        for _ in range(10):
            i = rng.randrange(n)
            p = t.create_proof(i)
            assert mo.check_proof(data[i], i, t.root(), p)
            if i == n - 1:
                assert mo.check_proof_last(data[i], i, t.root(), p)


# ------------------------------------------------------------------------------- device

def _slices(seed, nslices, n, S, stride_pad=0):
    stride = S + stride_pad
    raw = np.frombuffer(o.splitmix64_bytes(seed, nslices * n * stride + 8), np.uint8)[: nslices * n * stride]
    return raw.reshape(nslices, n, stride)


def _device_build(ctx, arr, n, S, want_nodes=True, want_proofs=True):
    dev = torch.device("cuda:0")
    nslices, _, stride = arr.shape
    d = torch.from_numpy(np.ascontiguousarray(arr).reshape(-1).copy()).to(dev)
    h = rs.merkle_height(n)
    cnt = rs.merkle_node_count(n)
    roots = torch.zeros(nslices * 32, dtype=torch.uint8, device=dev)
    nstride = (32 * cnt + 15) // 16 * 16
    pstride = (32 * h * n + 15) // 16 * 16
    nodes = torch.zeros(nslices * nstride, dtype=torch.uint8, device=dev) if want_nodes else None
    proofs = torch.zeros(max(1, nslices * pstride), dtype=torch.uint8, device=dev) if want_proofs else None
    rs.merkle_build_batch(ctx, n, S, nslices, d, stride, n * stride, roots, nodes, nstride, proofs, pstride)
    torch.cuda.synchronize()
    out_r = roots.cpu().numpy().reshape(nslices, 32)
    out_n = nodes.cpu().numpy()[: nslices * nstride].reshape(nslices, nstride) if want_nodes else None
    out_p = proofs.cpu().numpy()[: nslices * pstride].reshape(nslices, pstride) if want_proofs and pstride else None
    return out_r, out_n, out_p, h, cnt


@pytest.mark.gpu
@pytest.mark.parametrize("n,S,nslices,pad", [(64, 1024, 9, 0), (64, 62, 5, 0), (64, 2, 3, 0), (64, 0, 2, 0),
                                             (64, 4096, 3, 0), (33, 100, 4, 4), (1, 64, 3, 0), (2, 5, 7, 3),
                                             (3, 1024, 5, 0), (63, 30, 6, 2), (64, 1000, 5, 24)])
def test_device_tree_matches_oracle(ctx, n, S, nslices, pad):
    """Roots, every node and every leaf's proof, bit-exact (aligned and unaligned leaves)."""
    arr = _slices(0xBEEF + n * 7 + S, nslices, n, S, pad)
    roots, nodes, proofs, h, cnt = _device_build(ctx, arr, n, S)
    for s in range(nslices):
        t = mo.MerkleTree([arr[s, j, :S].tobytes() for j in range(n)])
        assert roots[s].tobytes() == t.root()
        assert nodes[s, : 32 * cnt].tobytes() == b"".join(t.nodes)
        if h:
            for j in range(n):
                assert proofs[s, 32 * h * j: 32 * h * (j + 1)].tobytes() == b"".join(t.create_proof(j)), (s, j)


@pytest.mark.gpu
def test_device_empty_leaf_trees_give_empty_roots(ctx, empty_roots):
    """2^h empty leaves -> EMPTY_ROOTS[h] (merkle.rs empty_roots test), h <= 6."""
    for hh in range(7):
        n = 1 << hh
        roots, _, _, _, _ = _device_build(ctx, np.zeros((2, n, 16), np.uint8), n, 0, False, False)
        assert all(roots[s].tobytes() == empty_roots[hh] for s in range(2))


@pytest.mark.gpu
def test_device_verify_accepts_valid_and_rejects_tampered(ctx):
    dev = torch.device("cuda:0")
    n, S, nslices = 64, 1024, 4
    arr = _slices(77, nslices, n, S)
    roots, _, proofs, h, _ = _device_build(ctx, arr, n, S, want_nodes=False)
    rng = random.Random(3)
    items = [(s, j) for s in range(nslices) for j in range(n)]
    leaves = np.stack([arr[s, j] for s, j in items])
    idx = np.array([j for _, j in items], np.uint32)
    rts = np.stack([roots[s] for s, _ in items])
    prf = np.stack([proofs[s, 32 * h * j: 32 * h * (j + 1)] for s, j in items])
    expect = np.ones(len(items), np.uint8)
    for t in rng.sample(range(len(items)), 40):  # tamper: leaf byte, proof byte, index, root
        kind = t % 4
        if kind == 0:
            leaves[t, rng.randrange(S)] ^= 1
        elif kind == 1:
            prf[t, rng.randrange(32 * h)] ^= 0x80
        elif kind == 2:
            idx[t] ^= 1 << rng.randrange(h)
        else:
            rts[t, rng.randrange(32)] ^= 4
        expect[t] = 0
    td = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    ok = torch.zeros(len(items), dtype=torch.uint8, device=dev)
    rs.merkle_verify_batch(ctx, len(items), S, td(leaves), S, td(idx), td(rts), 32, td(prf), 32 * h, h, ok)
    got = ok.cpu().numpy()
    assert np.array_equal(got, expect)
    for t in range(0, len(items), 37):  # the oracle agrees item by item
        s, j = items[t]
        proof = [prf[t, 32 * q: 32 * (q + 1)].tobytes() for q in range(h)]
        assert mo.check_proof(leaves[t].tobytes(), int(idx[t]), rts[t].tobytes(), proof) == bool(got[t])


@pytest.mark.gpu
def test_slice_tree_over_device_shreds(ctx):
    """Shredder path end to end: coder_shred_batch codewords (32 data + 32 coding shreds)
    -> slice trees on the same buffer == oracle coder_shred + build_merkle_tree."""
    dev = torch.device("cuda:0")
    S, nslices = 1024, 6
    rng = random.Random(9)
    # every payload pads to shred size S (reed_solomon.rs:94-95): 32*S - 64 <= len < 32*S
    payloads = [rng.randbytes(rng.randint(32 * S - 64, 32 * S - 1)) for _ in range(nslices)]
    pay = torch.zeros((nslices, 32 * S), dtype=torch.uint8, device=dev)
    lens = []
    for i, p in enumerate(payloads):
        if p:
            pay[i, : len(p)] = torch.frombuffer(bytearray(p), dtype=torch.uint8).to(dev)
        lens.append(len(p))
    cw = torch.zeros((nslices, 64 * S), dtype=torch.uint8, device=dev)
    rs.coder_shred_batch(ctx, 32, nslices, S, pay, 32 * S, lens, cw, 64 * S)
    roots = torch.zeros(nslices * 32, dtype=torch.uint8, device=dev)
    rs.merkle_build_batch(ctx, 64, S, nslices, cw, S, 64 * S, roots)
    got = roots.cpu().numpy().reshape(nslices, 32)
    for i, p in enumerate(payloads):
        raw = o.coder_shred(p, 32)
        assert got[i].tobytes() == mo.slice_tree(raw.data, raw.coding).root()
