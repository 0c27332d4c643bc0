"""Ed25519 shred signatures: oracle pins, the kernels' arithmetic
run on the host against the oracle (CPU), and the device batches vs the oracle (GPU).

Pins: RFC 8032 §7.1 TESTs 1-3 (tests/golden/ed25519_rfc8032.json).  The ZIP-215 verdicts
for malformed encodings (small-order / non-canonical points, s >= l) follow the published
rules of ed25519-zebra 4.2.0 restated in oracle/ed25519_oracle.py -- parity unpinned
against the crate itself (not vendored, not buildable here)."""

import json
import os
import random
import subprocess

import numpy as np
import pytest

import ed25519_oracle as eo
import merkle_oracle as mo
from ed_cases import le, verify_cases

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden", "ed25519_rfc8032.json")
CSRC = os.path.join(ROOT, "alpenglow_amd", "csrc")
HOSTCHK_SRC = os.path.join(ROOT, "tests", "native", "ed_host_check.cpp")
HOSTCHK = os.path.join(ROOT, "tests", "native", "_build", "ed_host_check")


def rfc_vectors():
    with open(GOLD) as f:
        return json.load(f)["vectors"]


# ---- oracle pins (CPU) -------------------------------------------------------------------

@pytest.mark.parametrize("v", rfc_vectors(), ids=lambda v: v["name"])
def test_oracle_rfc8032(v):
    sk, pk, msg, sig = (bytes.fromhex(v[k]) for k in ("secret", "public", "message", "signature"))
    assert eo.secret_to_public(sk) == pk
    assert eo.sign(sk, msg) == sig
    assert eo.verify(pk, msg, sig)
    assert not eo.verify(pk, msg + b"\x00", sig)


def test_oracle_group_laws():
    B = eo.B
    assert eo.is_identity(eo.scalar_mult(eo.L, B))                  # B has order l
    assert eo.compress(B).hex() == "58" + "66" * 31                 # RFC 8032 base point encoding
    a, b = 12345678901234567890, 98765432109876543210
    lhs = eo.scalar_mult(a + b, B)
    rhs = eo.point_add(eo.scalar_mult(a, B), eo.scalar_mult(b, B))
    assert eo.point_equal(lhs, rhs)
    assert len(eo.small_order_encodings()) == 8
    for enc in eo.small_order_encodings():
        assert eo.is_identity(eo.scalar_mult(8, eo.decompress(enc)))


def test_oracle_zip215_rules():
    ident = le(1)
    assert eo.verify(ident, b"m", ident + le(0))                    # small order, cofactored
    assert eo.verify(le(eo.P + 1), b"m", ident + le(0))             # non-canonical y accepted
    assert eo.verify(le(1 | 1 << 255), b"m", ident + le(0))         # negative zero accepted
    assert not eo.verify(ident, b"m", ident + le(eo.L))             # s >= l rejected
    sk = bytes(range(32))
    sig = eo.sign(sk, b"m")
    assert eo.verify(eo.secret_to_public(sk), b"m", sig)


def test_oracle_validate_shred_rules():
    sk = bytes(range(32))
    pk = eo.secret_to_public(sk)
    c1 = eo.slice_commitment(5, 2, False, bytes(32))
    c2 = eo.slice_commitment(5, 3, False, bytes(32))
    s1 = eo.sign(sk, c1)
    assert eo.validate_shred(c1, s1, pk, None) == eo.OK
    assert eo.validate_shred(c1, s1, eo.secret_to_public(bytes(32)), None) == eo.INVALID_SIGNATURE
    assert eo.validate_shred(c1, bytes(64), pk, c1) == eo.OK                   # cache hit: no check
    assert eo.validate_shred(c1, s1, pk, c2) == eo.EQUIVOCATION
    assert eo.validate_shred(c1, bytes(64), pk, c2) == eo.INVALID_SIGNATURE
    assert len(c1) == eo.SLICE_COMMITMENT_LEN == 49


# ---- the kernels' arithmetic on the host (CPU) --------------------------------------------

@pytest.fixture(scope="module")
def hostchk():
    srcs = [HOSTCHK_SRC, os.path.join(CSRC, "ed25519_core.hpp")]
    if not os.path.exists(HOSTCHK) or os.path.getmtime(HOSTCHK) < max(os.path.getmtime(s) for s in srcs):
        os.makedirs(os.path.dirname(HOSTCHK), exist_ok=True)
        subprocess.run(["hipcc", "--offload-host-only", "-O1", "-std=c++20", f"-I{CSRC}", HOSTCHK_SRC, "-o", HOSTCHK],
                       check=True, capture_output=True)

    def run(lines):
        out = subprocess.run([HOSTCHK], input="\n".join(lines) + "\n", capture_output=True, text=True, check=True)
        return out.stdout.split()
    return run


def _h(b: bytes) -> str:
    return b.hex() if b else "-"


def test_host_core_rfc8032(hostchk):
    vs = rfc_vectors()
    lines = []
    for v in vs:
        lines += [f"pk {v['secret']}", f"sign {v['secret']} {v['message'] or '-'}",
                  f"verify {v['public']} {v['message'] or '-'} {v['signature']}"]
    out = hostchk(lines)
    for i, v in enumerate(vs):
        assert out[3 * i] == v["public"]
        assert out[3 * i + 1] == v["signature"]
        assert out[3 * i + 2] == "1"


def test_host_core_sign_random(hostchk):
    rng = random.Random(3)
    seeds = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(12)]
    msgs = [bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 49, 77, 111, 112, 239, 300]))) for _ in seeds]
    out = hostchk([f"sign {s.hex()} {_h(m)}" for s, m in zip(seeds, msgs)] + [f"pk {s.hex()}" for s in seeds])
    for i, (s, m) in enumerate(zip(seeds, msgs)):
        assert out[i] == eo.sign(s, m).hex()
        assert out[len(seeds) + i] == eo.secret_to_public(s).hex()


def test_host_core_verify_cases(hostchk):
    cases = verify_cases(n_random=12)
    out = hostchk([f"verify {pk.hex()} {_h(m)} {sig.hex()}" for pk, m, sig in cases])
    want = ["1" if eo.verify(pk, m, sig) else "0" for pk, m, sig in cases]
    assert out == want
    assert "1" in want and "0" in want


# ---- device batches (GPU) ----------------------------------------------------------------

def _dev(b: bytes):
    import torch
    return torch.tensor(list(b), dtype=torch.uint8, device="cuda:0")


def _cat(items):
    return _dev(b"".join(items))


@pytest.mark.gpu
def test_gpu_public_key_and_sign_rfc8032(ctx):
    from alpenglow_amd import rs
    vs = rfc_vectors()
    seeds = _cat([bytes.fromhex(v["secret"]) for v in vs])
    pks = _dev(bytes(32 * len(vs)))
    rs.ed25519_public_key_batch(ctx, len(vs), seeds, pks)
    ctx.synchronize()
    got = pks.cpu().numpy().tobytes()
    for i, v in enumerate(vs):
        assert got[32 * i:32 * i + 32].hex() == v["public"]
    # one message length per call: sign each vector on its own
    for i, v in enumerate(vs):
        msg = bytes.fromhex(v["message"])
        sig = _dev(bytes(64))
        rs.ed25519_sign_batch(ctx, 1, seeds[32 * i:], 32, pks[32 * i:], 32, _dev(msg) if msg else None, 0,
                              len(msg), sig)
        ctx.synchronize()
        assert sig.cpu().numpy().tobytes().hex() == v["signature"]


@pytest.mark.gpu
def test_gpu_sign_batch_vs_oracle(ctx):
    from alpenglow_amd import rs
    rng = random.Random(11)
    n, mlen = 300, 49
    seeds_b = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(n)]
    msgs_b = [bytes(rng.getrandbits(8) for _ in range(mlen)) for _ in range(n)]
    seeds, msgs = _cat(seeds_b), _cat(msgs_b)
    pks = _dev(bytes(32 * n))
    sigs = _dev(bytes(64 * n))
    rs.ed25519_public_key_batch(ctx, n, seeds, pks)
    rs.ed25519_sign_batch(ctx, n, seeds, 32, pks, 32, msgs, mlen, mlen, sigs)
    ctx.synchronize()
    got_pk = pks.cpu().numpy().tobytes()
    got = sigs.cpu().numpy().tobytes()
    for t in range(0, n, 7):  # oracle is slow: every 7th
        assert got_pk[32 * t:32 * t + 32] == eo.secret_to_public(seeds_b[t])
        assert got[64 * t:64 * t + 64] == eo.sign(seeds_b[t], msgs_b[t])


@pytest.mark.gpu
def test_gpu_verify_batch_vs_oracle(ctx):
    import torch
    from alpenglow_amd import rs
    cases = verify_cases(n_random=40)
    n = len(cases)
    stride = max(len(m) for _, m, _ in cases)
    msgs = bytearray(stride * n)
    for t, (_, m, _) in enumerate(cases):
        msgs[stride * t:stride * t + len(m)] = m
    lens = torch.tensor([len(m) for _, m, _ in cases], dtype=torch.int32, device="cuda:0")
    ok = torch.full((n,), 7, dtype=torch.uint8, device="cuda:0")
    rs.ed25519_verify_batch(ctx, n, _cat([pk for pk, _, _ in cases]), 32, _dev(bytes(msgs)), stride,
                            _cat([s for _, _, s in cases]), 64, ok, msg_lens=lens)
    ctx.synchronize()
    got = ok.cpu().numpy().tolist()
    want = [1 if eo.verify(pk, m, s) else 0 for pk, m, s in cases]
    assert got == want
    assert sum(want) > 20 and want.count(0) > 20


@pytest.mark.gpu
def test_gpu_verify_shared_key_large_batch(ctx):
    """One leader key, many commitments (the receive path's shape); every 97th tampered."""
    import torch
    from alpenglow_amd import rs
    rng = random.Random(5)
    sk = bytes(rng.getrandbits(8) for _ in range(32))
    n = 4096
    msgs = torch.randint(0, 256, (n, 49), dtype=torch.uint8, device="cuda:0")
    seeds = _dev(sk)
    pk = _dev(bytes(32))
    rs.ed25519_public_key_batch(ctx, 1, seeds, pk)
    sigs = torch.zeros((n, 64), dtype=torch.uint8, device="cuda:0")
    rs.ed25519_sign_batch(ctx, n, seeds, 0, pk, 0, msgs, 49, 49, sigs)
    sigs[::97, 40] ^= 1
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda:0")
    rs.ed25519_verify_batch(ctx, n, pk, 0, msgs, 49, sigs, 64, ok, msg_len=49)
    ctx.synchronize()
    want = np.ones(n, np.uint8)
    want[::97] = 0
    assert np.array_equal(ok.cpu().numpy(), want)
    mh, sh = msgs.cpu().numpy(), sigs.cpu().numpy()
    pkb = pk.cpu().numpy().tobytes()
    assert pkb == eo.secret_to_public(sk)
    for t in (0, 1, 97, 1000, n - 1):
        assert eo.verify(pkb, mh[t].tobytes(), sh[t].tobytes()) == bool(want[t])


def _make_slice(rng, sk, slot, slice_index, is_last, shred_bytes=1024, n_leaves=64):
    """64 shreds of one slice with their Merkle proofs, root and the leader's signature."""
    leaves = [bytes(rng.getrandbits(8) for _ in range(shred_bytes)) for _ in range(n_leaves)]
    tree = mo.MerkleTree(leaves)
    root = tree.root()
    commit = eo.slice_commitment(slot, slice_index, is_last, root)
    sig = eo.sign(sk, commit)
    proofs = [b"".join(tree.create_proof(i)) for i in range(n_leaves)]
    return leaves, proofs, root, commit, sig


@pytest.mark.gpu
def test_gpu_shred_validate_batch(ctx):
    """ValidatedShred::try_new over shreds of two slices: valid, cache hit, equivocation,
    wrong key, tampered header / payload / proof / signature (validated_shred.rs tests)."""
    import torch
    from alpenglow_amd import rs
    rng = random.Random(9)
    sk = bytes(rng.getrandbits(8) for _ in range(32))
    pk = eo.secret_to_public(sk)
    other_pk = eo.secret_to_public(bytes(32))
    S = 1024
    la, pa, ra, ca, sa = _make_slice(rng, sk, 10, 0, False, S)
    lb, pb, rb, cb, sb = _make_slice(rng, sk, 10, 1, True, S)
    height = len(pa[0]) // 32
    rows = []  # (leaf, proof, index, slot, slice, is_last, sig, cached, key, expected)
    for i in range(64):
        rows.append((la[i], pa[i], i, 10, 0, 0, sa, None, pk, eo.OK))
    for i in range(0, 64, 3):
        rows.append((lb[i], pb[i], i, 10, 1, 1, sb, cb, pk, eo.OK))            # cache hit
        rows.append((lb[i], pb[i], i, 10, 1, 1, sb, ca, pk, eo.EQUIVOCATION))  # valid, other commitment
    rows.append((la[5], pa[5], 5, 10, 0, 0, sa, None, other_pk, eo.INVALID_SIGNATURE))
    rows.append((la[5], pa[5], 5, 11, 0, 0, sa, None, pk, eo.INVALID_SIGNATURE))     # cross-slot
    rows.append((la[5], pa[5], 5, 10, 1, 0, sa, None, pk, eo.INVALID_SIGNATURE))     # cross-slice
    rows.append((la[5], pa[5], 5, 10, 0, 1, sa, None, pk, eo.INVALID_SIGNATURE))     # is_last flip
    rows.append((la[5], pa[5], 5, 10, 0, 1, sa, ca, pk, eo.INVALID_SIGNATURE))       # ... with a cache
    bad = bytearray(la[6]); bad[100] ^= 4
    rows.append((bytes(bad), pa[6], 6, 10, 0, 0, sa, None, pk, eo.INVALID_SIGNATURE))
    rows.append((la[6], pa[6], 7, 10, 0, 0, sa, None, pk, eo.INVALID_SIGNATURE))     # wrong index
    badsig = bytearray(sa); badsig[3] ^= 1
    rows.append((la[7], pa[7], 7, 10, 0, 0, bytes(badsig), None, pk, eo.INVALID_SIGNATURE))
    rows.append((la[7], pa[7], 7, 10, 0, 0, bytes(badsig), ca, pk, eo.OK))           # cache hit skips it
    # one pk per call: split rows by key
    for key in (pk, other_pk):
        sel = [r for r in rows if r[8] == key]
        n = len(sel)
        # the oracle's own verdicts agree with the expectations
        for r in sel:
            commit = eo.slice_commitment(r[3], r[4], bool(r[5]), mo.derive_root(r[0], r[2], [
                r[1][32 * h:32 * h + 32] for h in range(height)]))
            assert eo.validate_shred(commit, r[6], key, r[7]) == r[9]
        data = _cat([r[0] for r in sel])
        proofs = _cat([r[1] for r in sel])
        idx = torch.tensor([r[2] for r in sel], dtype=torch.int32, device="cuda:0")
        slots = torch.tensor([r[3] for r in sel], dtype=torch.int64, device="cuda:0")
        slices = torch.tensor([r[4] for r in sel], dtype=torch.int64, device="cuda:0")
        last = torch.tensor([r[5] for r in sel], dtype=torch.uint8, device="cuda:0")
        sigs = _cat([r[6] for r in sel])
        cached = _cat([r[7] if r[7] is not None else bytes(49) for r in sel])
        has = torch.tensor([r[7] is not None for r in sel], dtype=torch.uint8, device="cuda:0")
        status = torch.full((n,), 9, dtype=torch.uint8, device="cuda:0")
        roots = torch.zeros((n, 32), dtype=torch.uint8, device="cuda:0")
        rs.shred_validate_batch(ctx, n, data, S, S, idx, proofs, 32 * height, height, slots, slices, last, sigs,
                                64, _dev(key), status, cached=cached, has_cached=has, roots_out=roots)
        ctx.synchronize()
        assert status.cpu().numpy().tolist() == [r[9] for r in sel]
        rr = roots.cpu().numpy()
        for t, r in enumerate(sel):
            want_root = mo.derive_root(r[0], r[2], [r[1][32 * h:32 * h + 32] for h in range(height)])
            assert rr[t].tobytes() == want_root


@pytest.mark.gpu
def test_gpu_slice_sign_batch(ctx):
    import torch
    from alpenglow_amd import rs
    rng = random.Random(13)
    sk = bytes(rng.getrandbits(8) for _ in range(32))
    n = 64
    roots_b = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(n)]
    slots = [rng.getrandbits(40) for _ in range(n)]
    slices = [rng.getrandbits(20) for _ in range(n)]
    last = [rng.getrandbits(1) for _ in range(n)]
    seed = _dev(sk)
    pk = _dev(bytes(32))
    rs.ed25519_public_key_batch(ctx, 1, seed, pk)
    sigs = torch.zeros((n, 64), dtype=torch.uint8, device="cuda:0")
    commits = torch.zeros((n, 49), dtype=torch.uint8, device="cuda:0")
    rs.slice_sign_batch(ctx, n, seed, pk, torch.tensor(slots, dtype=torch.int64, device="cuda:0"),
                        torch.tensor(slices, dtype=torch.int64, device="cuda:0"),
                        torch.tensor(last, dtype=torch.uint8, device="cuda:0"), _cat(roots_b), sigs, commits)
    ctx.synchronize()
    sh, ch = sigs.cpu().numpy(), commits.cpu().numpy()
    for t in range(0, n, 5):
        c = eo.slice_commitment(slots[t], slices[t], bool(last[t]), roots_b[t])
        assert ch[t].tobytes() == c
        assert sh[t].tobytes() == eo.sign(sk, c)
