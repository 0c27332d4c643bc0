"""AONT / PETS payload transforms: AES-128 known answers, the
oracle's CTR / SHA-256 / tail rules, and device parity through the C ABI.

Pins: AES-128 by FIPS-197 Appendix C.1 and NIST SP 800-38A F.1.1 (ECB-AES128) known-answer
vectors, on the oracle and on the library's tables; SHA-256 by hashlib.  The CTR flavour
(ctr::Ctr64LE, zero IV) is recalled, not pinned (oracle/cipher_oracle.py header).
"""

import random

import numpy as np
import pytest
import torch  # before the library: torch's HIP runtime must be the process's first

import cipher_oracle as co
import rs_oracle as o
from alpenglow_amd import rs

KAT = [  # (key, plaintext, ciphertext)
    ("000102030405060708090a0b0c0d0e0f", "00112233445566778899aabbccddeeff", "69c4e0d86a7b0430d8cdb78070b4c55a"),
    ("2b7e151628aed2a6abf7158809cf4f3c", "6bc1bee22e409f96e93d7e117393172a", "3ad77bb40d7a3660a89ecaf32466ef97"),
    ("2b7e151628aed2a6abf7158809cf4f3c", "ae2d8a571e03ac9c9eb76fac45af8e51", "f5d3d58503b9699de785895a96fdbaaf"),
    ("2b7e151628aed2a6abf7158809cf4f3c", "30c81c46a35ce411e5fbc1191a0a52ef", "43b1cd7f598ece23881b00e3ed030688"),
    ("2b7e151628aed2a6abf7158809cf4f3c", "f69f2445df4f9b17ad2b417be66c3710", "7b0c785e27e8ad3f8223207104725dd4"),
]


@pytest.mark.parametrize("key,pt,ct", KAT)
def test_aes_known_answers_oracle_and_library(key, pt, ct):
    k, p, c = bytes.fromhex(key), bytes.fromhex(pt), bytes.fromhex(ct)
    assert co.aes128_encrypt_block(k, p) == c
    assert rs.aes128_encrypt_block(k, p) == c


def test_oracle_ctr_and_transform_roundtrips():
    """crypto/cipher.rs roundtrip / random_keys_differ; shredder.rs decrypt_payload."""
    rng = random.Random(1)
    pt = b"some plaintext payload"
    k1, k2 = rng.randbytes(16), rng.randbytes(16)
    c1 = co.apply_keystream(k1, pt)
    assert c1 != pt and co.apply_keystream(k1, c1) == pt
    assert co.apply_keystream(k2, pt) != c1
    for n in (0, 1, 15, 16, 17, 100):
        payload = rng.randbytes(n)
        for aont in (True, False):
            enc = co.aont_encrypt(payload, k1) if aont else co.pets_encrypt(payload, k1)
            assert len(enc) == n + 16
            assert co.decrypt_payload(enc, aont) == payload
    assert co.decrypt_payload(b"short", True) is None


def _batch(rng, n, max_len, stride):
    lens = [rng.randint(0, max_len) for _ in range(n)]
    buf = np.frombuffer(o.splitmix64_bytes(rng.randrange(1 << 30), n * stride + 8), np.uint8)[: n * stride]
    return lens, buf.reshape(n, stride).copy()


@pytest.mark.gpu
@pytest.mark.parametrize("n,max_len,stride", [(9, 5000, 5008), (17, 33, 40), (5, 32767 + 16, 32784), (3, 16, 19)])
def test_device_keystream_and_sha256_match_oracle(ctx, n, max_len, stride):
    dev = torch.device("cuda:0")
    rng = random.Random(n + max_len)
    lens, host = _batch(rng, n, max_len, stride)
    keys = np.frombuffer(rng.randbytes(16 * n), np.uint8)
    d = torch.from_numpy(host.reshape(-1).copy()).to(dev)
    dk = torch.from_numpy(keys.copy()).to(dev)
    dig = torch.zeros(32 * n, dtype=torch.uint8, device=dev)
    rs.sha256_batch(ctx, n, d, stride, lens, dig)
    rs.cipher_apply_keystream_batch(ctx, n, dk, d, stride, lens)
    torch.cuda.synchronize()
    got, gd = d.cpu().numpy().reshape(n, stride), dig.cpu().numpy().reshape(n, 32)
    for b in range(n):
        L = lens[b]
        assert gd[b].tobytes() == co.sha256(host[b, :L].tobytes())
        assert got[b, :L].tobytes() == co.apply_keystream(keys[16 * b: 16 * b + 16].tobytes(), host[b, :L].tobytes())
        assert got[b, L:].tobytes() == host[b, L:].tobytes()  # nothing past the length


@pytest.mark.gpu
@pytest.mark.parametrize("scheme", [rs.AON_AONT, rs.AON_PETS])
def test_device_aon_encrypt_decrypt_match_oracle(ctx, scheme):
    dev = torch.device("cuda:0")
    rng = random.Random(7 + scheme)
    n, stride = 12, 32784
    lens = [rng.choice([0, 1, 15, 16, 100, 4095, 32751]) for _ in range(n)]
    host = np.zeros((n, stride), np.uint8)
    pays = [rng.randbytes(L) for L in lens]
    for b, p in enumerate(pays):
        host[b, : len(p)] = np.frombuffer(p, np.uint8)
    keys = np.frombuffer(rng.randbytes(16 * n), np.uint8)
    d = torch.from_numpy(host.reshape(-1).copy()).to(dev)
    rs.aon_encrypt_batch(ctx, scheme, n, torch.from_numpy(keys.copy()).to(dev), d, stride, lens)
    torch.cuda.synchronize()
    enc = d.cpu().numpy().reshape(n, stride)
    aont = scheme == rs.AON_AONT
    for b in range(n):
        k = keys[16 * b: 16 * b + 16].tobytes()
        want = co.aont_encrypt(pays[b], k) if aont else co.pets_encrypt(pays[b], k)
        assert enc[b, : lens[b] + 16].tobytes() == want
    out = rs.aon_decrypt_batch(ctx, scheme, n, d, stride, [L + 16 for L in lens])
    dec = d.cpu().numpy().reshape(n, stride)
    for b in range(n):
        assert out[b] == lens[b]
        assert dec[b, : lens[b]].tobytes() == pays[b]


@pytest.mark.gpu
def test_device_aon_decrypt_bad_encoding(ctx):
    dev = torch.device("cuda:0")
    d = torch.arange(3 * 64, dtype=torch.int32, device=dev).to(torch.uint8)
    before = d.cpu().numpy().copy()
    out = rs.aon_decrypt_batch(ctx, rs.AON_AONT, 3, d, 64, [5, 16, 40])
    assert out[0] == -23 and out[1] == 0 and out[2] == 24
    after = d.cpu().numpy()
    assert np.array_equal(after[:64], before[:64]) and np.array_equal(after[64:128], before[64:128])


@pytest.mark.gpu
@pytest.mark.parametrize("scheme,num_coding", [(rs.AON_AONT, 32), (rs.AON_PETS, 33)])
def test_aon_shredder_roundtrip_on_device(ctx, scheme, num_coding):
    """AontShredder / PetsShredder at the payload + RS level (shredder.rs:403-500): encrypt,
    shred (32 data + num_coding coding shreds of 1 KiB), lose shreds (PETS always loses the
    key-bearing last data shred), deshred, decrypt == payload; coding shreds == the oracle's."""
    dev = torch.device("cuda:0")
    rng = random.Random(11 + scheme)
    S, n = 1024, 5
    stride = (32 + num_coding) * S
    pays = [rng.randbytes(rng.randint(32 * S - 64 - 16, 32 * S - 1 - 16)) for _ in range(n)]
    cw = torch.zeros((n, stride), dtype=torch.uint8, device=dev)
    for b, p in enumerate(pays):
        cw[b, : len(p)] = torch.frombuffer(bytearray(p), dtype=torch.uint8).to(dev)
    keys = np.frombuffer(rng.randbytes(16 * n), np.uint8)
    lens = [len(p) for p in pays]
    rs.aon_encrypt_batch(ctx, scheme, n, torch.from_numpy(keys.copy()).to(dev), cw, stride, lens)
    rs.coder_shred_batch(ctx, num_coding, n, S, None, 0, [L + 16 for L in lens], cw, stride)
    host = cw.cpu().numpy()
    aont = scheme == rs.AON_AONT
    for b in range(n):
        k = keys[16 * b: 16 * b + 16].tobytes()
        enc = co.aont_encrypt(pays[b], k) if aont else co.pets_encrypt(pays[b], k)
        raw = o.coder_shred(enc, num_coding)
        assert host[b, 32 * S:].tobytes() == b"".join(raw.coding)
    dp, cp = [], []
    for b in range(n):
        lost = set(rng.sample(range(32 + num_coding), num_coding))
        if not aont:
            lost.add(31)
            lost.discard(next(iter(lost - {31})))
        dp += [0 if i in lost else 1 for i in range(32)]
        cp += [0 if 32 + j in lost else 1 for j in range(num_coding)]
        cw[b, : 32 * S].view(32, S)[[i for i in range(32) if i in lost]] = 0
    res = rs.coder_deshred_batch(ctx, num_coding, n, S, cw, stride, dp, cp, mode=rs.DECODE_ANY_K, as_array=True)
    assert all(res[b] == lens[b] + 16 for b in range(n)), res
    out = rs.aon_decrypt_batch(ctx, scheme, n, cw, stride, [int(r) for r in res])
    dec = cw.cpu().numpy()
    for b in range(n):
        assert out[b] == lens[b]
        assert dec[b, : lens[b]].tobytes() == pays[b]
