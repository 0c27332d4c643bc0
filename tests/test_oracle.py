"""CPU tests: the oracle against its mathematical pins, the golden fixtures and the
behaviours the reference's own tests pin (reed_solomon.rs:244-347, shredder.rs:655-869).

The oracle restates reed-solomon-simd 3.1.0; parity against the crate itself is unpinned
(no known-answer vectors exist in the reference and the crate cannot be built here).
"""

import hashlib
import os
import random

import numpy as np
import pytest

import ro_c
import rs_oracle as o

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def sha(b):
    return hashlib.sha256(b).hexdigest()


# ---------------------------------------------------------------------------- field pins

def test_tables_match_golden(golden):
    exp, log, skew, lw = o.tables()
    t = golden["tables"]
    assert sha(exp.astype("<u2").tobytes()) == t["exp_sha256"]
    assert sha(log.astype("<u2").tobytes()) == t["log_sha256"]
    assert sha(skew.astype("<u2").tobytes()) == t["skew_sha256"]
    assert sha(lw.astype("<u2").tobytes()) == t["log_walsh_sha256"]


def test_c_oracle_tables_equal_python():
    a = o.tables()
    b = ro_c.tables()
    for x, y in zip(a, b):
        assert np.array_equal(x.astype(np.uint16), y)


def test_polynomial_is_primitive_and_tables_are_inverse():
    exp, log, _, _ = o.tables()
    # log is a bijection from nonzero elements onto 0..65534 (0x1002D primitive)
    assert sorted(log[1:].tolist()) == list(range(65535))
    x = np.arange(1, 65536)
    assert np.array_equal(exp[log[x]], x)


def gf_mul(a, b):
    exp, log, _, _ = o.tables()
    if a == 0 or b == 0:
        return 0
    s = int(log[a]) + int(log[b])
    return int(exp[(s + (s >> 16)) & 0xFFFF])


def gf_inv(a):
    exp, log, _, _ = o.tables()
    return int(exp[(65535 - int(log[a])) % 65535])


def test_cantor_basis_recurrence():
    # In Cantor coordinates beta_i = 1 << i and beta_i^2 + beta_i = beta_{i-1}.
    for i in range(1, 16):
        b = 1 << i
        assert gf_mul(b, b) ^ b == 1 << (i - 1)
    assert gf_mul(1, 1) == 1


def lagrange_eval(xs, ys, x):
    acc = 0
    for i, (xi, yi) in enumerate(zip(xs, ys)):
        num, den = 1, 1
        for j, xj in enumerate(xs):
            if j != i:
                num = gf_mul(num, x ^ xj)
                den = gf_mul(den, xi ^ xj)
        acc ^= gf_mul(yi, gf_mul(num, gf_inv(den)))
    return acc


def test_highrate_encode_is_lagrange_interpolation():
    """32:32 HighRate: parity j = P(omega_j) where P interpolates data i at omega_{32+i}
    and omega_x = x (Cantor basis)."""
    rng = np.random.default_rng(7)
    data = rng.integers(0, 65536, size=32, dtype=np.int64)
    shards = [bytes([int(v) & 0xFF, int(v) >> 8]) for v in data]  # S = 2: one symbol
    rec = o.encode(shards, 32)
    xs = [32 + i for i in range(32)]
    for j in range(32):
        want = lagrange_eval(xs, [int(v) for v in data], j)
        got = rec[j][0] | (rec[j][1] << 8)
        assert got == want


@pytest.mark.parametrize("k,m", [(32, 32), (16, 4), (16, 3), (13, 4), (64, 4), (5, 2), (17, 2), (9, 1), (3, 1),
                                 (100, 3), (48, 16), (20, 30), (64, 64), (32, 64), (32, 33), (20, 100),
                                 (64, 33), (17, 128)])
def test_encoder_is_rs_interpolation(k, m):
    """Every geometry's encoder, pinned to a closed-form Reed-Solomon definition that does
    not use the FFT, skew factors, chunk accumulation or truncation rules of the restatement:
      HighRate (C = next_pow2(m), N = next_pow2(C + k)): recovery j = P(omega_j), P the unique
        polynomial of degree < N - C with P(omega_{C+i}) = data_i and P(omega_x) = 0 for
        C + k <= x < N (the zero padding up to a whole power-of-two point set);
      LowRate (C = next_pow2(k)): recovery i = P(omega_{C+i}), P of degree < C with
        P(omega_i) = data_i (i < k) and P(omega_x) = 0 for k <= x < C.
    Together with the 32:32 case above this pins multi-chunk HighRate (16:4), the k < m
    tails (20:30), 64:64 and the LowRate shredders (CodingOnly 32:64, PETS 32:33)."""
    rng = np.random.default_rng(k * 1000 + m)
    data = [int(v) for v in rng.integers(0, 65536, size=k)]
    rec = o.encode([bytes([v & 0xFF, v >> 8]) for v in data], m)
    got = [r[0] | (r[1] << 8) for r in rec]
    if o.use_high_rate(k, m):
        C = o.next_pow2(m)
        N = o.next_pow2(C + k)
        xs = [C + i for i in range(k)] + list(range(C + k, N))
        ys = data + [0] * (N - C - k)
        pts = list(range(m))
    else:
        C = o.next_pow2(k)
        xs = list(range(C))
        ys = data + [0] * (C - k)
        pts = [C + i for i in range(m)]
    assert got == [lagrange_eval(xs, ys, x) for x in pts]


@pytest.mark.parametrize("size,delta", [(8, 0), (8, 8), (32, 0), (32, 32), (64, 64)])
def test_ifft_inverts_fft(size, delta):
    rng = np.random.default_rng(size + delta)
    v = rng.integers(0, 65536, size=(size, 5), dtype=np.uint16)
    w = v.copy()
    o.fft(w, 0, size, size, delta)
    o.ifft(w, 0, size, size, delta)
    assert np.array_equal(w, v)


def test_locator_fwht_equals_direct_product():
    """eval_poly (FWHT route of the crate) == log prod_{e != x}(x + e) (direct)."""
    rng = random.Random(3)
    erased = np.zeros(65536, np.int64)
    E = rng.sample(range(64), 20)
    erased[E] = 1
    loc = o.erasure_locator(erased, 64)
    exp, log, _, _ = o.tables()
    for x in range(64):
        acc = 1
        for e in E:
            if e != x:
                acc = gf_mul(acc, x ^ e)
        assert int(exp[int(loc[x]) % 65535]) == acc


def _walsh_mod(v):
    """Unnormalised Walsh-Hadamard transform over Z/65535 (the kernels' lane-shuffle stages)."""
    v = v.copy()
    d = 1
    while d < len(v):
        for i in range(len(v)):
            if not i & d:
                a, b = v[i], v[i | d]
                v[i], v[i | d] = (a + b) % 65535, (a - b) % 65535
        d <<= 1
    return v


@pytest.mark.parametrize("N,W", [(64, 64), (64, 32), (64, 16), (128, 128)])
def test_window_locator_walsh_route(N, W):
    """decode_rows / decode_rows128 (rs_kernels.hip): loc(x) = sum_{e erased, e != x} log(x ^ e)
    mod 65535 as the XOR convolution of L (L(z) = log z, L(0) = 0, zero past W) with the
    erasure indicator, i.e. H(H(L) * H(I)) / N over Z/65535 (N^-1 = 1024 / 512 since 2^16 = 1),
    against the loop form; the constants exp[loc] then agree bit for bit (exp[65535] = exp[0])."""
    exp, log, _, _ = o.tables()
    assert pow(N, -1, 65535) == {64: 1024, 128: 512}[N] and int(exp[65535]) == int(exp[0])
    L = np.array([int(log[z]) % 65535 if 0 < z < W else 0 for z in range(N)], np.int64)
    hl = _walsh_mod(L) * pow(N, -1, 65535) % 65535
    rng = np.random.default_rng(N * 1000 + W)
    for _ in range(24):
        ind = np.zeros(N, np.int64)
        ind[:W] = rng.random(W) < rng.random()
        got = _walsh_mod(hl * _walsh_mod(ind) % 65535)
        for x in range(W):
            want = 0
            for y in range(W):
                if ind[y] and y != x:
                    want = (want + int(log[x ^ y])) % 65535
            assert got[x] == want, (x, got[x], want)
            assert int(exp[65535 - got[x]]) == int(exp[(65535 - want) % 65535])


def test_poly_basis_powers():
    """The per-call server's locator (rs_kernels.hip PkLocTables, poly_pow_a) computes a
    decoder constant to_poly(exp[l]) as a^l in GF(2)[a] / (a^16 + a^5 + a^3 + a^2 + 1), from
    the tables a^i and a^(256 i): to_poly (the basis map of rs_device.hpp, kBasisMat[0] of the
    generated rs_consts.inc) sends exp[l] to the l-th power of the polynomial generator for
    every l, exp[65535] included."""
    import re

    exp, _, _, _ = o.tables()
    inc = open(os.path.join(ROOT, "alpenglow_amd", "csrc", "rs_consts.inc")).read()
    body = re.search(r"kBasisMat\[2\]\[16\] = \{(.*?)\};", inc, re.S).group(1)
    rows = [int(x, 0) for x in re.findall(r"0x[0-9A-Fa-f]+|\d+", body)][:16]

    def to_poly(c):
        return sum(((bin(rows[o_] & c).count("1") & 1) << o_) for o_ in range(16))

    def pmul(a, b):
        r = 0
        for i in range(16):
            if b >> i & 1:
                r ^= a << i
        for i in range(30, 15, -1):
            if r >> i & 1:
                r ^= (1 << i) ^ (0x2D << (i - 16))
        return r

    lo = [1]
    for _ in range(255):
        lo.append(pmul(lo[-1], 2))
    a256 = pmul(lo[255], 2)
    hi = [1]
    for _ in range(255):
        hi.append(pmul(hi[-1], a256))
    tp = np.array([to_poly(int(x)) for x in exp[:65536]], np.int64)
    got = np.array([pmul(hi[l_ >> 8], lo[l_ & 255]) for l_ in range(65536)], np.int64)
    assert np.array_equal(tp, got)


# ------------------------------------------------------------------------ layout & rate

def test_shard_layout_roundtrip_and_tail_split():
    for S in (2, 30, 62, 64, 66, 126, 128, 1024, 1026):
        b = o.splitmix64_bytes(S, S)
        assert o.symbols_to_shard(o.shard_to_symbols(b), S) == b
    # tail chunk of T bytes: symbol j = b[j] | b[T/2 + j] << 8 (crate Shards::insert)
    b = bytes(range(6))
    assert list(o.shard_to_symbols(b)) == [0 | 3 << 8, 1 | 4 << 8, 2 | 5 << 8]
    full = bytes(range(64))
    s = o.shard_to_symbols(full)
    assert s[0] == 0 | 32 << 8 and s[31] == 31 | 63 << 8


def test_rate_rule():
    assert o.use_high_rate(32, 32) and o.use_high_rate(16, 4) and o.use_high_rate(64, 64)
    assert not o.use_high_rate(32, 64) and not o.use_high_rate(32, 33)
    assert o.use_high_rate(20, 30) and not o.use_high_rate(30, 20)  # tie: k <= m -> HighRate
    with pytest.raises(o.RSError):
        o.use_high_rate(0, 1)
    with pytest.raises(o.RSError):
        o.use_high_rate(65536, 2)


# ------------------------------------------------------------------------- golden vectors

def _shards(seed, n, S):
    raw = o.splitmix64_bytes(seed, n * S)
    return [raw[i * S:(i + 1) * S] for i in range(n)]


def test_encode_golden(golden):
    for c in golden["encode"]:
        orig = _shards(c["seed"], c["k"], c["S"])
        rec = b"".join(o.encode(orig, c["m"]))
        assert sha(rec) == c["recovery"]["sha256"], c
        if "hex" in c["recovery"]:
            assert rec.hex() == c["recovery"]["hex"]
        # the C restatement agrees
        got = ro_c.encode(np.frombuffer(b"".join(orig), np.uint8).reshape(c["k"], c["S"]), c["m"])
        assert got.tobytes() == rec, c


def test_decode_golden(golden):
    for c in golden["decode"]:
        k, m, S = c["k"], c["m"], c["S"]
        orig = _shards(c["seed"], k, S)
        rec = o.encode(orig, m)
        og = {i: orig[i] for i in range(k) if i not in c["erased_original"]}
        rg = {j: rec[j] for j in range(m) if j not in c["erased_recovery"]}
        res = o.decode(k, m, og, rg)
        assert sha(b"".join(res[i] for i in sorted(res))) == c["restored"]["sha256"]
        assert all(res[i] == orig[i] for i in res)


def test_coder_golden(golden):
    for c in golden["coder"]:
        payload = o.splitmix64_bytes(c["seed"], c["payload_len"])
        raw = o.coder_shred(payload, c["num_coding"])
        assert len(raw.data[0]) == c["shred_bytes"]
        assert sha(b"".join(raw.data)) == c["data_sha256"]
        assert sha(b"".join(raw.coding)) == c["coding_sha256"]


# --------------------------------------------- behaviours pinned by the reference tests

def _into_shreds(raw, data_shreds=32):
    allsh = [(True, d) for d in raw.data[:data_shreds]] + [(False, c) for c in raw.coding]
    assert len(allsh) == 64
    return allsh


def _keep(shreds, idx):
    return [s if i in idx else None for i, s in enumerate(shreds)]


@pytest.mark.parametrize("size", [0, 31, o.MAX_DATA_PER_SLICE] + list(range(16383, 16415, 7)))
def test_restore_sizes(size):
    """reed_solomon.rs:244-276: restore_full / restore_tiny / restore_empty / restore_various
    (recovered from the data shreds only, take_and_map_enough_shreds :359-369)."""
    payload = o.splitmix64_bytes(size + 11, size)
    raw = o.coder_shred(payload, 32)
    sh = _keep(_into_shreds(raw), set(range(32)))
    got, raw2 = o.coder_deshred(sh, 32, 32)
    assert got == payload
    assert raw2.coding == raw.coding


def test_shred_too_much_data():
    with pytest.raises(o.RSError) as e:
        o.coder_shred(bytes(o.MAX_DATA_PER_SLICE + 1), 32)
    assert e.value.kind == "TooMuchData"


def test_deshred_patterns_of_shredding_roundtrip():
    """shredder.rs:655-706: all, first 32, last 32, {0} + {33..63}, middle 16..47, all
    but one; 1 and 31 shreds fail with NotEnoughShreds."""
    payload = o.splitmix64_bytes(99, o.MAX_DATA_PER_SLICE)
    raw = o.coder_shred(payload, 32)
    sh = _into_shreds(raw)
    for idx in [set(range(64)), set(range(32)), set(range(32, 64)), {0} | set(range(33, 64)),
                set(range(16, 48)), set(range(1, 64))]:
        got, raw2 = o.coder_deshred(_keep(sh, idx), 32, 32)
        assert got == payload
        assert raw2.data == raw.data and raw2.coding == raw.coding
    for idx in [{0}, set(range(31))]:
        with pytest.raises(o.RSError) as e:
            o.coder_deshred(_keep(sh, idx), 32, 32)
        assert e.value.kind == "NotEnoughShreds"


def test_deshred_all_zero_payload_rejected():
    """reed_solomon.rs:304-328."""
    sh = [(True, bytes(1024))] * 32 + [(False, bytes(1024))] * 32
    with pytest.raises(o.RSError) as e:
        o.coder_deshred(_keep(sh, set(range(32))), 32, 32)
    assert e.value.kind == "InvalidPadding"


def test_validated_shreds_rules():
    """reed_solomon.rs:330-347 and validated_shreds.rs:126-148."""
    raw = o.coder_shred(b"x" * 100, 32)
    sh = _into_shreds(raw)
    assert o.validate_shreds(sh, 32, 32) is not None
    odd = [(True, bytes(1023))] * 32 + [(False, bytes(1023))] * 32
    assert o.validate_shreds(odd, 32, 32) is None
    assert o.validate_shreds(sh, 1, 63) is None        # data shreds in coding positions
    assert o.validate_shreds(sh, 63, 1) is None        # coding shreds in data positions
    mixed = list(sh)
    mixed[0] = (True, bytes(2))
    assert o.validate_shreds(mixed, 32, 32) is None    # different sizes
    assert o.validate_shreds([None] * 64, 32, 32) is None


def test_deshred_rejects_oversized():
    """shredder.rs:812-830: even-sized shreds above MAX_DATA_PER_SHRED -> TooMuchData."""
    sh = [(True, bytes(1026))] * 32 + [(False, bytes(1026))] * 32
    with pytest.raises(o.RSError) as e:
        o.coder_deshred(_keep(sh, set(range(32))), 32, 32)
    assert e.value.kind == "TooMuchData"


def test_tampered_coding_shred_changes_reencode():
    """shredder.rs:759-776: re-encoding from the data shreds exposes a flipped parity byte."""
    payload = o.splitmix64_bytes(5, o.MAX_DATA_PER_SLICE)
    raw = o.coder_shred(payload, 32)
    tampered = bytearray(raw.coding[0])
    tampered[0] ^= 0xFF
    _, raw2 = o.coder_deshred(_keep(_into_shreds(raw), set(range(32))), 32, 32)
    assert raw2.coding[0] != bytes(tampered)


@pytest.mark.parametrize("k,m", [(32, 32), (16, 4), (64, 64), (32, 64), (32, 33), (3, 7), (100, 3)])
def test_random_erasure_roundtrips(k, m):
    rng = random.Random(k * 1000 + m)
    S = 66
    orig = _shards(k * m, k, S)
    rec = o.encode(orig, m)
    for _ in range(4):
        keep = set(rng.sample(range(k + m), k))
        og = {i: orig[i] for i in range(k) if i in keep}
        rg = {j: rec[j] for j in range(m) if k + j in keep}
        res = o.decode(k, m, og, rg)
        assert all(res[i] == orig[i] for i in res)
        # the C oracle decodes the same bytes
        op = np.array([i in keep for i in range(k)], np.uint8)
        rp = np.array([k + j in keep for j in range(m)], np.uint8)
        ob = np.frombuffer(b"".join(orig), np.uint8).reshape(k, S) * op[:, None]
        rb = np.frombuffer(b"".join(rec), np.uint8).reshape(m, S)
        assert ro_c.decode(ob.astype(np.uint8), op, rb, rp).tobytes() == b"".join(orig)


# ------------------------------------------------- the CPU baseline engine (bench.py)

@pytest.mark.skipif(not ro_c.avx2_available(), reason="host without AVX2")
@pytest.mark.parametrize("k,m,S", [(32, 32, 1024), (32, 32, 2048), (16, 4, 4096), (64, 64, 128), (32, 64, 1024),
                                   (32, 33, 192), (20, 30, 128), (100, 3, 64), (3, 1, 64)])
def test_avx2_engine_matches_scalar_oracle(k, m, S):
    """oracle/rs_cpu_avx2.c (the crate's Avx2 engine restated: nibble-table multiplies, the
    FWHT eval_poly locator, every received shard used) gives the scalar oracle's bytes."""
    rng = np.random.default_rng(k * 7 + m * 3 + S)
    blocks = rng.integers(0, 256, size=(3, k, S), dtype=np.uint8)
    rec = ro_c.encode_blocks(blocks, m, engine="avx2")
    assert np.array_equal(rec, ro_c.encode_blocks(blocks, m))
    cw = np.concatenate([blocks, rec], axis=1)
    r = random.Random(S)
    for _ in range(3):
        keep = set(r.sample(range(k + m), k + r.randint(0, min(m, 3))))
        op = np.array([i in keep for i in range(k)], np.uint8)
        rp = np.array([k + j in keep for j in range(m)], np.uint8)
        damaged = cw.copy()
        damaged[:, :k][:, op == 0] = 0
        got = ro_c.decode_blocks(damaged, k, op, rp, engine="avx2")
        assert np.array_equal(got, blocks)


@pytest.mark.parametrize("seed", range(4))
def test_window128_two_pass_split(seed):
    """The identity decode_x16's W = 128 passes rely on (rs_kernels.hip decode_x16 PASS 1/2):
    the crate decoder's IFFT_128 -> formal derivative -> FFT_128 equals, per output half o,
    FFT_64 (skew delta 64 o) of P(u_o) ^ u_(1-o), where u_h = IFFT_64 of window half h (delta
    64 h) and P = the derivative without its self term -- because the size-128 layer's skew
    factor (index 63) is zero.  Checked on random work vectors with the oracle's transforms."""
    _, _, skew, _ = o.tables()
    assert int(skew[63]) == o.GF_MODULUS
    rng = np.random.default_rng(seed)
    work = rng.integers(0, 65536, size=(128, 5), dtype=np.uint16)
    ref = work.copy()
    o.ifft(ref, 0, 128, 128, 0)
    o.formal_derivative(ref)
    o.fft(ref, 0, 128, 128, 0)
    u = work.copy()
    o.ifft(u, 0, 64, 64, 0)
    o.ifft(u, 64, 64, 64, 64)

    def P(v):
        d = v.copy()
        o.formal_derivative(d)
        return d ^ v

    for h in (0, 1):
        x = P(u[64 * h:64 * h + 64]) ^ u[64 * (1 - h):64 * (1 - h) + 64]
        o.fft(x, 0, 64, 64, 64 * h)
        assert np.array_equal(x, ref[64 * h:64 * h + 64])
