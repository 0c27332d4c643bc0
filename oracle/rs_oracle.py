"""CPU oracle: a numpy restatement of the Reed-Solomon path the reference shredder uses.

TEST INFRASTRUCTURE ONLY.  Nothing in ``alpenglow_amd/`` imports, links or executes this
file; only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
use it, and only as the checker.

What it restates
----------------
1. ``reed-solomon-simd`` 3.1.0, the third-party crate the reference gets its arithmetic
   from (``/root/reference/Cargo.toml:44``, pinned at ``Cargo.lock:2280-2288``,
   checksum ``cffef052...a072``).  The crate is NOT vendored in the reference and cannot
   be fetched here (no network), so its published algorithm (the Leopard-RS GF(2^16)
   additive-FFT codec of Lin, Chung and Han) is restated from the crate's public design,
   following ``SURVEY.md`` Appendix A:

   * field tables (LFSR poly 0x1002D, Cantor basis)          -> ``_build_tables``
   * skew factors and the log-Walsh table                    -> ``_build_tables``
   * FFT / IFFT butterflies with truncation                  -> ``fft`` / ``ifft``
   * shard byte layout (64-byte chunks, lo/hi byte planes)   -> ``shard_to_symbols``
   * rate choice (``rate.rs`` ``use_high_rate``)             -> ``use_high_rate``
   * HighRate / LowRate encoders and decoders                -> ``encode`` / ``decode``
   * error variants                                          -> ``RSError``

2. ``ReedSolomonCoder`` (``/root/reference/src/shredder/reed_solomon.rs:47-232``): the
   padding, split, reassembly, padding-strip and re-encode rules, and the
   ``ValidatedShreds`` checks (``validated_shreds.rs:34-114``).

Parity status: PARITY UNPINNED at the reference boundary.  The reference's own tests
hold no known-answer vectors for coding-shred bytes (``SURVEY.md`` section 8c), and the
crate cannot be built or imported here.  What *is* pinned:

* the field and evaluation-point conventions, by the mathematical self-checks in
  ``tests/test_oracle.py`` (Cantor recurrence, 0x1002D primitive, FFT encode equals
  Lagrange interpolation through the data points, IFFT o FFT = id, MDS round trips);
* every behaviour the reference's tests pin (round trips over the erasure patterns of
  ``shredder.rs:655-706``, padding sizes of ``reed_solomon.rs:244-276``, the error
  mapping of ``reed_solomon.rs:278-347`` and ``shredder.rs:708-869``).

Pure numpy; vectorised over symbol positions, so a few MiB encode in well under a second.
"""

from __future__ import annotations

import functools
from dataclasses import dataclass

import numpy as np

GF_BITS = 16
GF_ORDER = 1 << GF_BITS          # 65536
GF_MODULUS = GF_ORDER - 1        # 65535
GF_POLYNOMIAL = 0x1002D
CANTOR_BASIS = (
    0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
    0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E,
)

# reed_solomon.rs / shredder.rs constants (shredder.rs:42-54)
DATA_SHREDS = 32
TOTAL_SHREDS = 64
MAX_DATA_PER_SHRED = 1024
MAX_DATA_PER_SLICE_AFTER_PADDING = DATA_SHREDS * MAX_DATA_PER_SHRED
MAX_DATA_PER_SLICE = MAX_DATA_PER_SLICE_AFTER_PADDING - 1


class RSError(Exception):
    """Crate ``reed_solomon_simd::Error`` variants and ``ReedSolomonCoder`` errors."""

    def __init__(self, kind: str, **info):
        super().__init__(kind, info)
        self.kind = kind
        self.info = info


# --------------------------------------------------------------------------------------
# Field tables
# --------------------------------------------------------------------------------------

def _add_mod(x, y):
    """``add_mod``: x + y mod 65535 with 65535 as an alias of 0 (crate engine/mod.rs)."""
    s = np.asarray(x, dtype=np.int64) + np.asarray(y, dtype=np.int64)
    return ((s + (s >> GF_BITS)) & 0xFFFF).astype(np.int64)


def _sub_mod(x, y):
    """``sub_mod``: x - y mod 65535 computed on u32 wrap-around like the crate."""
    d = (np.asarray(x, dtype=np.int64) - np.asarray(y, dtype=np.int64)) & 0xFFFFFFFF
    return ((d + (d >> GF_BITS)) & 0xFFFF).astype(np.int64)


def _fwht(data: np.ndarray, truncated_size: int) -> None:
    """In-place Walsh-Hadamard transform mod 65535 (crate ``fwht.rs``).

    The crate fuses two layers per pass and skips groups starting at or beyond
    ``truncated_size`` (they are all-zero); the result equals the full transform of the
    zero-padded input, which is what this radix-2 form computes.
    """
    n = data.shape[0]
    dist = 1
    while dist < n:
        v = data.reshape(-1, 2, dist)
        a = v[:, 0, :].copy()
        b = v[:, 1, :].copy()
        v[:, 0, :] = _add_mod(a, b)
        v[:, 1, :] = _sub_mod(a, b)
        dist <<= 1
    del truncated_size  # all-zero tail: skipping it changes nothing


@functools.lru_cache(maxsize=1)
def _build_tables():
    """exp/log, skew and log_walsh tables (crate ``engine/tables.rs``)."""
    # LFSR table (stored in "exp" first, as the crate does)
    exp = np.zeros(GF_ORDER, dtype=np.int64)
    state = 1
    for i in range(GF_MODULUS):
        exp[state] = i
        state <<= 1
        if state >= GF_ORDER:
            state ^= GF_POLYNOMIAL
    exp[0] = GF_MODULUS

    # conversion to the Cantor basis
    log = np.zeros(GF_ORDER, dtype=np.int64)
    for i in range(GF_BITS):
        width = 1 << i
        log[width:2 * width] = log[0:width] ^ CANTOR_BASIS[i]
    log = exp[log]
    exp2 = np.zeros(GF_ORDER, dtype=np.int64)
    exp2[log] = np.arange(GF_ORDER, dtype=np.int64)
    exp2[GF_MODULUS] = exp2[0]
    exp = exp2

    def mul_scalar(x: int, log_m: int) -> int:
        if x == 0:
            return 0
        s = int(log[x]) + int(log_m)
        return int(exp[(s + (s >> GF_BITS)) & 0xFFFF])

    def add_mod_scalar(x: int, y: int) -> int:
        s = x + y
        return (s + (s >> GF_BITS)) & 0xFFFF

    # skew factors
    skew = np.zeros(GF_MODULUS, dtype=np.int64)
    temp = [1 << i for i in range(1, GF_BITS)]
    for m in range(GF_BITS - 1):
        step = 1 << (m + 1)
        skew[(1 << m) - 1] = 0
        for i in range(m, GF_BITS - 1):
            s = 1 << (i + 1)
            j = (1 << m) - 1
            idx = np.arange(j, s, step, dtype=np.int64)
            skew[idx + s] = skew[idx] ^ temp[i]
        temp[m] = GF_MODULUS - int(log[mul_scalar(temp[m], int(log[temp[m] ^ 1]))])
        for i in range(m + 1, GF_BITS - 1):
            temp[i] = mul_scalar(temp[i], add_mod_scalar(int(log[temp[i] ^ 1]), temp[m]))
    skew = log[skew]

    # log_walsh
    log_walsh = log.copy()
    log_walsh[0] = 0
    _fwht(log_walsh, GF_ORDER)

    for t in (exp, log, skew, log_walsh):
        t.setflags(write=False)
    return exp, log, skew, log_walsh


def tables():
    """Return (exp, log, skew, log_walsh) as read-only int64 arrays."""
    return _build_tables()


def mul(x: np.ndarray, log_m: int) -> np.ndarray:
    """Vectorised ``mul(x, log_m)`` = x * exp(log_m) (0 stays 0)."""
    exp, log, _, _ = _build_tables()
    x = np.asarray(x, dtype=np.int64)
    r = exp[_add_mod(log[x], log_m)]
    return np.where(x == 0, 0, r).astype(np.uint16)


# --------------------------------------------------------------------------------------
# FFT / IFFT.  `work` is an (n_rows, n_symbols) uint16 array; rows are
# shards, columns are independent codewords.
# --------------------------------------------------------------------------------------

def _bfly_fft(x: np.ndarray, y: np.ndarray, log_m: int) -> None:
    if log_m != GF_MODULUS:
        x ^= mul(y, log_m)
    y ^= x


def _bfly_ifft(x: np.ndarray, y: np.ndarray, log_m: int) -> None:
    y ^= x
    if log_m != GF_MODULUS:
        x ^= mul(y, log_m)


def fft(work: np.ndarray, pos: int, size: int, truncated_size: int, skew_delta: int) -> None:
    """Decimation-in-time FFT over ``work[pos:pos+size]`` evaluated at points
    ``skew_delta + i``; only outputs below ``truncated_size`` are required."""
    _, _, skew, _ = _build_tables()
    dist = size >> 1
    while dist >= 1:
        for r in range(0, truncated_size, 2 * dist):
            log_m = int(skew[r + dist + skew_delta - 1])
            x = work[pos + r: pos + r + dist]
            y = work[pos + r + dist: pos + r + 2 * dist]
            _bfly_fft(x, y, log_m)
        dist >>= 1


def ifft(work: np.ndarray, pos: int, size: int, truncated_size: int, skew_delta: int) -> None:
    """Inverse FFT over ``work[pos:pos+size]``; inputs at or beyond ``truncated_size``
    are zero."""
    _, _, skew, _ = _build_tables()
    dist = 1
    while dist < size:
        for r in range(0, truncated_size, 2 * dist):
            log_m = int(skew[r + dist + skew_delta - 1])
            x = work[pos + r: pos + r + dist]
            y = work[pos + r + dist: pos + r + 2 * dist]
            _bfly_ifft(x, y, log_m)
        dist <<= 1


def fft_skew_end(work, pos, size, truncated_size):
    fft(work, pos, size, truncated_size, pos + size)


def ifft_skew_end(work, pos, size, truncated_size):
    ifft(work, pos, size, truncated_size, pos + size)


def formal_derivative(work: np.ndarray) -> None:
    """``work[i - w .. i] ^= work[i .. i + w]`` for i = 1.., w = lowest set bit of i."""
    n = work.shape[0]
    for i in range(1, n):
        w = i & -i
        work[i - w: i] ^= work[i: i + w]


# --------------------------------------------------------------------------------------
# Shard byte layout: 64-byte chunks; symbol j of a chunk is
# chunk[j] | chunk[32 + j] << 8; a tail chunk of T < 64 bytes splits at T / 2.
# --------------------------------------------------------------------------------------

def shard_to_symbols(shard) -> np.ndarray:
    b = np.frombuffer(bytes(shard), dtype=np.uint8)
    n = b.shape[0]
    if n == 0 or n % 2:
        raise RSError("InvalidShardSize", shard_bytes=n)
    whole = n // 64
    tail = n % 64
    parts = []
    if whole:
        c = b[: whole * 64].reshape(whole, 64).astype(np.uint16)
        parts.append((c[:, :32] | (c[:, 32:] << 8)).reshape(-1))
    if tail:
        t = b[whole * 64:].astype(np.uint16)
        h = tail // 2
        parts.append(t[:h] | (t[h:] << 8))
    return np.concatenate(parts).astype(np.uint16)


def symbols_to_shard(sym: np.ndarray, shard_bytes: int) -> bytes:
    sym = np.asarray(sym, dtype=np.uint16)
    whole = shard_bytes // 64
    tail = shard_bytes % 64
    out = np.empty(shard_bytes, dtype=np.uint8)
    if whole:
        s = sym[: whole * 32].reshape(whole, 32)
        o = out[: whole * 64].reshape(whole, 64)
        o[:, :32] = (s & 0xFF).astype(np.uint8)
        o[:, 32:] = (s >> 8).astype(np.uint8)
    if tail:
        h = tail // 2
        s = sym[whole * 32: whole * 32 + h]
        out[whole * 64: whole * 64 + h] = (s & 0xFF).astype(np.uint8)
        out[whole * 64 + h:] = (s >> 8).astype(np.uint8)
    return out.tobytes()


# --------------------------------------------------------------------------------------
# Rate selection (crate rate.rs)
# --------------------------------------------------------------------------------------

def next_pow2(x: int) -> int:
    return 1 if x <= 1 else 1 << (x - 1).bit_length()


def check_counts(k: int, m: int) -> None:
    if k > GF_ORDER or m > GF_ORDER:
        raise RSError("UnsupportedShardCount", original_count=k, recovery_count=m)
    smaller_pow2 = min(next_pow2(k), next_pow2(m))
    larger = max(k, m)
    if k == 0 or m == 0 or smaller_pow2 + larger > GF_ORDER:
        raise RSError("UnsupportedShardCount", original_count=k, recovery_count=m)


def use_high_rate(k: int, m: int) -> bool:
    """HighRate if next_pow2(k) > next_pow2(m); LowRate if smaller; on a tie the crate
    deliberately picks HighRate when k <= m (its "wrong rate on purpose" branch)."""
    check_counts(k, m)
    pk, pm = next_pow2(k), next_pow2(m)
    if pk < pm:
        return False
    if pk > pm:
        return True
    return k <= m


def check_shard_bytes(shard_bytes: int) -> None:
    if shard_bytes == 0 or shard_bytes % 2:
        raise RSError("InvalidShardSize", shard_bytes=shard_bytes)


# --------------------------------------------------------------------------------------
# Encoders on symbol matrices
# --------------------------------------------------------------------------------------

def encode_symbols(orig: np.ndarray, m: int) -> np.ndarray:
    """orig: (k, nsym) uint16 -> recovery (m, nsym) uint16."""
    k, nsym = orig.shape
    if use_high_rate(k, m):
        chunk = next_pow2(m)
        rows = max(chunk, -(-k // chunk) * chunk)
        work = np.zeros((rows, nsym), dtype=np.uint16)
        work[:k] = orig
        first = min(k, chunk)
        ifft_skew_end(work, 0, chunk, first)
        if k > chunk:
            cs = chunk
            while cs + chunk <= k:
                ifft_skew_end(work, cs, chunk, chunk)
                work[:chunk] ^= work[cs: cs + chunk]
                cs += chunk
            last = k % chunk
            if last:
                work[cs + last:] = 0
                ifft_skew_end(work, cs, chunk, last)
                work[:chunk] ^= work[cs: cs + chunk]
        fft(work, 0, chunk, m, 0)
        return work[:m].copy()
    chunk = next_pow2(k)
    rows = max(chunk, -(-m // chunk) * chunk)
    work = np.zeros((rows, nsym), dtype=np.uint16)
    work[:k] = orig
    ifft(work, 0, chunk, k, 0)
    cs = chunk
    while cs < m:
        work[cs: cs + chunk] = work[:chunk]
        cs += chunk
    cs = 0
    while cs + chunk <= m:
        fft_skew_end(work, cs, chunk, chunk)
        cs += chunk
    last = m % chunk
    if last:
        fft_skew_end(work, cs, chunk, last)
    return work[:m].copy()


def encode(original_shards, m: int) -> list[bytes]:
    """``ReedSolomonEncoder`` new/add_original_shard xk/encode/recovery_iter."""
    k = len(original_shards)
    check_counts(k, m)
    if k == 0:
        raise RSError("TooFewOriginalShards", original_count=k, original_received_count=0)
    shard_bytes = len(original_shards[0])
    check_shard_bytes(shard_bytes)
    for s in original_shards:
        if len(s) != shard_bytes:
            raise RSError("DifferentShardSize", shard_bytes=shard_bytes, got=len(s))
    orig = np.stack([shard_to_symbols(s) for s in original_shards])
    rec = encode_symbols(orig, m)
    return [symbols_to_shard(r, shard_bytes) for r in rec]


# --------------------------------------------------------------------------------------
# Decoders -- the crate's exact algorithm, using every present shard
# --------------------------------------------------------------------------------------

def erasure_locator(erased: np.ndarray, truncated_size: int) -> np.ndarray:
    """``eval_poly``: log of prod_{e erased, e != x} (x + e) for every x, via the
    FWHT convolution the crate uses.  ``erased`` is a 0/1 array of length 65536."""
    _, _, _, log_walsh = _build_tables()
    e = erased.astype(np.int64).copy()
    _fwht(e, truncated_size)
    prod = e * log_walsh
    e = _add_mod(prod & 0xFFFF, prod >> GF_BITS)
    _fwht(e, GF_ORDER)
    return e


def decode_symbols(k: int, m: int, orig: dict, rec: dict) -> dict:
    """orig/rec: index -> uint16 symbol vector.  Returns index -> restored symbols for
    every missing original."""
    check_counts(k, m)
    if len(orig) + len(rec) < k:
        raise RSError("NotEnoughShards", original_count=k,
                      original_received_count=len(orig), recovery_received_count=len(rec))
    if len(orig) == k:
        return {}
    nsym = next(iter((orig or rec).values())).shape[0]
    erased = np.zeros(GF_ORDER, dtype=np.int64)
    if use_high_rate(k, m):
        chunk = next_pow2(m)
        end = chunk + k
        W = next_pow2(end)
        for i in range(m):
            if i not in rec:
                erased[i] = 1
        erased[m:chunk] = 1
        for i in range(k):
            if i not in orig:
                erased[chunk + i] = 1
        loc = erasure_locator(erased, end)
        work = np.zeros((W, nsym), dtype=np.uint16)
        for i, v in rec.items():
            work[i] = mul(v, int(loc[i]))
        for i, v in orig.items():
            work[chunk + i] = mul(v, int(loc[chunk + i]))
        ifft(work, 0, W, end, 0)
        formal_derivative(work)
        fft(work, 0, W, end, 0)
        return {i: mul(work[chunk + i], GF_MODULUS - int(loc[chunk + i]))
                for i in range(k) if i not in orig}
    chunk = next_pow2(k)
    end = chunk + m
    W = next_pow2(end)
    for i in range(k):
        if i not in orig:
            erased[i] = 1
    # originals k..chunk are the encoder's zero padding: known zeros, not erasures
    for i in range(m):
        if i not in rec:
            erased[chunk + i] = 1
    erased[end:] = 1
    loc = erasure_locator(erased, GF_ORDER)
    work = np.zeros((W, nsym), dtype=np.uint16)
    for i, v in orig.items():
        work[i] = mul(v, int(loc[i]))
    for i, v in rec.items():
        work[chunk + i] = mul(v, int(loc[chunk + i]))
    ifft(work, 0, W, end, 0)
    formal_derivative(work)
    fft(work, 0, W, k, 0)
    return {i: mul(work[i], GF_MODULUS - int(loc[i])) for i in range(k) if i not in orig}


def decode(k: int, m: int, original: dict, recovery: dict) -> dict:
    """``ReedSolomonDecoder``: original/recovery map index -> shard bytes.  Returns
    index -> restored original shard bytes (``DecoderResult::restored_original``)."""
    check_counts(k, m)
    sizes = {len(v) for v in list(original.values()) + list(recovery.values())}
    if not sizes:
        raise RSError("NotEnoughShards", original_count=k,
                      original_received_count=0, recovery_received_count=0)
    if len(sizes) != 1:
        raise RSError("DifferentShardSize")
    shard_bytes = sizes.pop()
    check_shard_bytes(shard_bytes)
    for i in original:
        if not 0 <= i < k:
            raise RSError("InvalidOriginalShardIndex", index=i)
    for i in recovery:
        if not 0 <= i < m:
            raise RSError("InvalidRecoveryShardIndex", index=i)
    o = {i: shard_to_symbols(v) for i, v in original.items()}
    r = {i: shard_to_symbols(v) for i, v in recovery.items()}
    res = decode_symbols(k, m, o, r)
    return {i: symbols_to_shard(v, shard_bytes) for i, v in res.items()}


# --------------------------------------------------------------------------------------
# ReedSolomonCoder (reed_solomon.rs:47-232) and ValidatedShreds (validated_shreds.rs)
# --------------------------------------------------------------------------------------

@dataclass
class RawShreds:
    data: list
    coding: list


def coder_shred(payload: bytes, num_coding: int) -> RawShreds:
    """``ReedSolomonCoder::shred`` (reed_solomon.rs:88-128)."""
    payload = bytes(payload)
    if len(payload) > MAX_DATA_PER_SLICE:
        raise RSError("TooMuchData")
    padding = 2 * DATA_SHREDS - len(payload) % (2 * DATA_SHREDS)
    shred_bytes = -(-(len(payload) + padding) // DATA_SHREDS)
    padded = payload + b"\x80" + b"\x00" * (padding - 1)
    data = [padded[i * shred_bytes:(i + 1) * shred_bytes] for i in range(DATA_SHREDS)]
    return RawShreds(data=data, coding=encode(data, num_coding))


def validate_shreds(shreds, data_shreds: int, coding_shreds: int):
    """``ValidatedShreds::try_new`` (validated_shreds.rs:34-70).  ``shreds`` is a list of
    TOTAL_SHREDS entries, each None or (is_data, bytes).  Returns None when invalid."""
    assert data_shreds + coding_shreds == TOTAL_SHREDS
    present = [s for s in shreds if s is not None]
    if not present:
        return None
    size = len(present[0][1])
    if size == 0 or size % 2:
        return None
    if any(len(s[1]) != size for s in present):
        return None
    for i, s in enumerate(shreds):
        if s is None:
            continue
        if (i < data_shreds) != bool(s[0]):
            return None
    return shreds


def coder_deshred(shreds, data_shreds: int, num_coding: int):
    """``ReedSolomonCoder::deshred`` (reed_solomon.rs:140-208) on validated shreds.
    Returns (payload, RawShreds) or raises RSError(NotEnoughShreds | TooMuchData |
    InvalidPadding)."""
    original = {i: shreds[i][1] for i in range(data_shreds) if shreds[i] is not None}
    recovery = {j - data_shreds: shreds[j][1]
                for j in range(data_shreds, TOTAL_SHREDS) if shreds[j] is not None}
    return coder_deshred_indexed(original, recovery, num_coding)


def coder_deshred_indexed(original: dict, recovery: dict, num_coding: int):
    """The body of ``ReedSolomonCoder::deshred`` (reed_solomon.rs:144-208) on the shreds'
    data indices (``data_shred_payloads``) and coding indices (``coding_shred_payloads``):
    the crate decoder over every given shred, padding strip, re-encode."""
    if len(original) + len(recovery) < DATA_SHREDS:
        raise RSError("NotEnoughShreds")
    restored = decode(DATA_SHREDS, num_coding, original, recovery)
    data = []
    payload = bytearray()
    for i in range(DATA_SHREDS):
        d = original[i] if i in original else restored[i]
        if len(payload) + len(d) > MAX_DATA_PER_SLICE_AFTER_PADDING:
            raise RSError("TooMuchData")
        payload += d
        data.append(bytes(d))
    stripped = bytes(payload).rstrip(b"\x00")
    if not stripped or stripped[-1] != 0x80:
        raise RSError("InvalidPadding")
    return stripped[:-1], RawShreds(data=data, coding=encode(data, num_coding))


# --------------------------------------------------------------------------------------
# Seeded inputs: splitmix64, u64 little-endian words
# --------------------------------------------------------------------------------------

BLOCK_SEED_BASE = 0x5EED_A19E_0000_0000


def splitmix64_bytes(seed: int, nbytes: int) -> bytes:
    n = -(-nbytes // 8)
    with np.errstate(over="ignore"):
        st = (np.uint64(seed & 0xFFFFFFFFFFFFFFFF)
              + np.arange(1, n + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15))
        z = st
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").tobytes()[:nbytes]


def block_bytes(block_index: int, nbytes: int) -> bytes:
    return splitmix64_bytes(BLOCK_SEED_BASE + block_index, nbytes)
