"""GPU parity tests: the HIP path (through the C ABI) against the oracle and the golden
fixtures.  Integer/byte work: every comparison is bit-exact.

Run on an MI355X with ``python -m pytest tests -m gpu``.
"""

import hashlib
import random

import numpy as np
import pytest

import ro_c
import rs_oracle as o
from alpenglow_amd import rs

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def sha(b):
    return hashlib.sha256(b).hexdigest()


def _shards(seed, n, S):
    raw = o.splitmix64_bytes(seed, n * S)
    return [raw[i * S:(i + 1) * S] for i in range(n)]


@pytest.fixture(scope="module")
def dev(ctx):
    """All torch work and every library launch go to one explicit (non-null) stream."""
    d = torch.device("cuda:0")
    s = torch.cuda.Stream(d)
    torch.cuda.set_stream(s)
    ctx.set_stream(s.cuda_stream)
    return d


def to_dev(a, dev):
    return torch.from_numpy(np.array(a, copy=True)).to(dev)


def gpu_encode(ctx, dev, blocks: np.ndarray, m: int) -> np.ndarray:
    """blocks: (n, k, S) uint8 -> (n, m, S) via the device-resident batch API."""
    n, k, S = blocks.shape
    d_in = to_dev(blocks.reshape(n, k * S), dev)
    d_out = torch.zeros((n, m * S), dtype=torch.uint8, device=dev)
    rs.encode_batch(ctx, k, m, S, n, d_in, k * S, d_out, m * S)
    return d_out.cpu().numpy().reshape(n, m, S)


def gpu_decode(ctx, dev, orig: np.ndarray, rec: np.ndarray, opres, rpres, mode):
    """orig (n,k,S) with absent shards arbitrary, rec (n,m,S) -> restored originals."""
    n, k, S = orig.shape
    m = rec.shape[1]
    d_o = to_dev(orig.reshape(n, k * S), dev)
    d_r = to_dev(rec.reshape(n, m * S), dev)
    rs.decode_batch(ctx, k, m, S, n, d_o, k * S, d_r, m * S, opres, rpres, mode=mode)
    return d_o.cpu().numpy().reshape(n, k, S)


# decode_c serves batches of at least this many 64-byte shard columns (256 tiles: fewer tiles
# than CUs are latency-bound and take the window decoder) -- rs_api.cpp decode_cols corr_geo
CORR_MIN_COLS = 64 * 256


def _blocks(seed, n, k, S):
    """(n, k, S) uint8 originals: the oracle's block_bytes for small batches, numpy's PCG64
    for large ones (data only; the parity is checked against the re-encoded blocks)."""
    if n * k * S <= (1 << 22):
        return np.stack([np.frombuffer(o.block_bytes(seed + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    return np.random.default_rng(seed).integers(0, 256, (n, k, S), dtype=np.uint8)


# ------------------------------------------------------------------------------ encode

def test_encode_golden(ctx, dev, golden):
    for c in golden["encode"]:
        k, m, S = c["k"], c["m"], c["S"]
        orig = np.frombuffer(b"".join(_shards(c["seed"], k, S)), np.uint8).reshape(1, k, S)
        got = gpu_encode(ctx, dev, orig, m)
        assert sha(got.tobytes()) == c["recovery"]["sha256"], (k, m, S)


def test_encode_crate_api(ctx, golden):
    for c in golden["encode"][:8]:
        k, m, S = c["k"], c["m"], c["S"]
        enc = rs.ReedSolomonEncoder(ctx, k, m, S)
        for s in _shards(c["seed"], k, S):
            enc.add_original_shard(s)
        rec = enc.encode()
        assert sha(b"".join(rec)) == c["recovery"]["sha256"]


@pytest.mark.parametrize("S,n", [(64, 1), (64, 65), (1024, 3), (1024, 77), (4096, 17), (32768, 9)])
def test_fast_encode_many_blocks(ctx, dev, S, n):
    assert rs.has_fast_path(32, 32, S)
    blocks = np.stack([np.frombuffer(o.block_bytes(b, 32 * S), np.uint8).reshape(32, S) for b in range(n)])
    got = gpu_encode(ctx, dev, blocks, 32)
    want = ro_c.encode_blocks(blocks, 32, threads=8)
    assert np.array_equal(got, want)
    assert rs.last_encode_kernels(ctx) == {"xform8"}  # fewer than 256 tiles: the latency route


@pytest.mark.parametrize("S,n,kernel", [
    (32768, 40, "xform4"),   # the headline shape (1 MiB blocks), 320 tiles
    (4096, 300, "xform4"),   # one tile per block, 300 tiles
    (65536, 18, "xform4"),   # 2 MiB shards (64 MiB blocks), 288 tiles
    (8192, 130, "xform8"),   # 256 KiB blocks: the measured 8 KiB-shard dispatch, 260 tiles
    (16384, 66, "xform8"),   # 512 KiB blocks: 16 KiB shards, 264 tiles
])
def test_headline_encode_dispatch(ctx, dev, S, n, kernel):
    """32:32 device-resident encodes of at least 256 tiles (64-column tiles): the headline
    kernel xform<4> and the 8 / 16 KiB-shard rule that sends those to xform8
    (launch_xform, rs_kernels.hip) against the C oracle, asserting which kernel ran."""
    tiles = n * (S // 64) // 64
    assert tiles >= 256
    blocks = _blocks(7100 + S, n, 32, S)
    got = gpu_encode(ctx, dev, blocks, 32)
    assert rs.last_encode_kernels(ctx) == {kernel}
    want = ro_c.encode_blocks(blocks, 32, threads=8)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("k,m", [(32, 32), (20, 30), (17, 17), (25, 32)])
def test_fast_encode_partial_geometries(ctx, dev, k, m):
    S = 128
    blocks = np.stack([np.frombuffer(o.block_bytes(100 + b, k * S), np.uint8).reshape(k, S) for b in range(5)])
    got = gpu_encode(ctx, dev, blocks, m)
    want = ro_c.encode_blocks(blocks, m)
    assert np.array_equal(got, want)


def test_encode_into_codeword_buffer(ctx, dev):
    """Data and parity of a block adjacent (k+m shards per block), strided calls."""
    k, m, S, n = 32, 32, 2048, 6
    cw = torch.zeros((n, (k + m) * S), dtype=torch.uint8, device=dev)
    rs.fill_splitmix(ctx, cw, n, k * S, (k + m) * S, o.BLOCK_SEED_BASE)
    rs.encode_batch(ctx, k, m, S, n, cw, (k + m) * S, cw.data_ptr() + k * S, (k + m) * S)
    host = cw.cpu().numpy().reshape(n, k + m, S)
    for b in range(n):
        assert host[b, :k].tobytes() == o.block_bytes(b, k * S)
    assert np.array_equal(host[:, k:], ro_c.encode_blocks(host[:, :k], m))


@pytest.mark.parametrize("k,m", [(64, 64), (33, 64), (40, 41), (48, 60)])
def test_fast_encode_64_point(ctx, dev, k, m):
    """Single-chunk HighRate with next_pow2(m) = 64: the 8-wave 64-point transform."""
    S = 4096 if k == 64 else 192
    assert rs.has_fast_path(k, m, S)
    n = 5
    blocks = np.stack([np.frombuffer(o.block_bytes(300 + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    got = gpu_encode(ctx, dev, blocks, m)
    want = ro_c.encode_blocks(blocks, m, threads=8)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("k,m,S", [(16, 4, 4096), (16, 3, 640), (13, 4, 128), (64, 4, 1024), (5, 2, 64),
                                   (9, 1, 192), (17, 2, 4096)])
def test_multichunk_small_encode(ctx, dev, k, m, S):
    """HighRate with next_pow2(m) <= 4 < k (BASELINE C4 16:4): the streaming encode_mc kernel."""
    assert rs.has_fast_path(k, m, S)
    n = 9
    blocks = np.stack([np.frombuffer(o.block_bytes(600 + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    assert np.array_equal(gpu_encode(ctx, dev, blocks, m), ro_c.encode_blocks(blocks, m, threads=8))


@pytest.mark.parametrize("k,m,S", [(32, 64, 1024), (32, 33, 4096), (20, 100, 128), (32, 20, 192), (17, 128, 64),
                                   (64, 33, 256), (40, 128, 128), (64, 192, 64)])
def test_lowrate_encode_transform(ctx, dev, k, m, S):
    """LowRate (CodingOnly 32:64, PETS 32:33, ...): two recovery chunks per launch for 32-point
    codes (pairs 0-1 and 2-3, odd counts and partial pairs included), one per chunk for 64-point."""
    assert rs.has_fast_path(k, m, S) and not rs.use_high_rate(k, m)
    n = 5
    blocks = np.stack([np.frombuffer(o.block_bytes(1100 + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    assert np.array_equal(gpu_encode(ctx, dev, blocks, m), ro_c.encode_blocks(blocks, m, threads=8))


@pytest.mark.parametrize("k,m,S", [(16, 4, 1000), (64, 64, 200), (32, 64, 1000), (32, 33, 1000), (32, 32, 1000)])
def test_generic_encode_multi_block(ctx, dev, k, m, S):
    blocks = np.stack([np.frombuffer(o.block_bytes(7 + b, k * S), np.uint8).reshape(k, S) for b in range(3)])
    assert np.array_equal(gpu_encode(ctx, dev, blocks, m), ro_c.encode_blocks(blocks, m))


def test_fill_splitmix_matches_oracle(ctx, dev):
    buf = torch.zeros((3, 4096), dtype=torch.uint8, device=dev)
    rs.fill_splitmix(ctx, buf, 3, 4096, 4096, o.BLOCK_SEED_BASE + 10)
    h = buf.cpu().numpy()
    for b in range(3):
        assert h[b].tobytes() == o.block_bytes(10 + b, 4096)


# ------------------------------------------------------------------------------ decode

@pytest.mark.parametrize("mode", [rs.DECODE_EXACT, rs.DECODE_ANY_K])
def test_decode_golden(ctx, dev, golden, mode):
    for c in golden["decode"]:
        k, m, S = c["k"], c["m"], c["S"]
        orig = _shards(c["seed"], k, S)
        rec = o.encode(orig, m)
        op = [0 if i in c["erased_original"] else 1 for i in range(k)]
        rp = [0 if j in c["erased_recovery"] else 1 for j in range(m)]
        ob = np.frombuffer(b"".join(orig), np.uint8).reshape(1, k, S).copy()
        for i in c["erased_original"]:
            ob[0, i] = 0xEE
        rb = np.frombuffer(b"".join(rec), np.uint8).reshape(1, m, S)
        got = gpu_decode(ctx, dev, ob, rb, op, rp, mode)
        restored = b"".join(got[0, i].tobytes() for i in sorted(c["erased_original"]))
        assert sha(restored) == c["restored"]["sha256"], (k, m, S, mode)
        assert got.tobytes() == b"".join(orig)


@pytest.mark.parametrize("erased", [list(range(16)), list(range(32)), [3, 17, 30]])
def test_fast_decode_from_recovery_set(ctx, dev, erased):
    """BASELINE C3 shape (scaled): 32:32, 16 (or 32) data shards erased per block."""
    k, m, S, n = 32, 32, 4096, 33
    blocks = np.stack([np.frombuffer(o.block_bytes(b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    rec = ro_c.encode_blocks(blocks, m, threads=8)
    damaged = blocks.copy()
    damaged[:, erased] = 0
    op = [0 if i in erased else 1 for i in range(k)]
    got = gpu_decode(ctx, dev, damaged, rec, op, [1] * m, rs.DECODE_ANY_K)
    assert np.array_equal(got, blocks)


@pytest.mark.parametrize("erased", [list(range(32)), list(range(64)), [0, 5, 63]])
def test_fast_decode_64_point(ctx, dev, erased):
    """64:64 with the full recovery set: 64-point transform restores the erased data."""
    k, m, S, n = 64, 64, 2048, 7
    blocks = np.stack([np.frombuffer(o.block_bytes(400 + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    rec = ro_c.encode_blocks(blocks, m, threads=8)
    damaged = blocks.copy()
    damaged[:, erased] = 0x33
    op = [0 if i in erased else 1 for i in range(k)]
    got = gpu_decode(ctx, dev, damaged, rec, op, [1] * m, rs.DECODE_ANY_K)
    assert np.array_equal(got, blocks)


@pytest.mark.parametrize("seed", [0, 1])
def test_transform64_geometries(ctx, dev, seed):
    """The 64-point transform (xform_h8): HighRate encodes with next_pow2(m) = 64, LowRate
    64-point chunk encodes and full-recovery decodes with per-block store masks, bit-exact
    against the C oracle."""
    for k, m, S, n in [(64, 64, 2048, 7), (33, 64, 192, 5), (48, 60, 192, 3), (40, 128, 128, 4),
                       (64, 192, 64, 3)]:
        blocks = np.stack([np.frombuffer(o.block_bytes(4000 + 9 * seed + b, k * S), np.uint8).reshape(k, S)
                           for b in range(n)])
        assert np.array_equal(gpu_encode(ctx, dev, blocks, m), ro_c.encode_blocks(blocks, m, threads=8)), (k, m)
    k, m, S, n = 64, 64, 1024, 9
    rng = random.Random(seed)
    blocks = np.stack([np.frombuffer(o.block_bytes(4100 + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    rec = ro_c.encode_blocks(blocks, m, threads=8)
    for per_block in (False, True):
        op = []
        for b in range(n):
            lost = set(rng.sample(range(k), rng.randrange(1, 64))) if per_block or b == 0 else lost
            op.append([0 if i in lost else 1 for i in range(k)])
        damaged = blocks.copy()
        damaged[np.array(op) == 0] = 0x5A
        flat = [x for row in op for x in row] if per_block else op[0]
        got = gpu_decode(ctx, dev, damaged, rec, flat, [1] * m * (n if per_block else 1), rs.DECODE_ANY_K)
        assert np.array_equal(got, blocks), per_block


@pytest.mark.parametrize("k,S,low", [(32, 2048, False), (64, 2048, False), (64, 1024, False), (64, 2048, True)])
def test_repeated_per_block_mask_reconstructs(ctx, dev, k, S, low):
    """Full-recovery reconstructs with a random store mask per block, repeated: an earlier
    64-point kernel skipped whole lane classes' stores in 14-45 % of such calls (timing
    dependent), which single calls rarely caught."""
    m, n = k, 64
    rng = random.Random(k * 7 + S + low)
    blocks = np.stack([np.frombuffer(o.block_bytes(4200 + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    d_rec = to_dev(ro_c.encode_blocks(blocks, m, threads=8).reshape(n, m * S), dev)
    span = k // 2 if low else k  # low: every erasure in the lower half (the pruned-FFT kernels)
    for it in range(12):
        opa = np.ones((n, k), np.uint8)
        for b in range(n):
            opa[b, rng.sample(range(span), rng.randrange(1, span))] = 0
        damaged = blocks.copy()
        damaged[opa == 0] = 0x5A
        d_o = to_dev(damaged.reshape(n, k * S), dev)
        rs.decode_batch(ctx, k, m, S, n, d_o, k * S, d_rec, m * S, opa.reshape(-1), np.ones(n * m, np.uint8),
                        mode=rs.DECODE_ANY_K)
        assert np.array_equal(d_o.cpu().numpy().reshape(n, k, S), blocks), it


@pytest.mark.parametrize("k,m", [(20, 30), (17, 24), (40, 50)])
def test_any_k_decode_partial_recovery_block(ctx, dev, k, m):
    """m < next_pow2(m): all recovery shards present is NOT a full transform set (points
    m..N-1 were never stored); the decode must still restore the originals exactly."""
    S, n = 256, 4
    blocks = np.stack([np.frombuffer(o.block_bytes(500 + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    rec = ro_c.encode_blocks(blocks, m, threads=8)
    erased = list(range(0, k, 3))
    damaged = blocks.copy()
    damaged[:, erased] = 0
    op = [0 if i in erased else 1 for i in range(k)]
    for mode in (rs.DECODE_ANY_K, rs.DECODE_EXACT):
        got = gpu_decode(ctx, dev, damaged, rec, op, [1] * m, mode)
        assert np.array_equal(got, blocks), mode


def _random_pattern_case(rng, k, m, S, n, seed, lose_rec):
    blocks = np.stack([np.frombuffer(o.block_bytes(seed + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    rec = ro_c.encode_blocks(blocks, m, threads=8)
    op, rp, damaged = [], [], blocks.copy()
    for b in range(n):
        lr = rng.randrange(0, lose_rec + 1)
        e = rng.randrange(1, m - lr + 1)
        lost, lost_r = rng.sample(range(k), min(e, k)), rng.sample(range(m), lr)
        damaged[b, lost] = 0xC3
        op += [0 if i in lost else 1 for i in range(k)]
        rp += [0 if j in lost_r else 1 for j in range(m)]
    return blocks, rec, damaged, op, rp


@pytest.mark.parametrize("k,m,S,n", [(16, 4, 4096, 6), (16, 4, 640, 11), (24, 8, 1024, 5), (20, 12, 192, 7),
                                     (32, 32, 1024, 13), (32, 16, 4096, 3), (48, 16, 2048, 4), (17, 15, 64, 9)])
@pytest.mark.parametrize("mode", [rs.DECODE_EXACT, rs.DECODE_ANY_K])
def test_general_decode_one_pattern(ctx, dev, k, m, S, n, mode):
    """Bitsliced general decoder (decode_x, W = 32 / 64), one erasure pattern for the
    batch including lost recovery shards; tiles may straddle blocks."""
    rng = random.Random(k * 1000 + m + S)
    blocks = np.stack([np.frombuffer(o.block_bytes(700 + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    rec = ro_c.encode_blocks(blocks, m, threads=8)
    lr = rng.randrange(0, m // 2 + 1)
    e = max(1, min(k, m - lr))
    lost, lost_r = rng.sample(range(k), e), rng.sample(range(m), lr)
    damaged = blocks.copy()
    damaged[:, lost] = 0x99
    op = [0 if i in lost else 1 for i in range(k)]
    rp = [0 if j in lost_r else 1 for j in range(m)]
    got = gpu_decode(ctx, dev, damaged, rec, op, rp, mode)
    assert np.array_equal(got, blocks)


@pytest.mark.parametrize("k,m,S,n", [(32, 32, 4096, 12), (16, 4, 8192, 9), (32, 16, 4096, 6)])
def test_general_decode_per_block_patterns(ctx, dev, k, m, S, n):
    """Random pattern per block (per-block tiles, S a multiple of 4 KiB), some blocks with
    the full recovery set (transform kernel), others with lost recovery shards."""
    rng = random.Random(k + m + n)
    blocks, rec, damaged, op, rp = _random_pattern_case(rng, k, m, S, n, 800, lose_rec=m // 2)
    for mode in (rs.DECODE_ANY_K, rs.DECODE_EXACT):
        got = gpu_decode(ctx, dev, damaged, rec, op, rp, mode)
        assert np.array_equal(got, blocks), mode


@pytest.mark.parametrize("k,S,n,ne,nl", [(32, 4096, 5, 16, 4), (32, 1024, 7, 16, 16), (32, 64, 70, 31, 1),
                                         (32, 8192, 3, 1, 16), (25, 2048, 4, 10, 7), (17, 64, 65, 5, 15),
                                         (32, 32768, 2, 16, 8), (20, 4096, 3, 20, 12), (32, 4096, 3, 4, 20),
                                         (32, 128, 33, 12, 13)])
def test_correction_decode_one_pattern(ctx, dev, k, S, n, ne, nl):
    """decode_c (32-point transform + K s correction) for k <= 32, m = 32 with ne erased
    originals and nl lost recovery shards; nl > 16 falls back to decode_x.  ANY_K: the
    restored originals must equal the encoded ones."""
    m = 32
    rng = random.Random(k * 7919 + S + ne * 31 + nl)
    lost, lost_r = rng.sample(range(k), ne), rng.sample(range(m), nl)
    op = [0 if i in lost else 1 for i in range(k)]
    rp = [0 if j in lost_r else 1 for j in range(m)]
    # n blocks (fewer tiles than CUs: the window decoder) and a batch of CORR_MIN_COLS columns
    # (decode_c itself when nl <= 16)
    for nb in (n, max(n, -(-CORR_MIN_COLS // (S // 64)))):
        blocks = _blocks(900 + nb, nb, k, S)
        rec = ro_c.encode_blocks(blocks, m, threads=8)
        damaged = blocks.copy()
        damaged[:, lost] = 0x5A
        rec_d = rec.copy()
        rec_d[:, lost_r] = 0xA5  # lost recovery shards must not be read
        got = gpu_decode(ctx, dev, damaged, rec_d, op, rp, rs.DECODE_ANY_K)
        assert np.array_equal(got, blocks), nb
        classes = rs.last_decode_classes(ctx)
        if nb * (S // 64) >= CORR_MIN_COLS and 0 < nl <= 16:
            assert classes.get("correction", 0) > 0, classes
        else:
            assert "correction" not in classes, classes


@pytest.mark.parametrize("S,n", [(4096, 256), (8192, 128)])
def test_correction_decode_per_block_patterns(ctx, dev, S, n):
    """A random pattern per block across the 32:32 decoders: full recovery set (transform),
    1..16 lost recovery shards (decode_c), more (decode_x), nothing erased; then a second
    pattern set through the same context (pattern cache)."""
    k = m = 32
    blocks = _blocks(1300, n, k, S)
    rec = ro_c.encode_blocks(blocks, m, threads=8)
    for seed in (1, 2):
        rng = random.Random(S + n + seed)
        op, rp, damaged, rec_d = [], [], blocks.copy(), rec.copy()
        for b in range(n):
            nl = rng.choice([0, 1, 2, 4, 8, 15, 16, 17, 24])
            ne = rng.randrange(0, m - nl + 1)
            lost, lost_r = rng.sample(range(k), min(ne, k)), rng.sample(range(m), nl)
            damaged[b, lost] = 0x77
            rec_d[b, lost_r] = 0x11
            op += [0 if i in lost else 1 for i in range(k)]
            rp += [0 if j in lost_r else 1 for j in range(m)]
        got = gpu_decode(ctx, dev, damaged, rec_d, op, rp, rs.DECODE_ANY_K)
        assert np.array_equal(got, blocks), seed
        assert rs.last_decode_classes(ctx).get("correction", 0) > 0


@pytest.mark.parametrize("k,m,S,n", [(16, 4, 4096, 6), (16, 3, 640, 5), (13, 4, 128, 7), (64, 4, 1024, 3),
                                     (5, 2, 64, 9), (9, 1, 192, 4), (17, 2, 4096, 3), (16, 4, 64, 33)])
def test_syndrome_decode_one_pattern(ctx, dev, k, m, S, n):
    """Syndrome decoder (decode_syn: m <= 4, ANY_K): every erasure count 1..m - lost
    recovery, lost recovery shards, tiles straddling blocks (S < 4 KiB)."""
    rng = random.Random(k * 7 + m * 3 + S)
    blocks = np.stack([np.frombuffer(o.block_bytes(1300 + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    rec = ro_c.encode_blocks(blocks, m, threads=8)
    for lr in range(0, m):
        for e in range(1, m - lr + 1):
            lost, lost_r = rng.sample(range(k), e), rng.sample(range(m), lr)
            damaged = blocks.copy()
            damaged[:, lost] = 0x5A
            op = [0 if i in lost else 1 for i in range(k)]
            rp = [0 if j in lost_r else 1 for j in range(m)]
            got = gpu_decode(ctx, dev, damaged, rec, op, rp, rs.DECODE_ANY_K)
            assert np.array_equal(got, blocks), (lost, lost_r)


@pytest.mark.parametrize("k,m,S,n", [(16, 4, 4096, 10), (64, 4, 4096, 5), (16, 2, 8192, 7)])
def test_syndrome_decode_per_block_patterns(ctx, dev, k, m, S, n):
    """Random pattern per block through the syndrome decoder (block-aligned tiles)."""
    rng = random.Random(k + 5 * m + n)
    blocks, rec, damaged, op, rp = _random_pattern_case(rng, k, m, S, n, 1400, lose_rec=m // 2)
    got = gpu_decode(ctx, dev, damaged, rec, op, rp, rs.DECODE_ANY_K)
    assert np.array_equal(got, blocks)


@pytest.mark.parametrize("k,m,S,n", [(32, 64, 1024, 5), (20, 100, 128, 6), (32, 33, 4096, 3), (17, 128, 64, 9),
                                     (32, 128, 256, 4)])
def test_lowrate_decode_from_full_chunk(ctx, dev, k, m, S, n):
    """LowRate decode through the transform (ANY_K): a fully present recovery chunk j gives
    every original; CodingOnlyShredder's reference-bench pattern is 32:64 with chunk 1."""
    rng = random.Random(k * 3 + m + S)
    blocks = np.stack([np.frombuffer(o.block_bytes(1600 + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    rec = ro_c.encode_blocks(blocks, m, threads=8)
    for j in range(min(4, m // 32)):
        lost = rng.sample(range(k), rng.randint(1, k))
        damaged = blocks.copy()
        damaged[:, lost] = 0x3C
        op = [0 if i in lost else 1 for i in range(k)]
        rp = [1 if 32 * j <= i < 32 * (j + 1) else rng.randint(0, 1) for i in range(m)]
        got = gpu_decode(ctx, dev, damaged, rec, op, rp, rs.DECODE_ANY_K)
        assert np.array_equal(got, blocks), (j, lost)


def test_lowrate_decode_per_block_chunks(ctx, dev):
    """Per-block patterns over different recovery chunks (one launch per chunk in use)."""
    k, m, S, n = 32, 64, 4096, 6
    rng = random.Random(99)
    blocks = np.stack([np.frombuffer(o.block_bytes(1700 + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    rec = ro_c.encode_blocks(blocks, m, threads=8)
    op, rp, damaged = [], [], blocks.copy()
    for b in range(n):
        j = b % 2
        lost = rng.sample(range(k), rng.randint(1, k))
        damaged[b, lost] = 0
        op += [0 if i in lost else 1 for i in range(k)]
        rp += [1 if 32 * j <= i < 32 * (j + 1) else 0 for i in range(m)]
    assert np.array_equal(gpu_decode(ctx, dev, damaged, rec, op, rp, rs.DECODE_ANY_K), blocks)


def test_syndrome_decode_pattern_cache(ctx, dev):
    """Back-to-back syndrome decodes with different patterns of one shape."""
    k, m, S, n = 16, 4, 4096, 3
    blocks = np.stack([np.frombuffer(o.block_bytes(1500 + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    rec = ro_c.encode_blocks(blocks, m, threads=8)
    for lost, lost_r in [([0, 1, 2, 3], []), ([15], [0, 1, 2]), ([0, 1, 2, 3], []), ([4, 9], [3]), ([15], [0, 1, 2])]:
        damaged = blocks.copy()
        damaged[:, lost] = 0
        op = [0 if i in lost else 1 for i in range(k)]
        rp = [0 if j in lost_r else 1 for j in range(m)]
        assert np.array_equal(gpu_decode(ctx, dev, damaged, rec, op, rp, rs.DECODE_ANY_K), blocks)


def test_general_decode_pattern_cache(ctx, dev):
    """Back-to-back calls with different patterns of the same shape must not reuse stale
    per-pattern matrices."""
    k, m, S, n = 32, 32, 4096, 4
    blocks = np.stack([np.frombuffer(o.block_bytes(900 + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    rec = ro_c.encode_blocks(blocks, m, threads=8)
    for lost, lost_r in [([0, 1, 2], [5]), ([7, 8], [0, 1, 2]), ([0, 1, 2], [5]), ([31], [31])]:
        damaged = blocks.copy()
        damaged[:, lost] = 0
        op = [0 if i in lost else 1 for i in range(k)]
        rp = [0 if j in lost_r else 1 for j in range(m)]
        assert np.array_equal(gpu_decode(ctx, dev, damaged, rec, op, rp, rs.DECODE_ANY_K), blocks)


def test_decode_per_block_patterns(ctx, dev):
    """Random per-block patterns: some blocks have the full recovery set (bitsliced
    kernel), others lost recovery shards too (generic kernel)."""
    rng = random.Random(11)
    k, m, S, n = 32, 32, 1024, 24
    blocks = np.stack([np.frombuffer(o.block_bytes(50 + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    rec = ro_c.encode_blocks(blocks, m, threads=8)
    op, rp = [], []
    damaged = blocks.copy()
    for b in range(n):
        if b % 3 == 0:
            lost = rng.sample(range(k), 16)
            lost_r = []
        elif b % 3 == 1:
            lost = rng.sample(range(k), 10)
            lost_r = rng.sample(range(m), 20)
        else:
            lost, lost_r = [], rng.sample(range(m), 5)
        damaged[b, lost] = 0x5A
        op += [0 if i in lost else 1 for i in range(k)]
        rp += [0 if j in lost_r else 1 for j in range(m)]
    for mode in (rs.DECODE_ANY_K, rs.DECODE_EXACT):
        got = gpu_decode(ctx, dev, damaged, rec, op, rp, mode)
        assert np.array_equal(got, blocks), mode


def test_exact_decode_matches_crate_algorithm_on_inconsistent_input(ctx, dev):
    """A tampered recovery shard: EXACT mode reproduces the crate decoder's bytes (every
    present shard used), the same as the oracle's exact decoder."""
    k, m, S = 32, 32, 256
    orig = np.frombuffer(o.block_bytes(3, k * S), np.uint8).reshape(k, S)
    rec = ro_c.encode(orig, m)
    rec[0, 0] ^= 0xFF
    op = np.ones(k, np.uint8)
    op[:8] = 0
    rp = np.ones(m, np.uint8)
    damaged = orig * op[:, None]
    want = ro_c.decode(damaged.astype(np.uint8), op, rec, rp)
    got = gpu_decode(ctx, dev, damaged[None].astype(np.uint8), rec[None], op.tolist(), rp.tolist(), rs.DECODE_EXACT)
    assert np.array_equal(got[0], want)


def test_decode_not_enough_leaves_input_untouched(ctx, dev):
    k, m, S = 32, 32, 64
    orig = np.frombuffer(o.block_bytes(9, k * S), np.uint8).reshape(1, k, S).copy()
    rec = ro_c.encode(orig[0], m)[None]
    d_o = to_dev(orig.reshape(1, -1), dev)
    before = d_o.clone()
    op = [1] * 10 + [0] * 22
    rp = [1] * 21 + [0] * 11
    with pytest.raises(rs.RSError) as e:
        rs.decode_batch(ctx, k, m, S, 1, d_o, k * S, to_dev(rec.reshape(1, -1), dev), m * S, op, rp)
    assert e.value.kind == "NotEnoughShards"
    assert torch.equal(d_o, before)


def test_decoder_crate_api(ctx):
    k, m, S = 32, 32, 512
    orig = _shards(77, k, S)
    rec = o.encode(orig, m)
    dec = rs.ReedSolomonDecoder(ctx, k, m, S)
    for i in range(5, k):
        dec.add_original_shard(i, orig[i])
    for j in range(0, m, 2):
        dec.add_recovery_shard(j, rec[j])
    res = dec.decode()
    assert sorted(res) == list(range(5)) and all(res[i] == orig[i] for i in res)
    with pytest.raises(rs.RSError) as e:
        dec.add_original_shard(40, orig[0])
    assert e.value.kind == "InvalidOriginalShardIndex"
    dec.reset(k, m, S)
    dec.add_original_shard(1, orig[1])
    with pytest.raises(rs.RSError) as e:
        dec.add_original_shard(1, orig[1])
    assert e.value.kind == "DuplicateOriginalShardIndex"
    with pytest.raises(rs.RSError) as e:
        dec.add_recovery_shard(2, orig[1][:-2])
    assert e.value.kind == "DifferentShardSize"
    with pytest.raises(rs.RSError) as e:
        dec.decode()
    assert e.value.kind == "NotEnoughShards"


def test_encoder_crate_api_errors(ctx):
    with pytest.raises(rs.RSError) as e:
        rs.ReedSolomonEncoder(ctx, 32, 32, 63)
    assert e.value.kind == "InvalidShardSize"
    enc = rs.ReedSolomonEncoder(ctx, 2, 2, 4)
    enc.add_original_shard(b"abcd")
    with pytest.raises(rs.RSError) as e:
        enc.encode()
    assert e.value.kind == "TooFewOriginalShards"
    enc.add_original_shard(b"efgh")
    with pytest.raises(rs.RSError) as e:
        enc.add_original_shard(b"ijkl")
    assert e.value.kind == "TooManyOriginalShards"
    assert b"".join(enc.encode()) == b"".join(o.encode([b"abcd", b"efgh"], 2))


# ----------------------------------------------------------- ReedSolomonCoder semantics

def _into(raw, data_shreds=32):
    return [(True, d) for d in raw.data[:data_shreds]] + [(False, c) for c in raw.coding]


def _keep(shreds, idx):
    return [s if i in idx else None for i, s in enumerate(shreds)]


def test_coder_shred_golden(ctx, golden):
    coder = rs.ReedSolomonCoder(ctx, 32)
    for c in golden["coder"]:
        raw = coder.shred(o.splitmix64_bytes(c["seed"], c["payload_len"]))
        assert len(raw.data[0]) == c["shred_bytes"]
        assert sha(b"".join(raw.data)) == c["data_sha256"]
        assert sha(b"".join(raw.coding)) == c["coding_sha256"]


def test_coder_shredding_roundtrip_regular(ctx):
    """shredder.rs:655-706 for RegularShredder (32:32)."""
    coder = rs.ReedSolomonCoder(ctx, 32)
    payload = o.splitmix64_bytes(21, rs.MAX_DATA_PER_SLICE)
    raw = coder.shred(payload)
    sh = _into(raw)
    for idx in [set(range(64)), set(range(32)), set(range(32, 64)), {0} | set(range(33, 64)),
                set(range(16, 48)), set(range(1, 64))]:
        got, raw2 = coder.deshred(_keep(sh, idx))
        assert got == payload
        assert raw2.data == raw.data and raw2.coding == raw.coding
    for idx in [{0}, set(range(31)), set()]:
        with pytest.raises(rs.RSError) as e:
            coder.deshred(_keep(sh, idx))
        assert e.value.kind == "NotEnoughShards"


def test_coder_coding_only_and_pets(ctx):
    """CodingOnlyShredder (32:64, no data shreds) and PetsShredder (32:33, 31 data shreds,
    the key-carrying data shred never sent) -- shredder.rs:362-446."""
    payload = o.splitmix64_bytes(8, 20000)
    co = rs.ReedSolomonCoder(ctx, 64)
    raw = co.shred(payload)
    assert b"".join(raw.coding) == b"".join(o.coder_shred(payload, 64).coding)
    sh = [(False, c) for c in raw.coding]
    for idx in [set(range(64)), set(range(32)), set(range(32, 64))]:
        got, _ = co.deshred(_keep(sh, idx), data_shreds=0)
        assert got == payload
    pets = rs.ReedSolomonCoder(ctx, 33)
    raw = pets.shred(payload)
    sh = [(True, d) for d in raw.data[:31]] + [(False, c) for c in raw.coding]
    for idx in [set(range(64)), set(range(32, 64)), set(range(1, 33))]:
        got, raw2 = pets.deshred(_keep(sh, idx), data_shreds=31)
        assert got == payload and raw2.coding == raw.coding


def test_coder_error_mapping(ctx):
    coder = rs.ReedSolomonCoder(ctx, 32)
    with pytest.raises(rs.RSError) as e:
        coder.shred(bytes(rs.MAX_DATA_PER_SLICE + 1))
    assert e.value.kind == "TooMuchData"
    zero = [(True, bytes(1024))] * 32 + [(False, bytes(1024))] * 32
    with pytest.raises(rs.RSError) as e:
        coder.deshred(_keep(zero, set(range(32))))
    assert e.value.kind == "InvalidPadding"
    big = [(True, bytes(1026))] * 32 + [(False, bytes(1026))] * 32
    with pytest.raises(rs.RSError) as e:
        coder.deshred(_keep(big, set(range(32))))
    assert e.value.kind == "TooMuchData"
    raw = coder.shred(b"hello")
    wrong = [(False, d) for d in raw.data] + [(False, c) for c in raw.coding]
    with pytest.raises(rs.RSError) as e:
        coder.deshred(wrong)
    assert e.value.kind == "InvalidLayout"
    odd = [(True, bytes(3))] * 32 + [None] * 32
    with pytest.raises(rs.RSError) as e:
        coder.deshred(odd)
    assert e.value.kind == "InvalidLayout"


# ------------------------------------------------------------------ coder batches (§8 f1)

def _payload_lens(rng, S, n):
    """Payload lengths that all pad to shred size S (reed_solomon.rs:94-95)."""
    return [rng.randrange(max(0, 32 * S - 64), 32 * S) for _ in range(n)]


@pytest.mark.parametrize("S,n,inplace", [(1024, 6, False), (62, 5, False), (64, 9, True), (1024, 3, True)])
def test_coder_shred_batch(ctx, dev, S, n, inplace):
    rng = random.Random(S * 7 + n)
    m = 32
    lens = _payload_lens(rng, S, n)
    payloads = [o.splitmix64_bytes(1000 + b, L) for b, L in enumerate(lens)]
    stride = (32 + m) * S
    cw = np.full((n, stride), 0xEE, np.uint8)
    if inplace:
        for b, p in enumerate(payloads):
            cw[b, :len(p)] = np.frombuffer(p, np.uint8)
        d_cw = to_dev(cw, dev)
        rs.coder_shred_batch(ctx, m, n, S, None, 0, lens, d_cw, stride)
    else:
        P = (32 * S + 15) // 16 * 16
        pay = np.zeros((n, P), np.uint8)
        for b, p in enumerate(payloads):
            pay[b, :len(p)] = np.frombuffer(p, np.uint8)
        d_pay, d_cw = to_dev(pay, dev), to_dev(cw, dev)
        rs.coder_shred_batch(ctx, m, n, S, d_pay, P, lens, d_cw, stride)
    host = d_cw.cpu().numpy()
    for b in range(n):
        raw = o.coder_shred(payloads[b], m)
        assert host[b, :32 * S].tobytes() == b"".join(raw.data)
        assert host[b, 32 * S:].tobytes() == b"".join(raw.coding)


def test_coder_shred_batch_errors(ctx, dev):
    cw = torch.zeros((2, 64 * 64), dtype=torch.uint8, device=dev)
    with pytest.raises(rs.RSError) as e:
        rs.coder_shred_batch(ctx, 32, 2, 64, None, 0, [2000, 40000], cw, 64 * 64)
    assert e.value.kind == "TooMuchData"
    with pytest.raises(rs.RSError):  # 100 pads to S = 4, not 64
        rs.coder_shred_batch(ctx, 32, 2, 64, None, 0, [2000, 100], cw, 64 * 64)


@pytest.mark.parametrize("S", [1024, 96])
@pytest.mark.parametrize("mode", [rs.DECODE_EXACT, rs.DECODE_ANY_K])
@pytest.mark.parametrize("m", [32, 33, 64])
def test_coder_deshred_batch(ctx, dev, S, mode, m):
    """Batched deshred vs the oracle's ReedSolomonCoder::deshred: restored payload, all data
    shards, re-encoded coding shards; NotEnoughShreds / InvalidPadding slices untouched.
    m = 64 is CodingOnlyShredder's coder (LowRate 32:64; at S = 1024 the device-pattern path
    with the W = 128 window), including slices that keep only coding shreds; m = 33 is
    PetsShredder's (the same window, coding shreds past 33 never present)."""
    rng = random.Random(S + mode + m)
    n = 9
    stride = (32 + m) * S
    lens = _payload_lens(rng, S, n)
    cw = np.zeros((n, stride), np.uint8)
    for b in range(n):
        if b == 6:    # all-zero data: consistent codeword, invalid padding
            continue
        if b == 7:    # random data without a 0x80 marker at the end of the nonzero bytes
            data = bytearray(o.splitmix64_bytes(77, 32 * S))
            data[-1] = 0x11
            cw[b, :32 * S] = np.frombuffer(bytes(data), np.uint8)
            cw[b, 32 * S:] = np.frombuffer(b"".join(o.encode([bytes(data[i * S:(i + 1) * S])
                                                             for i in range(32)], m)), np.uint8)
            continue
        raw = o.coder_shred(o.splitmix64_bytes(2000 + b, lens[b]), m)
        cw[b] = np.frombuffer(b"".join(raw.data) + b"".join(raw.coding), np.uint8)
    present = []
    for b in range(n):
        if b == 0:
            keep = set(range(32 + m))
        elif b == 1:
            keep = set(range(32, 64))           # all data lost (coding 0..31)
        elif b == 2 and m > 32:
            keep = set(rng.sample(range(32, 32 + m), 32))  # coding shreds only (CodingOnly random arrival)
        elif b == 3:
            keep = set(rng.sample(range(32 + m), 31))  # not enough
        else:
            keep = set(rng.sample(range(32 + m), rng.randrange(32, 32 + m)))
        present.append(keep)
    damaged = cw.copy()
    for b in range(n):
        for i in range(32 + m):
            if i not in present[b]:
                damaged[b, i * S:(i + 1) * S] = 0xAB
    dp = [1 if i in present[b] else 0 for b in range(n) for i in range(32)]
    cp = [1 if 32 + j in present[b] else 0 for b in range(n) for j in range(m)]
    d_cw = to_dev(damaged, dev)
    res = rs.coder_deshred_batch(ctx, m, n, S, d_cw, stride, dp, cp, mode)
    host = d_cw.cpu().numpy()
    for b in range(n):
        orig_b = {i: cw[b, i * S:(i + 1) * S].tobytes() for i in range(32) if i in present[b]}
        rec_b = {j: cw[b, (32 + j) * S:(33 + j) * S].tobytes() for j in range(m) if 32 + j in present[b]}
        try:
            payload, raw = o.coder_deshred_indexed(orig_b, rec_b, m)
        except o.RSError as err:  # wrapper NotEnoughShreds maps to the crate status code
            assert res[b] == {"NotEnoughShreds": "NotEnoughShards"}.get(err.kind, err.kind), (b, res[b])
            for j in range(m):  # the received coding shreds untouched (absent ones unspecified)
                if 32 + j in present[b]:
                    assert host[b, (32 + j) * S:(33 + j) * S].tobytes() == damaged[b, (32 + j) * S:(33 + j) * S].tobytes()
            continue
        assert res[b] == len(payload), (b, res[b])
        assert host[b, :len(payload)].tobytes() == payload
        assert host[b, :32 * S].tobytes() == b"".join(raw.data)
        assert host[b, 32 * S:].tobytes() == b"".join(raw.coding)


@pytest.mark.gpu
@pytest.mark.parametrize("S", [1024, 128])
@pytest.mark.parametrize("keep,kernels", [
    (set(range(64, 96)), {"lowrate"}),                            # coding 32..63 (the reference bench)
    (set(range(32, 64)), {"lowrate"}),                            # coding 0..31
    (set(range(16)) | set(range(32, 48)), {"lowrate2"}),          # absent shreds in both chunks
    (set(range(8)) | set(range(72, 96)), {"lowrate2"}),
])
def test_coder_deshred_uniform_lowrate_chunks(ctx, dev, S, keep, kernels):
    """CodingOnlyShredder's coder (LowRate 32:64) with one pattern for the batch and exactly 32
    kept shreds: the codeword is unique, so the re-encode only needs the absent coding shreds;
    when they all lie in one 32-shard recovery chunk that chunk alone is encoded (one 32-point
    transform, store mask of the absent shreds), else both (the two-chunk kernel).  Against the
    oracle's ReedSolomonCoder::deshred (reed_solomon.rs:140-208); absent shreds hold garbage,
    one slice has an invalid padding (its coding shreds stay as received)."""
    m, n = 64, 6
    stride = (32 + m) * S
    rng = random.Random(S + len(keep))
    lens = _payload_lens(rng, S, n)
    cw = np.zeros((n, stride), np.uint8)
    for b in range(n):
        if b == 3:  # random data without a padding marker
            data = bytearray(o.splitmix64_bytes(330 + S, 32 * S))
            data[-1] = 0x11
            cw[b, :32 * S] = np.frombuffer(bytes(data), np.uint8)
            cw[b, 32 * S:] = np.frombuffer(b"".join(o.encode([bytes(data[i * S:(i + 1) * S]) for i in range(32)], m)),
                                           np.uint8)
            continue
        raw = o.coder_shred(o.splitmix64_bytes(4400 + b + S, lens[b]), m)
        cw[b] = np.frombuffer(b"".join(raw.data) + b"".join(raw.coding), np.uint8)
    damaged = cw.copy()
    for b in range(n):
        for i in range(32 + m):
            if i not in keep:
                damaged[b, i * S:(i + 1) * S] = (0x3C + i) & 0xFF
    dp = [1 if i in keep else 0 for _ in range(n) for i in range(32)]
    cp = [1 if 32 + j in keep else 0 for _ in range(n) for j in range(m)]
    d_cw = to_dev(damaged, dev)
    res = rs.coder_deshred_batch(ctx, m, n, S, d_cw, stride, dp, cp, rs.DECODE_ANY_K)
    assert rs.last_encode_kernels(ctx) == kernels
    host = d_cw.cpu().numpy()
    for b in range(n):
        orig_b = {i: cw[b, i * S:(i + 1) * S].tobytes() for i in range(32) if i in keep}
        rec_b = {j: cw[b, (32 + j) * S:(33 + j) * S].tobytes() for j in range(m) if 32 + j in keep}
        try:
            payload, raw = o.coder_deshred_indexed(orig_b, rec_b, m)
        except o.RSError as err:
            assert b == 3 and res[b] == err.kind, (b, res[b], err.kind)
            for j in range(m):
                if 32 + j in keep:
                    assert host[b, (32 + j) * S:(33 + j) * S].tobytes() == damaged[b, (32 + j) * S:(33 + j) * S].tobytes()
            continue
        assert res[b] == len(payload), (b, res[b])
        assert host[b, :32 * S].tobytes() == b"".join(raw.data), b
        assert host[b, 32 * S:].tobytes() == b"".join(raw.coding), b


@pytest.mark.parametrize("S", [1024, 512, 64, 1000, 1022, 80, 126])
@pytest.mark.parametrize("mode", [rs.DECODE_ANY_K, rs.DECODE_EXACT])
def test_coder_deshred_fused_coding_restore(ctx, dev, mode, S):
    """The follower's deshred at exactly k = 32 kept shreds (slot_block_data.rs:343-355): the
    window decoder restores the absent coding shreds in the same transform as the data shreds
    (16 columns per shred -- 1 KiB, or 960 + T bytes -- decode_pk<-1>; other sizes decode_h8<-1>;
    the TAIL variants move a last chunk of T = S mod 64 >= 16 bytes (S = 1000, 1022, 80, 126)
    whole; no re-encode pass),
    bit-exact against the oracle's re-encode (o.encode of the restored data,
    reed_solomon.rs:206), mixed with slices that keep the separate re-encode (surplus shreds;
    every data shred present), NotEnoughShreds and InvalidPadding slices.  Every absent shred is
    overwritten with garbage first.  The kernel record names the fused window kernel."""
    rng = random.Random(0xF05E + mode + S)
    n, m = 64, 32
    stride = (32 + m) * S
    lens = _payload_lens(rng, S, n)
    cw = np.zeros((n, stride), np.uint8)
    for b in range(n):
        if b in (6, 40):  # random data without a padding marker: InvalidPadding
            data = bytearray(o.splitmix64_bytes(900 + b, 32 * S))
            data[-1] = 0x11
            cw[b, :32 * S] = np.frombuffer(bytes(data), np.uint8)
            cw[b, 32 * S:] = np.frombuffer(b"".join(o.encode([bytes(data[i * S:(i + 1) * S]) for i in range(32)], m)),
                                           np.uint8)
            continue
        raw = o.coder_shred(o.splitmix64_bytes(3000 + b, lens[b]), m)
        cw[b] = np.frombuffer(b"".join(raw.data) + b"".join(raw.coding), np.uint8)
    present = []
    for b in range(n):
        if b == 1:
            keep = set(range(32))                     # every data shred, no coding: re-encode
        elif b == 2:
            keep = set(range(32, 64))                 # every coding shred, no data
        elif b == 3:
            keep = set(rng.sample(range(64), 31))     # NotEnoughShreds
        elif b % 9 == 5 and mode == rs.DECODE_ANY_K:
            keep = set(rng.sample(range(64), 36))     # surplus: the separate re-encode
        else:
            keep = set(rng.sample(range(64), 32))     # random 32-of-64 arrival: fused
        present.append(keep)
    damaged = cw.copy()
    for b in range(n):
        for i in range(64):
            if i not in present[b]:
                damaged[b, i * S:(i + 1) * S] = (0x5A + i) & 0xFF
    dp = [1 if i in present[b] else 0 for b in range(n) for i in range(32)]
    cp = [1 if 32 + j in present[b] else 0 for b in range(n) for j in range(m)]
    d_cw = to_dev(damaged, dev)
    res = rs.coder_deshred_batch(ctx, m, n, S, d_cw, stride, dp, cp, mode)
    host = d_cw.cpu().numpy()
    ok = 0
    for b in range(n):
        orig_b = {i: cw[b, i * S:(i + 1) * S].tobytes() for i in range(32) if i in present[b]}
        rec_b = {j: cw[b, (32 + j) * S:(33 + j) * S].tobytes() for j in range(m) if 32 + j in present[b]}
        try:
            payload, raw = o.coder_deshred_indexed(orig_b, rec_b, m)
        except o.RSError as err:
            assert res[b] == {"NotEnoughShreds": "NotEnoughShards"}.get(err.kind, err.kind), (b, res[b])
            for i in present[b]:
                assert host[b, i * S:(i + 1) * S].tobytes() == damaged[b, i * S:(i + 1) * S].tobytes(), (b, i)
            continue
        ok += 1
        assert res[b] == len(payload), (b, res[b])
        assert host[b, :32 * S].tobytes() == b"".join(raw.data), b
        assert host[b, 32 * S:].tobytes() == b"".join(raw.coding), b
    assert ok >= n - 4
    assert rs.last_window_kernels(ctx) == {"decode_pk_fused" if (S + 63) // 64 == 16 else "decode_h8_fused"}


@pytest.mark.parametrize("S", [1024, 256, 1000, 968, 66])
def test_coder_deshred_fused_at_scale(ctx, dev, S):
    """The fused route at production scale: 4096 slices, each received as a random 32 of its 64
    shreds (absent shreds overwritten with garbage); S = 1000 / 968 / 66 end in a tail chunk of
    40 / 8 / 2 bytes (short tails take the device path because no slice needs the re-encode).  Every slice must come back as its
    original codeword (data and coding shreds); the kernel record shows the fused window
    decoder ran and no re-encode kernel was launched (no slice has surplus or every data
    shred).  A sample of slices is also checked against the oracle's coder."""
    rng = np.random.default_rng(0xFA57 + S)
    n, m = 4096, 32
    L = 32 * S - 1
    stride = 64 * S
    d_cw = torch.empty((n, stride), dtype=torch.uint8, device=dev)
    rs.fill_splitmix(ctx, d_cw, n, 32 * S, stride, 0xF0F0)
    rs.coder_shred_batch(ctx, m, n, S, None, 0, np.full(n, L, np.uint32), d_cw, stride)
    want = d_cw.clone()
    arrived = np.argsort(rng.random((n, 64)), axis=1)[:, :32]
    present = np.zeros((n, 64), np.uint8)
    np.put_along_axis(present, arrived, 1, axis=1)
    pres = torch.from_numpy(present).to(dev)
    view = d_cw.view(n, 64, S)
    garbage = torch.full_like(view, 0xA5)
    view.copy_(torch.where(pres.bool().unsqueeze(-1), view, garbage))
    dp = np.ascontiguousarray(present[:, :32]).reshape(-1)
    cp = np.ascontiguousarray(present[:, 32:]).reshape(-1)
    res = rs.coder_deshred_batch(ctx, m, n, S, d_cw, stride, dp, cp, rs.DECODE_ANY_K, as_array=True)
    assert (res == L).all()
    assert torch.equal(d_cw, want)
    assert rs.last_window_kernels(ctx) == {"decode_pk_fused" if (S + 63) // 64 == 16 else "decode_h8_fused"}
    assert rs.last_encode_kernels(ctx) == set()  # the re-encode was skipped
    host = want[:4].cpu().numpy()
    for b in range(4):
        raw = o.coder_shred(host[b, :L].tobytes(), m)
        assert host[b].tobytes() == b"".join(raw.data) + b"".join(raw.coding), b


# --------------------------------------------------------- host-memory (PCIe) pipeline

@pytest.mark.parametrize("k,m,S,n", [(32, 32, 32768, 70), (16, 4, 4096, 9), (32, 64, 1024, 5)])
def test_host_memory_encode_pipeline(ctx, k, m, S, n):
    """Host buffers, several staging groups (64 MiB each) in flight."""
    blocks = np.stack([np.frombuffer(o.block_bytes(1300 + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    want = ro_c.encode_blocks(blocks, m, threads=8)
    orig = np.ascontiguousarray(blocks.reshape(n, k * S))
    rec = np.zeros((n, m * S), np.uint8)
    rs.encode_batch(ctx, k, m, S, n, orig.ctypes.data, k * S, rec.ctypes.data, m * S, memory=rs.MEM_HOST)
    assert np.array_equal(rec.reshape(n, m, S), want)


@pytest.mark.parametrize("case", ["full_recovery", "lost_coding", "per_block", "exact"])
def test_host_memory_decode_pipeline(ctx, case):
    k, m, S, n = 32, 32, 32768, 70
    rng = random.Random(hash(case) & 0xFFFF)
    blocks = np.stack([np.frombuffer(o.block_bytes(1400 + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    rec = ro_c.encode_blocks(blocks, m, threads=8)
    if case == "per_block":
        op, rp = [], []
        for b in range(n):
            lost = rng.sample(range(k), rng.randrange(1, 17))
            lost_r = rng.sample(range(m), rng.randrange(0, 8))
            op += [0 if i in lost else 1 for i in range(k)]
            rp += [0 if j in lost_r else 1 for j in range(m)]
        opa = np.array(op, np.uint8).reshape(n, k)
    else:
        lost = rng.sample(range(k), 16)
        op = [0 if i in lost else 1 for i in range(k)]
        rp = [1] * m if case in ("full_recovery", "exact") else [0 if j in (3, 9) else 1 for j in range(m)]
        opa = np.tile(np.array(op, np.uint8), (n, 1))
    damaged = blocks.copy()
    damaged[opa == 0] = 0x6D
    orig = np.ascontiguousarray(damaged.reshape(n, k * S))
    recb = np.ascontiguousarray(rec.reshape(n, m * S))
    mode = rs.DECODE_EXACT if case == "exact" else rs.DECODE_ANY_K
    rs.decode_batch(ctx, k, m, S, n, orig.ctypes.data, k * S, recb.ctypes.data, m * S, op, rp, mode=mode,
                    memory=rs.MEM_HOST)
    assert np.array_equal(orig.reshape(n, k, S), blocks)


# ------------------------------------------------- C4 sweep points at their full shard size

@pytest.mark.parametrize("k,m,S,n", [(16, 4, 65536, 3), (16, 4, 262144, 2), (32, 32, 32768, 4),
                                     (32, 32, 131072, 2), (64, 64, 16384, 3), (64, 64, 65536, 2)])
def test_c4_large_shard_sizes(ctx, dev, k, m, S, n):
    """BASELINE configs[3] block sizes above the other tests' shard sizes (S up to 256 KiB):
    device-resident encode, then reconstruct with k/2 (at most m) data shards erased, and a
    per-block random pattern that also loses coding shards (the general decoders), all
    compared with the C oracle (catches 32-bit offset and tiling faults at these sizes)."""
    assert rs.has_fast_path(k, m, S)
    blocks = np.stack([np.frombuffer(o.block_bytes(5000 + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    rec = gpu_encode(ctx, dev, blocks, m)
    assert np.array_equal(rec, ro_c.encode_blocks(blocks, m, threads=8))
    e = min(k // 2, m)
    damaged = blocks.copy()
    damaged[:, :e] = 0
    got = gpu_decode(ctx, dev, damaged, rec, [0] * e + [1] * (k - e), [1] * m, rs.DECODE_ANY_K)
    assert np.array_equal(got, blocks)
    # per-block random patterns with lost coding shreds
    rng = random.Random(k * 1000 + S)
    lc = min(4, m - e) if m > e else 0
    e2 = min(e, m - lc)
    op, rp = [], []
    damaged = blocks.copy()
    rec2 = rec.copy()
    for b in range(n):
        lost = set(rng.sample(range(k), e2))
        lost_r = set(rng.sample(range(m), lc))
        op += [0 if i in lost else 1 for i in range(k)]
        rp += [0 if j in lost_r else 1 for j in range(m)]
        for i in lost:
            damaged[b, i] = 0x5A
        for j in lost_r:
            rec2[b, j] = 0xA5
    for mode in (rs.DECODE_ANY_K, rs.DECODE_EXACT):
        got = gpu_decode(ctx, dev, damaged, rec2, op, rp, mode)
        assert np.array_equal(got, blocks), mode


def test_fast_decode_low_half_pruned(ctx, dev):
    """32:32 from the full recovery set with every erased original among shards 0..15: the
    output-pruned transform (16-point FFT tail).  Per-block random subsets (1..16 erased,
    incl. single shards), S = 4096 (whole tiles per block) and S = 64 (tiles straddle
    blocks), against the original data."""
    rng = random.Random(77)
    k, m = 32, 32
    for S, n in [(4096, 13), (64, 200)]:
        blocks = np.stack([np.frombuffer(o.block_bytes(700 + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
        rec = ro_c.encode_blocks(blocks, m, threads=8)
        damaged = blocks.copy()
        op = []
        for b in range(n):
            lost = set(rng.sample(range(16), rng.randint(1, 16)))
            op += [0 if i in lost else 1 for i in range(k)]
            for i in lost:
                damaged[b, i] = 0xC3
        got = gpu_decode(ctx, dev, damaged, rec, op, [1] * (m * n), rs.DECODE_ANY_K)
        assert np.array_equal(got, blocks), S
        # one shared pattern: shards 15 and 0 only
        d1 = blocks.copy()
        d1[:, [0, 15]] = 0
        got = gpu_decode(ctx, dev, d1, rec, [0] + [1] * 14 + [0] + [1] * 16, [1] * m, rs.DECODE_ANY_K)
        assert np.array_equal(got, blocks), S


@pytest.mark.parametrize("S,n", [(1024, 40), (96, 30), (192, 25), (64, 70), (2048, 9)])
@pytest.mark.parametrize("mode", [rs.DECODE_ANY_K, rs.DECODE_EXACT])
def test_decode_per_slice_random_patterns(ctx, dev, S, n, mode):
    """The follower's deshred shape (slot_block_data.rs:331-370): 32:32, every slice loses
    an arbitrary set of data AND coding shreds (here: keeps a random 32..40 of 64).  With
    S < 4 KiB the tiles straddle slices: the per-lane-pattern general decoder.  Compared
    with the original data; ANY_K uses exactly 32 survivors, EXACT all present shards."""
    rng = random.Random(S * 31 + n + mode)
    k = m = 32
    blocks = np.stack([np.frombuffer(o.block_bytes(900 + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    rec = ro_c.encode_blocks(blocks, m, threads=8)
    d_o, d_r, op, rp = blocks.copy(), rec.copy(), [], []
    for b in range(n):
        keep = set(rng.sample(range(64), rng.randint(32, 40)))
        if b % 7 == 0:
            keep = set(range(32, 64))  # all coding present: the transform path, mixed in
        op += [1 if i in keep else 0 for i in range(k)]
        rp += [1 if 32 + j in keep else 0 for j in range(m)]
        for i in range(k):
            if i not in keep:
                d_o[b, i] = 0x77
        for j in range(m):
            if 32 + j not in keep:
                d_r[b, j] = 0x99
    got = gpu_decode(ctx, dev, d_o, d_r, op, rp, mode)
    assert np.array_equal(got, blocks)


@pytest.mark.parametrize("S,n", [(1024, 300), (960, 257), (1000, 300), (192, 131), (64, 600), (2000, 90), (968, 200),
                                 (1022, 150), (66, 400)])
def test_decode_device_patterns_lost_coding(ctx, dev, S, n):
    """Per-block patterns of the 32:32 code with lost coding shreds on tiles that straddle blocks
    (S < 4 KiB; S = 1000 / 2000 / 1022 / 968 / 66 with their tails as the last column of the
    same decode, decode_h8 / decode_pk TAIL, no restride): the window decode
    with its masks built on the device from the packed presence words (decode_cols_device_
    patterns).  Random 8-20 data shards erased and 1-12 coding shards lost per block, a few
    blocks with every data shard present; absent shards overwritten with garbage; ANY_K.
    Compared with the original data, and the class record counts every block's pattern."""
    rng = random.Random(S * 13 + n)
    k = m = 32
    blocks = _blocks(4400 + S, n, k, S)
    rec = ro_c.encode_blocks(blocks, m, threads=8)
    d_o, d_r, op, rp = blocks.copy(), rec.copy(), [], []
    restore = 0
    for b in range(n):
        lost_c = set(rng.sample(range(m), rng.randint(1, 12)))
        erased = set() if b % 11 == 3 else set(rng.sample(range(k), rng.randint(8, min(20, m - len(lost_c)))))
        restore += 1 if erased else 0
        op += [0 if i in erased else 1 for i in range(k)]
        rp += [0 if j in lost_c else 1 for j in range(m)]
        for i in erased:
            d_o[b, i] = 0x77
        for j in lost_c:
            d_r[b, j] = 0x99
    got = gpu_decode(ctx, dev, d_o, d_r, op, rp, rs.DECODE_ANY_K)
    assert np.array_equal(got, blocks)
    parts = 1  # one decode, the tail (if any) as its last column
    assert rs.last_decode_classes(ctx) == {"window64": parts * restore, "none": parts * (n - restore)}


@pytest.mark.parametrize("k,m,n", [(32, 32, 25), (32, 32, 64), (32, 64, 11), (20, 40, 9)])
def test_packed_window64_follower(ctx, dev, k, m, n):
    """decode_pk (the W = 64 window with packed locator products) on 1 KiB shreds, ANY_K: the
    follower's random 32-of-64 arrival (exactly k survivors, the device-pattern path's shape),
    slices with every data shred present, slices that lost only coding shreds, an odd slice
    count (a one-slice last tile) and the LowRate sub-window (32:64, 20:40), against the
    original data.  Every lost shred's bytes are overwritten first."""
    S = 1024
    rng = random.Random(k * 7 + m + n)
    blocks = np.stack([np.frombuffer(o.block_bytes(5100 + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    rec = ro_c.encode_blocks(blocks, m, threads=8)
    d_o, d_r, op, rp = blocks.copy(), rec.copy(), [], []
    pool = k + m if k > m else k + min(m, 32)
    for b in range(n):
        keep = set(rng.sample(range(pool), k))
        if b % 5 == 3:
            keep = set(range(k)) | set(rng.sample(range(k, pool), 3))  # nothing to restore
        if b % 7 == 5:
            keep = set(range(k + min(m, 32)))  # every shard inside the window
        op += [1 if i in keep else 0 for i in range(k)]
        rp += [1 if k + j in keep else 0 for j in range(m)]
        for i in range(k):
            if i not in keep:
                d_o[b, i] = 0x3C
        for j in range(m):
            if k + j not in keep:
                d_r[b, j] = 0xC3
    got = gpu_decode(ctx, dev, d_o, d_r, op, rp, rs.DECODE_ANY_K)
    assert np.array_equal(got, blocks)


@pytest.mark.parametrize("k,m", [(32, 32), (32, 64), (32, 33), (40, 16), (48, 8), (20, 40)])
@pytest.mark.parametrize("S,n", [(1024, 24), (64, 70), (192, 23)])
@pytest.mark.parametrize("mode", [rs.DECODE_ANY_K, rs.DECODE_EXACT])
def test_decode_per_lane_window64(ctx, dev, k, m, S, n, mode):
    """Per-lane W = 64 windows on 32-column tiles (decode_h8): HighRate with the originals in
    window half 1 (32:32), straddling both halves (40:16, 48:8: no pruned FFT half), and the
    LowRate sub-window (32:64, 32:33, 20:40: originals in half 0).  S = 64 puts 32 blocks
    in one tile (the most staged constants); S = 192 tiles that start mid-block.  Random
    per-block losses keeping k..k+4 shards, against the original data; the class must be
    window64 for some blocks (the others take the transform, LowRate-chunk, W = 128 or
    generic paths)."""
    rng = random.Random(k * 1009 + m * 31 + S + mode)
    blocks = np.stack([np.frombuffer(o.block_bytes(4400 + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    rec = ro_c.encode_blocks(blocks, m, threads=8)
    d_o, d_r, op, rp = blocks.copy(), rec.copy(), [], []
    for b in range(n):
        # LowRate: survivors inside the 64-point sub-window (recovery 0..31), else W = 128
        pool = k + m if k > m else k + min(m, 32)
        keep = set(rng.sample(range(pool), k + rng.randint(0, min(4, pool - k))))
        if b % 9 == 4:
            keep |= set(range(k))  # nothing to restore in this block
        op += [1 if i in keep else 0 for i in range(k)]
        rp += [1 if k + j in keep else 0 for j in range(m)]
        for i in range(k):
            if i not in keep:
                d_o[b, i] = 0x5A
        for j in range(m):
            if k + j not in keep:
                d_r[b, j] = 0xA5
    got = gpu_decode(ctx, dev, d_o, d_r, op, rp, mode)
    assert np.array_equal(got, blocks)
    classes = rs.last_decode_classes(ctx)
    if mode == rs.DECODE_ANY_K or k > m:  # the LowRate sub-window is ANY_K only
        assert classes.get("window64", 0) > 0, classes


# --------------------------------------------- shard sizes that are not whole 64-byte chunks

@pytest.mark.parametrize("k,m,S", [(32, 32, 62), (32, 32, 1000), (32, 32, 1022), (32, 64, 1000), (32, 33, 1022),
                                   (16, 4, 1000), (64, 64, 200), (20, 30, 66), (32, 32, 2)])
def test_tail_chunk_encode_decode(ctx, dev, k, m, S):
    """S mod 64 != 0 (reed_solomon.rs:94-95: every slice whose padded payload is not a
    multiple of 2 KiB): restrided onto the bitsliced kernels.  Encode and decode (shared
    pattern with lost coding shreds, per-block random patterns, both modes) against the C
    oracle, which restates the crate's tail layout."""
    assert rs.has_fast_path(k, m, S)
    n = 7
    blocks = np.stack([np.frombuffer(o.block_bytes(3100 + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    rec = gpu_encode(ctx, dev, blocks, m)
    assert np.array_equal(rec, ro_c.encode_blocks(blocks, m, threads=8))
    other = np.stack([np.frombuffer(o.block_bytes(9100 + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    rng = random.Random(k * 10007 + m * 101 + S)
    for per_block in (False, True):
        op, rp = [], []
        d_o, d_r = blocks.copy(), rec.copy()
        for b in range(n if per_block else 1):
            keep = set(rng.sample(range(k + m), k + rng.randint(0, min(3, m))))
            op += [1 if i in keep else 0 for i in range(k)]
            rp += [1 if k + j in keep else 0 for j in range(m)]
        for b in range(n):
            pb = b if per_block else 0
            for i in range(k):
                if not op[pb * k + i]:
                    d_o[b, i] = 0x3C
            for j in range(m):
                if not rp[pb * m + j]:
                    d_r[b, j] = 0xC3
        for mode in (rs.DECODE_ANY_K, rs.DECODE_EXACT):
            # the restride staging buffer keeps its bytes between calls: fill it with another
            # codeword set first, so a decoder reading an absent (unpacked) slot would fail
            gpu_encode(ctx, dev, other, m)
            got = gpu_decode(ctx, dev, d_o, d_r, op, rp, mode)
            assert np.array_equal(got, blocks), (per_block, mode)


@pytest.mark.parametrize("S,n", [(1000, 1040), (1022, 1030), (62, 16400), (2, 40), (66, 8200), (126, 9000),
                                 (1000, 9), (574, 2000), (84, 300), (48, 6000), (110, 500), (2040, 600),
                                 (2000, 20)])
@pytest.mark.parametrize("k", [32, 25])
def test_tail_chunks_in_kernel(ctx, dev, S, n, k):
    """32-point geometries whose shards end in the crate's split tail chunk (S mod 64 != 0):
    encode and the full-recovery reconstruct read and write the tail in place (the TAIL
    transforms: xform<4> at >= 256 tiles, xform8 below; rs_xform.hpp tile_io_g), no restride
    (tails under 16 bytes still restride).
    Tails of T = 2..62 bytes (odd and even halves), against the C oracle and the originals;
    per-block random erasures (and erasures confined to shards 0..15: the pruned FFT).  S =
    1000, 2000, 2040: 16 / 32 chunks per shard with T % 8 == 0, the tile order of C/4-chunk runs
    (tile_io_g); S = 1022 and the rest: 16-chunk runs."""
    m = 32
    blocks = _blocks(7300 + S + k, n, k, S)
    rec = gpu_encode(ctx, dev, blocks, m)
    kern = rs.last_encode_kernels(ctx)
    if S % 64 >= 16:  # tails under 16 bytes keep the restride (a 16-byte tail window would leave the tail)
        assert "restride" not in kern and kern <= {"xform4", "xform8"}, kern
    assert np.array_equal(rec, ro_c.encode_blocks(blocks, m, threads=8))
    rng = random.Random(S * 7 + n + k)
    for low in (False, True):
        op = []
        for b in range(n):
            lost = set(rng.sample(range(min(k, 16) if low else k), rng.randint(1, min(k, 16) if low else k)))
            op += [0 if i in lost else 1 for i in range(k)]
        d_o = blocks.copy()
        for b in range(n):
            for i in range(k):
                if not op[b * k + i]:
                    d_o[b, i] = 0x5C
        got = gpu_decode(ctx, dev, d_o, rec, op, [1] * (m * n), rs.DECODE_ANY_K)
        assert np.array_equal(got, blocks), low
        assert set(rs.last_decode_classes(ctx)) <= {"transform", "none"}


@pytest.mark.parametrize("k,m,S", [(32, 64, 1024), (32, 33, 2048), (20, 40, 128), (32, 64, 4096), (25, 33, 192)])
def test_lowrate_window_decode(ctx, dev, k, m, S):
    """LowRate (CodingOnly 32:64, PETS 32:33, shredder.rs:362-446) with mixed losses and no
    full recovery chunk: any 32 survivors among the originals (plus their zero padding)
    and recovery shreds 0..31 decode in the 64-point sub-window; patterns that need
    recovery shreds past 31 take the table-driven decoder.  Per-block random patterns
    (tiles straddle blocks below 4 KiB), ANY_K, against the original data."""
    n = 12
    blocks = np.stack([np.frombuffer(o.block_bytes(4100 + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    rec = gpu_encode(ctx, dev, blocks, m)
    assert np.array_equal(rec, ro_c.encode_blocks(blocks, m, threads=8))
    rng = random.Random(k * 7 + m + S)
    d_o, d_r, op, rp = blocks.copy(), rec.copy(), [], []
    for b in range(n):
        if b % 4 == 3 and m > 32:   # k - 1 survivors inside the window, the rest past recovery 31
            keep_o = set(rng.sample(range(k), 2))
            keep_r = set(range(32, m)) | set(rng.sample(range(32), k - 3))
        else:
            w = min(m, 32)
            keep_o = set(rng.sample(range(k), rng.randint(max(0, k - w), k)))
            keep_r = set(rng.sample(range(w), min(w, k - len(keep_o) + rng.randint(0, 2))))
        op += [1 if i in keep_o else 0 for i in range(k)]
        rp += [1 if j in keep_r else 0 for j in range(m)]
        for i in range(k):
            if i not in keep_o:
                d_o[b, i] = 0x11
        for j in range(m):
            if j not in keep_r:
                d_r[b, j] = 0x22
    got = gpu_decode(ctx, dev, d_o, d_r, op, rp, rs.DECODE_ANY_K)
    assert np.array_equal(got, blocks)


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [0, 7])
def test_decoder_crate_api_exact_semantics(ctx, extra):
    """The per-call decoder (zero-copy path) keeps the crate's EXACT results on arbitrary
    bytes: with exactly k shards present (extra = 0) any bytes fix one codeword, so the ANY_K
    kernels it then uses must agree with the crate's decoder; with surplus shards (extra = 7)
    and one tampered recovery shard the crate's every-shard algorithm must be reproduced."""
    k, m, S = 32, 32, 1024
    rng = np.random.default_rng(90 + extra)
    orig = rng.integers(0, 256, (k, S), dtype=np.uint8)
    rec = ro_c.encode(orig, m)
    if extra:
        rec[3, 17] ^= 0x5A  # inconsistent input
    else:
        rec = rng.integers(0, 256, (m, S), dtype=np.uint8)  # not a codeword with orig at all
    op = np.zeros(k, np.uint8)
    op[rng.choice(k, 12, replace=False)] = 1
    rp = np.zeros(m, np.uint8)
    rp[rng.choice(m, k - 12 + extra, replace=False)] = 1
    damaged = (orig * op[:, None]).astype(np.uint8)
    want = ro_c.decode(damaged, op, rec, rp)
    dec = rs.ReedSolomonDecoder(ctx, k, m, S)
    for i in np.flatnonzero(op):
        dec.add_original_shard(int(i), orig[i].tobytes())
    for j in np.flatnonzero(rp):
        dec.add_recovery_shard(int(j), rec[j].tobytes())
    res = dec.decode()
    assert sorted(res) == sorted(int(i) for i in np.flatnonzero(op == 0))
    for i, b in res.items():
        assert b == want[i].tobytes(), i


@pytest.mark.gpu
def test_crate_api_back_to_back_calls_see_fresh_bytes(ctx):
    """The per-call paths reuse one zero-copy staging buffer: consecutive calls with
    different bytes must each see their own (no stale cached copy of the previous call)."""
    k, m, S = 32, 32, 1024
    rng = np.random.default_rng(7)
    enc = rs.ReedSolomonEncoder(ctx, k, m, S)
    dec = rs.ReedSolomonDecoder(ctx, k, m, S)
    for it in range(6):
        orig = rng.integers(0, 256, (k, S), dtype=np.uint8)
        enc.reset(k, m, S)
        for i in range(k):
            enc.add_original_shard(orig[i].tobytes())
        rec = enc.encode()
        want = ro_c.encode(orig, m)
        assert [bytes(r) for r in rec] == [want[j].tobytes() for j in range(m)], it
        dec.reset(k, m, S)
        for j in range(m):
            dec.add_recovery_shard(j, want[j].tobytes())
        res = dec.decode()
        assert all(res[i] == orig[i].tobytes() for i in range(k)), it


# ------------------------------------------------ buffers at any alignment, odd strides

@pytest.mark.parametrize("k,m,S,shift,pad", [(32, 32, 1024, 2, 0), (32, 32, 1024, 8, 16), (32, 32, 1000, 0, 0),
                                             (32, 32, 1000, 6, 2), (16, 4, 1024, 4, 2), (32, 64, 1000, 2, 0),
                                             (64, 64, 192, 10, 4), (32, 32, 1024, 1, 1), (32, 32, 1022, 3, 0),
                                             (20, 30, 130, 2, 6)])
def test_unaligned_codewords(ctx, dev, k, m, S, shift, pad):
    """Codeword buffers at a byte offset `shift` with block stride (k + m) S + pad: the whole
    64-byte chunks run in place on the bitsliced kernels (any even alignment), the tail bytes
    (S mod 64) and byte-odd layouts go through the restride.  Encode against the C oracle;
    per-block random erasures (both modes), absent shards filled with garbage, against the
    originals."""
    n = 9
    stride = (k + m) * S + pad
    blocks = np.stack([np.frombuffer(o.block_bytes(7100 + b, k * S), np.uint8).reshape(k, S) for b in range(n)])
    want = ro_c.encode_blocks(blocks, m, threads=8)
    img = np.full(n * stride + shift + 64, 0xEE, np.uint8)
    for b in range(n):
        img[shift + b * stride: shift + b * stride + k * S] = blocks[b].reshape(-1)
    d = to_dev(img, dev)
    base = d.data_ptr() + shift
    rs.encode_batch(ctx, k, m, S, n, base, stride, base + k * S, stride)
    got = d.cpu().numpy()
    for b in range(n):
        cwb = got[shift + b * stride: shift + b * stride + (k + m) * S].reshape(k + m, S)
        assert np.array_equal(cwb[k:], want[b]), b
        assert np.array_equal(cwb[:k], blocks[b]), b
    assert np.all(got[:shift] == 0xEE) and np.all(got[shift + (n - 1) * stride + (k + m) * S:] == 0xEE)
    rng = random.Random(S * 7 + shift)
    for mode in (rs.DECODE_ANY_K, rs.DECODE_EXACT):
        op, rp = [], []
        img2 = got.copy()
        for b in range(n):
            keep = set(rng.sample(range(k + m), k + rng.randint(0, min(2, m))))
            op += [1 if i in keep else 0 for i in range(k)]
            rp += [1 if k + j in keep else 0 for j in range(m)]
            for s in range(k + m):
                if s not in keep:
                    o0 = shift + b * stride + s * S
                    img2[o0:o0 + S] = 0x5A
        d2 = to_dev(img2, dev)
        base = d2.data_ptr() + shift
        rs.decode_batch(ctx, k, m, S, n, base, stride, base + k * S, stride, op, rp, mode=mode)
        out = d2.cpu().numpy()
        for b in range(n):
            assert np.array_equal(out[shift + b * stride: shift + b * stride + k * S].reshape(k, S), blocks[b]), (b, mode)


# ------------------------------------------------ W = 128 windows (two 64-point passes)

def _w128_case(k, m, S, n, per_block, rng, lose_originals=None, lose_coding=None):
    blocks = np.stack([np.frombuffer(o.block_bytes(11000 + 97 * k + m + b, k * S), np.uint8).reshape(k, S)
                       for b in range(n)])
    rec = ro_c.encode_blocks(blocks, m, threads=8)
    op, rp = [], []
    d_o, d_r = blocks.copy(), rec.copy()
    for b in range(n if per_block else 1):
        lo = lose_originals if lose_originals is not None else rng.randint(1, k)
        lc = lose_coding if lose_coding is not None else m - (k - (k - lo)) - rng.randint(0, 2)
        lc = max(0, min(lc, m - lo))
        lost_o = set(rng.sample(range(k), lo))
        lost_r = set(rng.sample(range(m), lc))
        op += [0 if i in lost_o else 1 for i in range(k)]
        rp += [0 if j in lost_r else 1 for j in range(m)]
    for b in range(n):
        pb = b if per_block else 0
        for i in range(k):
            if not op[pb * k + i]:
                d_o[b, i] = 0x6B
        for j in range(m):
            if not rp[pb * m + j]:
                d_r[b, j] = 0xB6
    return blocks, d_o, d_r, op, rp


@pytest.mark.parametrize("k,m,S,n,per_block,lo,lc", [
    (32, 64, 1024, 96, True, 32, None),    # CodingOnly: every data shred lost, random 32 of 64 coding
    (32, 64, 1024, 48, True, None, None),  # CodingOnly mixed losses across both recovery chunks
    (64, 64, 4096, 6, True, 16, 8),        # 64:64, 8 lost coding shreds, per-block patterns
    (64, 64, 4096, 6, False, 16, 16),      # 64:64, 16 lost coding shreds, one pattern
    (64, 64, 1024, 40, True, 32, 12),      # 64:64 on 1 KiB shards: per-lane patterns
    (40, 64, 2048, 10, True, 20, 10),      # HighRate, originals at 64..103
    (20, 80, 2048, 10, True, 20, None),    # LowRate chunk 32, recovery up to position 111
])
def test_window128_decode(ctx, dev, k, m, S, n, per_block, lo, lc):
    """W = 128 windows (CodingOnly 32:64 arrival across both recovery chunks, 64:64 with lost
    coding shreds, LowRate past 64 positions) on the bitsliced two-pass decoder, ANY_K (and
    EXACT with exactly k survivors), absent shards filled with garbage, against the originals;
    the decode-class record shows the two-pass window served every pattern."""
    rng = random.Random(k * 1000 + m * 10 + S)
    blocks, d_o, d_r, op, rp = _w128_case(k, m, S, n, per_block, rng, lo, lc)
    got = gpu_decode(ctx, dev, d_o, d_r, op, rp, rs.DECODE_ANY_K)
    assert np.array_equal(got, blocks)
    classes = rs.last_decode_classes(ctx)
    assert set(classes) <= {"window128", "none", "correction", "window64"} and classes.get("window128", 0) > 0, classes
    # EXACT with exactly k survivors per pattern: the same kernels, the crate's bytes
    op2, rp2 = list(op), list(rp)
    for b in range(len(op) // k):
        surplus = sum(op2[b * k:(b + 1) * k]) + sum(rp2[b * m:(b + 1) * m]) - k
        for j in reversed(range(m)):
            if surplus and rp2[b * m + j]:
                rp2[b * m + j] = 0
                surplus -= 1
    got = gpu_decode(ctx, dev, d_o, d_r, op2, rp2, rs.DECODE_EXACT)
    assert np.array_equal(got, blocks)


@pytest.mark.parametrize("k,m", [(64, 64), (32, 64)])
def test_window128_per_block_mixed_classes(ctx, dev, k, m):
    """Per-block patterns on whole-tile shards (S = 4096: one pattern per tile) where only some
    blocks need the W = 128 window and the others decode by another class (nothing lost, the
    full recovery set, a W = 64 window): the window128 launch covers exactly its blocks' tiles
    (a zero-tile launch here once left their erased originals unrestored with status OK)."""
    S, n = 4096, 9
    rng = random.Random(128 * k + m)
    blocks = np.stack([np.frombuffer(o.block_bytes(31000 + 7 * k + b, k * S), np.uint8).reshape(k, S)
                       for b in range(n)])
    rec = ro_c.encode_blocks(blocks, m, threads=8)
    d_o, d_r = blocks.copy(), rec.copy()
    op, rp = [], []
    for b in range(n):
        kind = b % 3
        if kind == 0:    # W = 128: fewer than k survivors within the first 64 window positions
            if k == 64:  # HighRate 64:64: any lost coding shred with lost originals
                lost_o, lost_r = set(rng.sample(range(k), 16)), set(rng.sample(range(m), 8))
            else:        # LowRate 32:64: originals + first recovery chunk hold 24 < 32 survivors,
                         # and the second chunk is incomplete (no single-chunk decode)
                lost_o = set(rng.sample(range(k), 24))
                lost_r = set(rng.sample(range(32), 16)) | set(rng.sample(range(32, 64), 2))
        elif kind == 1:  # nothing lost, or only originals with the whole recovery set present
            lost_o = set(rng.sample(range(k), k // 4)) if b % 2 else set()
            lost_r = set()
        else:            # a few originals and a few coding shreds: whatever small class fits
            lost_o = set(rng.sample(range(k), 2))
            lost_r = set(rng.sample(range(m), 2))
        op += [0 if i in lost_o else 1 for i in range(k)]
        rp += [0 if j in lost_r else 1 for j in range(m)]
        for i in lost_o:
            d_o[b, i] = 0x6B
        for j in lost_r:
            d_r[b, j] = 0xB6
    got = gpu_decode(ctx, dev, d_o, d_r, op, rp, rs.DECODE_ANY_K)
    assert np.array_equal(got, blocks)
    classes = rs.last_decode_classes(ctx)
    assert classes.get("window128", 0) > 0 and len([c for c, v in classes.items() if v and c != "window128"]) > 0, classes


@pytest.mark.gpu
def test_per_call_server_jobs_and_restart(ctx):
    """The resident per-call server (latency_server_kernel): back-to-back shreds and
    coding-only deshreds of 32:32 slices with S % 64 == 0 run as mailbox jobs, other sizes take
    the launch path in between, and calls after a gap longer than the server's 20 ms idle
    timeout restart it -- every result against the oracle."""
    import time

    coder = rs.ReedSolomonCoder(ctx, 32)
    rng = random.Random(4242)
    sizes = [32767, 32704, 2047, 4095, 1000, 16383, 63, 0, 20000, 31999, 32700, 30999]
    jobs0 = rs.server_jobs(ctx)
    pk_calls = 0
    for i in range(45):
        payload = o.splitmix64_bytes(5000 + i, sizes[i % len(sizes)])
        raw = coder.shred(payload)
        exp = o.coder_shred(payload, 32)
        assert raw.data == exp.data and raw.coding == exp.coding, (i, len(payload))
        got, raw2 = coder.deshred([None] * 32 + [(False, c) for c in raw.coding])
        assert got == payload and raw2.coding == exp.coding, (i, len(payload))
        # random arrival: exactly 32 of 64 (S = 1 KiB or 960 + T: the server's decode_pk job, data
        # and coding restored in one job), and a surplus set (launch path)
        for cnt in (32, 40):
            keep = sorted(rng.sample(range(64), cnt))
            shreds = [((j < 32), (raw.data + raw.coding)[j]) if j in keep else None for j in range(64)]
            before = rs.server_jobs(ctx)["decode_pk"]
            got, raw3 = coder.deshred(shreds)
            assert got == payload and raw3.data == exp.data and raw3.coding == exp.coding, (i, keep)
            served = rs.server_jobs(ctx)["decode_pk"] - before
            lost = set(range(64)) - set(keep)
            S = len(raw.data[0])  # 1 KiB, or 960 + T with a T-byte tail (S = 1000, 1022, 970)
            pk_size = S == 1024 or 960 < S < 1024
            fits = (cnt == 32 and pk_size and any(j < 32 for j in lost)
                    and any(j >= 32 for j in lost))  # else: no decode, or the coding-only transform
            assert served == (1 if fits else 0), (i, cnt, len(raw.data[0]))
            pk_calls += served
        if i % 15 == 14:
            time.sleep(0.06)  # the server idles out; the next call relaunches it
    assert pk_calls >= 8
    # the crate-API decoder (INTEGRATION.md Route A) from a random 32 of 64: the same job, on a
    # fresh context whose first call is that job (the server needs the device tables)
    fctx = rs.Context(0)
    dec = rs.ReedSolomonDecoder(fctx, 32, 32, 1024)
    for it in range(6):
        orig = _shards(900 + it, 32, 1024)
        rec = o.encode(orig, 32)
        dec.reset(32, 32, 1024)
        keep = set(rng.sample(range(64), 32))
        for j in sorted(keep):
            if j < 32:
                dec.add_original_shard(j, orig[j])
            else:
                dec.add_recovery_shard(j - 32, rec[j - 32])
        before = rs.server_jobs(fctx)["decode_pk"]
        res = dec.decode()
        assert sorted(res) == [i for i in range(32) if i not in keep]
        assert all(res[i] == orig[i] for i in res), it
        pk = 0 < len(res) < 32 or (len(res) == 32 and keep != set(range(32, 64)))
        assert rs.server_jobs(fctx)["decode_pk"] - before == (1 if pk else 0)
        if pk:
            assert rs.last_decode_classes(fctx) == {"server_window64": 1}
    del dec
    fctx.close()


def test_server_timeout_abandons_staging_safely(ctx):  # ctx: torch initialises the device first
    """a per-call server job that times out abandons the pinned staging it named.
    The encoder / decoder that owned it must then drop its received shards and take a fresh
    buffer -- a retry without reset returns an error instead of handing null staging to the
    device, later adds land in the new buffer, and the context falls back to the launch path
    (results against the oracle).  The timeout is injected (ag_rs_internal_fail_next_server_job)."""
    k = m = 32
    S = 1024
    orig = _shards(777, k, S)
    rec = o.encode(orig, m)

    ectx = rs.Context(0)
    enc = rs.ReedSolomonEncoder(ectx, k, m, S)
    for s in orig:
        enc.add_original_shard(s)
    rs.fail_next_server_job(ectx)
    with pytest.raises(rs.RSError) as e:
        enc.encode()
    assert e.value.status == 102  # AG_RS_ERR_DEVICE
    with pytest.raises(rs.RSError) as e:  # retry without reset: the shards were dropped
        enc.encode()
    assert e.value.kind == "TooFewOriginalShards"
    for it in range(2):
        for s in orig:
            enc.add_original_shard(s)
        assert enc.encode() == rec, it  # launch path from now on

    dctx = rs.Context(0)
    dec = rs.ReedSolomonDecoder(dctx, k, m, S)
    for j in range(m):
        dec.add_recovery_shard(j, rec[j])
    rs.fail_next_server_job(dctx)
    with pytest.raises(rs.RSError) as e:
        dec.decode()
    assert e.value.status == 102
    with pytest.raises(rs.RSError) as e:
        dec.decode()
    assert e.value.kind == "NotEnoughShards"
    for j in range(m):
        dec.add_recovery_shard(j, rec[j])
    res = dec.decode()
    assert sorted(res) == list(range(k)) and all(res[i] == orig[i] for i in res)

    cctx = rs.Context(0)
    coder = rs.ReedSolomonCoder(cctx, 32)
    payload = o.splitmix64_bytes(99, 32767)  # S = 1024: a server job
    rs.fail_next_server_job(cctx)
    with pytest.raises(rs.RSError):
        coder.shred(payload)
    raw = coder.shred(payload)
    exp = o.coder_shred(payload, 32)
    assert raw.data == exp.data and raw.coding == exp.coding
    got, _ = coder.deshred([None] * 32 + [(False, c) for c in raw.coding])
    assert got == payload
    del enc, dec, coder
    for c in (ectx, dctx, cctx):
        c.close()
