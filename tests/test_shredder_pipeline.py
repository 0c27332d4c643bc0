"""The composed Shredder on the GPU (ag_shredder_shred_batch / ag_shredder_deshred_batch)
against the CPU composition of the reference's RegularShredder (oracle/shredder_oracle.py,
itself built from the pinned or restated oracle of every stage).  Byte-exact: datagrams,
raw shreds, payloads, per-slice errors.

Reference: /root/reference/src/shredder.rs:282-345 (shred / deshred), :533-625 (output
shreds, fill_missing_shreds, check_merkle_tree), validated_shred.rs:52-81 (receiver checks).
"""

import random

import numpy as np
import pytest

import ed25519_oracle as ed
import rs_oracle as o
import shred_wire_oracle as wire
import shredder_oracle as so
import slice_oracle as sl
from alpenglow_amd import rs

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

PKT = 1536  # datagram slot stride (>= 1325 bytes for a 1 KiB shred)
SEED = bytes(range(7, 39))


@pytest.fixture(scope="module")
def dev(ctx):
    d = torch.device("cuda:0")
    s = torch.cuda.Stream(d)
    torch.cuda.set_stream(s)
    ctx.set_stream(s.cuda_stream)
    return d


def _dev(a, dev):
    return torch.from_numpy(np.array(a, copy=True)).to(dev)


def _slices(rng, n, S):
    """n slices whose framed payloads all pad to shred size S (Slice::payload_bytes)."""
    lo, hi = 32 * S - 64, 32 * S - 1  # framed lengths with padded size 32 * S
    out = []
    for i in range(n):
        parent = (rng.randrange(1 << 40), bytes(rng.randrange(256) for _ in range(32))) if i % 2 else None
        framed = rng.randrange(max(lo, sl.header_len(parent)), min(hi, sl.MAX_DATA_PER_SLICE) + 1)
        data = bytes(rng.randrange(256) for _ in range(framed - sl.header_len(parent)))
        out.append((parent, data, rng.randrange(1 << 32), rng.randrange(1024), bool(i % 3 == 2)))
    return out


def _gpu_shred(ctx, dev, slices, S):
    n = len(slices)
    maxd = max(len(d) for _, d, *_ in slices)
    data = np.zeros((n, maxd), np.uint8)
    for b, (_, d, *_r) in enumerate(slices):
        data[b, :len(d)] = np.frombuffer(d, np.uint8)
    d_data = _dev(data, dev)
    slots = _dev(np.array([s[2] for s in slices], np.uint64), dev)
    sidx = _dev(np.array([s[3] for s in slices], np.uint64), dev)
    last = _dev(np.array([s[4] for s in slices], np.uint8), dev)
    seed = _dev(np.frombuffer(SEED, np.uint8), dev)
    pk = _dev(np.frombuffer(ed.secret_to_public(SEED), np.uint8), dev)
    cw = torch.zeros((n, 64 * S), dtype=torch.uint8, device=dev)
    pk_buf = torch.zeros((n * 64, PKT), dtype=torch.uint8, device=dev)
    lens = torch.zeros(n * 64, dtype=torch.int32, device=dev)
    roots = torch.zeros((n, 32), dtype=torch.uint8, device=dev)
    sigs = torch.zeros((n, 64), dtype=torch.uint8, device=dev)
    rs.shredder_shred_batch(ctx, n, S, [s[0] for s in slices], d_data, maxd, [len(s[1]) for s in slices], slots, sidx,
                            last, seed, pk, cw, pk_buf, PKT, lens, roots_out=roots, sigs_out=sigs)
    torch.cuda.synchronize()
    return cw, pk_buf, lens, roots, sigs, pk


def _packets(pk_buf, lens, n):
    p, ln = pk_buf.cpu().numpy(), lens.cpu().numpy()
    return [[p[b * 64 + j, :ln[b * 64 + j]].tobytes() for j in range(64)] for b in range(n)]


@pytest.mark.parametrize("S,n", [(1024, 5), (64, 6), (2, 3)])
def test_shred_batch_matches_oracle(ctx, dev, S, n):
    """RegularShredder::shred: framing, RS, Merkle, signature, datagrams (data shreds first)."""
    rng = random.Random(S * 31 + n)
    slices = _slices(rng, n, S)
    cw, pk_buf, lens, roots, sigs, _ = _gpu_shred(ctx, dev, slices, S)
    got = _packets(pk_buf, lens, n)
    cwh = cw.cpu().numpy()
    for b, (parent, data, slot, si, last) in enumerate(slices):
        want, raw, root, sig = so.shred(parent, data, slot, si, last, SEED)
        assert roots[b].cpu().numpy().tobytes() == root
        assert sigs[b].cpu().numpy().tobytes() == sig
        assert cwh[b].tobytes() == b"".join(raw.data + raw.coding)
        assert got[b] == want, b


def _deshred(ctx, dev, rows, pk, S):
    """rows: per slice 64 datagrams or None (absent)."""
    n = len(rows)
    buf = np.zeros((n * 64, PKT), np.uint8)
    ln = np.zeros(n * 64, np.int32)
    for b, r in enumerate(rows):
        for j, p in enumerate(r):
            if p is not None:
                buf[b * 64 + j, :len(p)] = np.frombuffer(p, np.uint8)
                ln[b * 64 + j] = len(p)
    d_buf, d_ln = _dev(buf, dev), _dev(ln, dev)
    cw = torch.zeros((n, 64 * S), dtype=torch.uint8, device=dev)
    res = rs.shredder_deshred_batch(ctx, n, S, d_buf, PKT, d_ln, pk, cw)
    return res, _packets(d_buf, d_ln, n), cw.cpu().numpy()


def _expect(rows, pk_bytes, S):
    """The oracle's verdict for every slice: receive (the receiver's checks) + Shredder::deshred
    with the crate's decoder over every kept shred, and the datagram slots after the call
    (kept ones as received, the others filled for a successful slice, untouched otherwise)."""
    out = []
    for r in rows:
        kept = so.receive(r, pk_bytes, S)
        st, res = so.deshred(kept)
        if st == so.OK:
            slots = [r[j] if kept[j] is not None else res["datagrams"][j] for j in range(64)]
        else:
            slots = [x if x is not None else b"" for x in r]
        out.append((st, res, slots))
    return out


def _check_against_oracle(res, out, cw, want):
    assert res.status.tolist() == [w[0] for w in want], \
        ([rs.STATUS_KIND.get(int(x), int(x)) for x in res.status], [w[0] for w in want])
    for b, (st, r, slots) in enumerate(want):
        assert out[b] == slots, b
        if st != so.OK:
            continue
        assert (int(res.slots[b]), int(res.slice_indices[b]), bool(res.is_last[b])) == r["header"]
        assert res.parents[b] == r["parent"]
        off, n = int(res.data_offsets[b]), int(res.data_lens[b])
        assert cw[b, off:off + n].tobytes() == r["data"]
        assert cw[b].tobytes() == b"".join(r["raw"].data + r["raw"].coding)


def _non_codeword(slice_, tamper):
    """The 64 datagrams of a leader that signs shreds which are no codeword: the slice's raw
    shreds with shred `tamper` altered after encoding."""
    p, d, slot, si, last = slice_
    raw = o.coder_shred(sl.payload_bytes(p, d), 32)
    shards = list(raw.data) + list(raw.coding)
    shards[tamper] = bytes(x ^ 0x5A for x in shards[tamper])
    return so.datagrams(shards[:32], shards[32:], slot, si, last, SEED)[0]


def test_deshred_batch_matches_oracle(ctx, dev):
    """Shredder::deshred behind the receiver's checks, one slice per outcome, the expected
    verdicts and bytes from the oracle (oracle/shredder_oracle.py: receive + deshred with the
    crate's decoder over every kept shred): all present, a random half, 31 shreds, a tampered
    datagram (dropped), leaders signing non-codewords (with the inconsistent shred withheld,
    held together with surplus shreds so that decoding from all kept shreds and from any 32
    of them disagree, and held with the last data shred present), a payload that is no
    SlicePayload and one without padding marker, a datagram in the wrong slot, a shred signed
    by another key.  Failed slices keep their datagrams; successful ones get every missing
    datagram, byte-exact."""
    S = 1024
    rng = random.Random(77)
    slices = _slices(rng, 12, S)
    clean = [so.shred(p, d, slot, si, last, SEED) for p, d, slot, si, last in slices]
    rows = [list(c[0]) for c in clean]
    keep = [None] * 12
    # 1: a random half; 2: 31 shreds; 3: 40 shreds, one tampered
    for b, cnt in ((1, 32), (2, 31), (3, 40)):
        keep[b] = set(rng.sample(range(64), cnt))
    t = sorted(keep[3])[5]
    bad = bytearray(rows[3][t])
    bad[40] ^= 1  # payload byte: the Merkle path no longer derives the signed root
    rows[3][t] = bytes(bad)
    # 4: the leader signs shreds that are no codeword; the receiver lacks the odd one
    rows[4] = _non_codeword(slices[4], 40)
    keep[4] = set(range(64)) - {40}
    # 5: valid padding, but the payload is no SlicePayload (Option tag 7)
    payload5 = b"\x07" + bytes(rng.randrange(256) for _ in range(32705))  # pads to S = 1024
    raw5 = o.coder_shred(payload5, 32)
    rows[5], _, _ = so.datagrams(raw5.data, raw5.coding, slices[5][2], slices[5][3], slices[5][4], SEED)
    # 6: no 0x80 marker before the trailing zeros (InvalidPadding)
    data6 = [bytes(rng.randrange(256) for _ in range(S)) for _ in range(32)]
    data6[31] = data6[31][:-1] + b"\x55"
    rows[6], _, _ = so.datagrams(data6, o.encode(data6, 32), slices[6][2], slices[6][3], slices[6][4], SEED)
    keep[6] = set(rng.sample(range(64), 48))
    # 7: datagram of shred 3 placed in slot 4 (slot 3 empty)
    keep[7] = set(range(64)) - {3}
    rows[7][4] = rows[7][3]
    # 8: shred 0 signed by another key (the first shred checked: no cached commitment)
    seed8 = bytes(range(100, 132))
    other, _, _ = so.datagrams(clean[8][1].data, clean[8][1].coding, slices[8][2], slices[8][3], slices[8][4], seed8)
    rows[8][0] = other[0]
    # 9: non-codeword (coding shred 62 altered) held by the receiver with data shreds 16..31
    #    missing: any 32 survivors (data 0..15 + coding 32..47) restore the honest data, which
    #    pads fine and then fails the Merkle check; the crate decodes from all 48 and restores
    #    other bytes, whose padding decides first
    rows[9] = _non_codeword(slices[9], 62)
    keep[9] = set(range(16)) | set(range(32, 64))
    # 10: the same with the last data shred held (data 8..23 missing): padding on received bytes
    rows[10] = _non_codeword(slices[10], 62)
    keep[10] = (set(range(8)) | set(range(24, 32))) | set(range(32, 64))
    # 11: the leader altered data shred 5; the receiver holds it and 40 others
    rows[11] = _non_codeword(slices[11], 5)
    keep[11] = {5} | set(rng.sample([j for j in range(64) if j != 5], 40))
    inp = [[r[j] if keep[b] is None or j in keep[b] else None for j in range(64)] for b, r in enumerate(rows)]
    pk_bytes = ed.secret_to_public(SEED)
    want = _expect(inp, pk_bytes, S)
    assert [w[0] for w in want][:9] == [0, 0, 9, 0, 24, 23, 23, 0, 0]  # the outcomes named above
    assert want[9][0] == 23 and want[10][0] == 24  # the crate's decoder decides case 9
    pk = _dev(np.frombuffer(pk_bytes, np.uint8), dev)
    res, out, cw = _deshred(ctx, dev, inp, pk, S)
    _check_against_oracle(res, out, cw, want)


# S = 1024: the fused window decode with the coding restore (decode_pk<-1>); S = 512 / 64:
# whole-chunk shreds on the other window decoders, whose exactly-32 slices re-encode only the
# absent coding shreds (store mask ~present) and whose Merkle rebuild reuses the proof check's
# leaf digests for kept rows; S = 2: a tail-only shred (S % 64 != 0: every coding shred
# re-encoded, the LIST leaf kernel) -- ADVICE r5.
@pytest.mark.parametrize("S", [1024, 512, 64, 2, 1000])
def test_deshred_batch_adversarial_random(ctx, dev, S):
    """24 slices, about half of them from a leader that altered one random shred after
    encoding, each received as a random 32..64 of its datagrams (every fourth slice exactly
    32): verdicts, filled datagrams and raw shreds equal the oracle's (every kept shred through
    the crate's decoder)."""
    rng = random.Random(2024 + S)
    slices = _slices(rng, 24, S)
    inp = []
    for b, sl_ in enumerate(slices):
        rows = _non_codeword(sl_, rng.randrange(64)) if b % 2 else so.shred(*sl_[:5], SEED)[0]
        keep = set(rng.sample(range(64), 32 if b % 4 < 2 else rng.randrange(32, 65)))
        inp.append([rows[j] if j in keep else None for j in range(64)])
    pk_bytes = ed.secret_to_public(SEED)
    want = _expect(inp, pk_bytes, S)
    pk = _dev(np.frombuffer(pk_bytes, np.uint8), dev)
    res, out, cw = _deshred(ctx, dev, inp, pk, S)
    _check_against_oracle(res, out, cw, want)


@pytest.mark.parametrize("S", [1024, 512, 64, 2, 1000])
def test_pipeline_roundtrip_random_arrival(ctx, dev, S):
    """shred_batch -> a random 32..64 of each slice's datagrams (every other slice exactly 32)
    -> deshred_batch restores every payload and every datagram (256 slices of shred size S)."""
    n = 256
    rng = random.Random(5 + S)
    slices = _slices(rng, n, S)
    cw, pk_buf, lens, _, _, pk = _gpu_shred(ctx, dev, slices, S)
    full = _packets(pk_buf, lens, n)
    inp = []
    for b in range(n):
        keep = set(rng.sample(range(64), 32 if b % 2 else rng.randrange(32, 65)))
        inp.append([full[b][j] if j in keep else None for j in range(64)])
    res, out, cw2 = _deshred(ctx, dev, inp, pk, S)
    assert (res.status == 0).all()
    assert out == full
    assert np.array_equal(cw2, cw.cpu().numpy())
    for b, (parent, data, *_r) in enumerate(slices):
        off, ln = int(res.data_offsets[b]), int(res.data_lens[b])
        assert res.parents[b] == parent and cw2[b, off:off + ln].tobytes() == data


# ---- the other shredders: CodingOnly, PETS, AONT (ag_shredder_*_batch_kind) ----------------

KINDS = [so.CODING_ONLY, so.PETS, so.AONT]


def _stride(kind, S):
    return (32 + so.CODING[kind]) * S + 12  # a padded codeword stride (multiple of 4, not of S)


def _slices_kind(rng, n, S, kind):
    """n slices whose framed payloads (+ the 16-byte key tail for PETS / AONT) pad to S."""
    extra = 16 if kind in (so.PETS, so.AONT) else 0
    lo, hi = 32 * S - 64 - extra, 32 * S - 1 - extra
    out = []
    for i in range(n):
        parent = (rng.randrange(1 << 40), bytes(rng.randrange(256) for _ in range(32))) if i % 2 else None
        framed = rng.randrange(max(lo, sl.header_len(parent)), min(hi, sl.MAX_DATA_PER_SLICE - extra) + 1)
        data = bytes(rng.randrange(256) for _ in range(framed - sl.header_len(parent)))
        out.append((parent, data, rng.randrange(1 << 32), rng.randrange(1024), bool(i % 3 == 2),
                    bytes(rng.randrange(256) for _ in range(16))))
    return out


def _gpu_shred_kind(ctx, dev, kind, slices, S):
    n = len(slices)
    maxd = max(len(d) for _, d, *_ in slices)
    data = np.zeros((n, maxd), np.uint8)
    for b, s_ in enumerate(slices):
        data[b, :len(s_[1])] = np.frombuffer(s_[1], np.uint8)
    stride = _stride(kind, S)
    cw = torch.zeros((n, stride), dtype=torch.uint8, device=dev)
    pk_buf = torch.zeros((n * 64, PKT), dtype=torch.uint8, device=dev)
    lens = torch.zeros(n * 64, dtype=torch.int32, device=dev)
    roots = torch.zeros((n, 32), dtype=torch.uint8, device=dev)
    sigs = torch.zeros((n, 64), dtype=torch.uint8, device=dev)
    pk = _dev(np.frombuffer(ed.secret_to_public(SEED), np.uint8), dev)
    keys = _dev(np.frombuffer(b"".join(s_[5] for s_ in slices), np.uint8), dev)
    rs.shredder_shred_batch_kind(ctx, kind, n, S, [s_[0] for s_ in slices], _dev(data, dev), maxd,
                                 [len(s_[1]) for s_ in slices], _dev(np.array([s_[2] for s_ in slices], np.uint64), dev),
                                 _dev(np.array([s_[3] for s_ in slices], np.uint64), dev),
                                 _dev(np.array([s_[4] for s_ in slices], np.uint8), dev),
                                 _dev(np.frombuffer(SEED, np.uint8), dev), pk, keys, cw, stride, pk_buf, PKT, lens,
                                 roots_out=roots, sigs_out=sigs)
    torch.cuda.synchronize()
    return cw, pk_buf, lens, roots, sigs, pk


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("S", [1024, 64])
def test_shred_batch_kind_matches_oracle(ctx, dev, kind, S):
    """CodingOnlyShredder / PetsShredder / AontShredder::shred (shredder.rs:361-500) composed on
    the device: datagrams (the shredder's data / coding layout), roots and signatures byte-exact
    against the oracle composition with the same keys."""
    rng = random.Random(S * 7 + kind)
    slices = _slices_kind(rng, 5, S, kind)
    cw, pk_buf, lens, roots, sigs, _ = _gpu_shred_kind(ctx, dev, kind, slices, S)
    got = _packets(pk_buf, lens, len(slices))
    for b, (parent, data, slot, si, last, key) in enumerate(slices):
        want, raw, root, sig = so.shred_kind(kind, parent, data, slot, si, last, SEED, key)
        assert roots[b].cpu().numpy().tobytes() == root, b
        assert sigs[b].cpu().numpy().tobytes() == sig, b
        assert got[b] == want, b


def _deshred_kind(ctx, dev, kind, rows, pk, S):
    n = len(rows)
    buf = np.zeros((n * 64, PKT), np.uint8)
    ln = np.zeros(n * 64, np.int32)
    for b, r in enumerate(rows):
        for j, p in enumerate(r):
            if p is not None:
                buf[b * 64 + j, :len(p)] = np.frombuffer(p, np.uint8)
                ln[b * 64 + j] = len(p)
    d_buf, d_ln = _dev(buf, dev), _dev(ln, dev)
    stride = _stride(kind, S)
    cw = torch.zeros((n, stride), dtype=torch.uint8, device=dev)
    res = rs.shredder_deshred_batch_kind(ctx, kind, n, S, d_buf, PKT, d_ln, pk, cw, stride)
    return res, _packets(d_buf, d_ln, n), cw.cpu().numpy()


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("S", [1024, 64, 1000])
def test_deshred_batch_kind_matches_oracle(ctx, dev, kind, S):
    """Shredder::deshred of the other three shredders behind the receiver's checks: 12 slices,
    every third from a leader that altered one shred after encoding, each received as a random
    32..64 of its datagrams (every other one exactly 32), one with 31 shreds and one with a
    tampered datagram; verdicts, filled datagrams and the parsed payload equal the oracle's
    (receive with the shredder's layout + deshred_kind: the crate's decoder over every kept
    shred, decrypt_payload, check_merkle_tree, SlicePayload)."""
    rng = random.Random(S * 11 + kind)
    slices = _slices_kind(rng, 12, S, kind)
    nd = so.DATA_OUT[kind]
    pk_bytes = ed.secret_to_public(SEED)
    inp = []
    for b, (parent, data, slot, si, last, key) in enumerate(slices):
        rows, raw, _, _ = so.shred_kind(kind, parent, data, slot, si, last, SEED, key)
        if b % 3 == 1:  # a leader that signs a non-codeword
            t = rng.randrange(64)
            shards = list(raw.data) + list(raw.coding)
            shards[t] = bytes(x ^ 0x5A for x in shards[t])
            rows = so.datagrams(shards[:nd], shards[nd:], slot, si, last, SEED)[0]
        cnt = 31 if b == 4 else 32 if b % 2 == 0 else rng.randrange(32, 65)
        keep = set(rng.sample(range(64), cnt))
        row = [rows[j] if j in keep else None for j in range(64)]
        if b == 6:
            t = sorted(keep)[3]
            bad = bytearray(row[t])
            bad[40] ^= 1  # no longer derives the signed root: dropped by the receiver
            row[t] = bytes(bad)
        inp.append(row)
    want = []
    for r in inp:
        kept = so.receive(r, pk_bytes, S, nd)
        st, res = so.deshred_kind(kept, kind)
        slots = ([r[j] if kept[j] is not None else res["datagrams"][j] for j in range(64)] if st == so.OK
                 else [x if x is not None else b"" for x in r])
        want.append((st, res, slots))
    assert want[4][0] == so.NOT_ENOUGH_SHARDS and sum(w[0] == so.OK for w in want) >= 6
    pk = _dev(np.frombuffer(pk_bytes, np.uint8), dev)
    res, out, cw = _deshred_kind(ctx, dev, kind, inp, pk, S)
    assert res.status.tolist() == [w[0] for w in want]
    stride = _stride(kind, S)
    for b, (st, r, slots) in enumerate(want):
        assert out[b] == slots, b
        if st != so.OK:
            continue
        assert (int(res.slots[b]), int(res.slice_indices[b]), bool(res.is_last[b])) == r["header"]
        assert res.parents[b] == r["parent"]
        off, ln = int(res.data_offsets[b]), int(res.data_lens[b])
        assert cw[b, off:off + ln].tobytes() == r["data"]


@pytest.mark.parametrize("kind", KINDS)
def test_pipeline_kind_roundtrip_random_arrival(ctx, dev, kind):
    """shred_batch_kind -> a random 32..64 of each slice's datagrams -> deshred_batch_kind
    restores every payload and every datagram (96 slices of 1 KiB shreds)."""
    S, n = 1024, 96
    rng = random.Random(900 + kind)
    slices = _slices_kind(rng, n, S, kind)
    cw, pk_buf, lens, _, _, pk = _gpu_shred_kind(ctx, dev, kind, slices, S)
    full = _packets(pk_buf, lens, n)
    inp = []
    for b in range(n):
        keep = set(rng.sample(range(64), 32 if b % 2 else rng.randrange(32, 65)))
        inp.append([full[b][j] if j in keep else None for j in range(64)])
    res, out, cw2 = _deshred_kind(ctx, dev, kind, inp, pk, S)
    assert (res.status == 0).all()
    assert out == full
    for b, (parent, data, *_r) in enumerate(slices):
        off, ln = int(res.data_offsets[b]), int(res.data_lens[b])
        assert res.parents[b] == parent and cw2[b, off:off + ln].tobytes() == data
