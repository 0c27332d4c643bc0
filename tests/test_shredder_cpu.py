"""The composed-Shredder CPU baseline (oracle/shredder_cpu.c, bench_shredder.py's cpu_baseline
leg) against the reference's composition restated in Python (oracle/shredder_oracle.py):
the same coding shreds, slice root and leader signature per slice, and a round trip through
its receive + deshred.  CPU only."""

import numpy as np

import ed25519_oracle as ed
import merkle_oracle as mk
import rs_oracle as o
import shredder_cpu as sc
import slice_oracle as so


def test_shredder_cpu_matches_oracle():
    seed = bytes(range(32))
    pk = ed.secret_to_public(seed)
    rng = np.random.default_rng(3)
    sizes = [32767 - 9, 1000, 20000]
    n = len(sizes)
    framed = [so.payload_bytes(None, rng.integers(0, 256, s, dtype=np.uint8).tobytes()) for s in sizes]
    payloads = np.zeros((n, 32768), np.uint8)
    for b, f in enumerate(framed):
        payloads[b, :len(f)] = np.frombuffer(f, np.uint8)
    lens = [len(f) for f in framed]
    slots, sidx, last = [5, 6, 7], [0, 1, 1023], [0, 0, 1]
    st, coding, roots, sigs = sc.run(sc.SHRED | sc.RECEIVE | sc.DESHRED, 2, payloads, lens, slots, sidx, last, seed, pk,
                                     outputs=True)
    # sizes 1000 and 20000 pad to shreds that are not whole 64-byte chunks: the Avx2 port
    # serves only the maximum-slice shape, so those report a failure
    assert st != 0
    st, coding, roots, sigs = sc.run(sc.SHRED | sc.RECEIVE | sc.DESHRED, 2, payloads[:1], lens[:1], slots[:1],
                                     sidx[:1], last[:1], seed, pk, outputs=True)
    assert st == 0
    raw = o.coder_shred(framed[0], 32)
    assert b"".join(raw.coding) == coding[0].tobytes()
    root = mk.slice_tree(raw.data, raw.coding).root()
    assert roots[0].tobytes() == root
    assert sigs[0].tobytes() == ed.sign(seed, ed.slice_commitment(slots[0], sidx[0], bool(last[0]), root))


def test_shredder_cpu_phases():
    seed = bytes(range(32))
    pk = ed.secret_to_public(seed)
    payload = so.payload_bytes(None, bytes(32767 - 9))
    t = sc.phase_us(payload, seed, pk, reps=3)
    assert all(x > 0 for x in t)
