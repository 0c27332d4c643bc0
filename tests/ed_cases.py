"""Shared Ed25519 test cases (seeded): valid signatures plus the malformed encodings the
ZIP-215 rules of ed25519-zebra 4.2.0 decide (crypto/signature.rs:100-103).  Expected
verdicts come from the oracle (oracle/ed25519_oracle.py)."""

import random

import ed25519_oracle as eo

P, L = eo.P, eo.L


def le(x: int) -> bytes:
    return int(x).to_bytes(32, "little")


def verify_cases(seed: int = 7, n_random: int = 24):
    """List of (pk, msg, sig) triples."""
    rng = random.Random(seed)
    cases = []
    keys = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(4)]
    pks = [eo.secret_to_public(k) for k in keys]
    for i in range(n_random):
        k = i % len(keys)
        msg = bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 1, 49, 49, 64, 111, 112, 200])))
        sig = eo.sign(keys[k], msg)
        cases.append((pks[k], msg, sig))
        # tampered message / signature / key
        if i % 4 == 0:
            cases.append((pks[k], msg + b"x", sig))
        if i % 4 == 1:
            bad = bytearray(sig)
            bad[rng.randrange(64)] ^= 1 << rng.randrange(8)
            cases.append((pks[k], msg, bytes(bad)))
        if i % 4 == 2:
            cases.append((pks[(k + 1) % len(keys)], msg, sig))
        if i % 4 == 3:  # s + l: same group element, non-canonical scalar -> rejected
            s = int.from_bytes(sig[32:], "little") + L
            if s < 2**256:
                cases.append((pks[k], msg, sig[:32] + le(s)))
    ident = le(1)
    small = eo.small_order_encodings()
    # cofactored equation: small-order A and R with s = 0 verify under ZIP-215
    for a in small:
        for r in small[:3]:
            cases.append((a, b"zip215", r + le(0)))
    # non-canonical y (y >= p) for A and R, "negative zero" x
    nc_one = le(P + 1)                       # y = p + 1 == 1 (the identity)
    neg_zero = le(1 | (1 << 255))            # identity with the sign bit set
    for a in (ident, nc_one, neg_zero):
        for r in (ident, nc_one, neg_zero):
            cases.append((a, b"noncanonical", r + le(0)))
    for y in range(19):                      # every non-canonical y in [p, 2^255)
        enc = le(P + y)
        if eo.decompress(enc) is not None:
            cases.append((enc, b"nc-y", ident + le(0)))
            cases.append((pks[0], b"nc-y", enc + le(0)))
    # random 32-byte strings as keys (about half do not decode)
    for _ in range(8):
        junk = bytes(rng.getrandbits(8) for _ in range(32))
        cases.append((junk, b"junk", eo.sign(keys[0], b"junk")))
    # s = l - 1 (largest canonical), s = l (smallest non-canonical)
    cases.append((pks[0], b"edge", ident + le(L - 1)))
    cases.append((pks[0], b"edge", ident + le(L)))
    return cases
