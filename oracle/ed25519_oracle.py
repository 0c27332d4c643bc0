"""CPU restatement of the reference's shred signatures -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench_sig.py's cpu_baseline leg use this module,
as the checker; the product path (libalpenglow_rs.so, ag_ed25519_* / ag_shred_*) never
calls it.

What it restates
  crypto/signature.rs:60-104   SecretKey::{to_pk, sign_bytes}, Signature::verify_bytes --
                               thin wrappers over the crate ed25519-zebra 4.2.0
                               (Cargo.lock:783-786) on curve25519-dalek 4.1.3 (:548-551).
                               Neither crate is vendored (no network), so their published
                               algorithms are restated here:
    keygen / sign  RFC 8032 §5.1.5-5.1.6 (ed25519-zebra SigningKey::from / sign).
    verify         ZIP-215 rules (ed25519-zebra VerificationKey::verify / verify_prehashed):
                   s must be canonical (< l); A and R need only decode to curve points --
                   y is read from 255 bits and reduced mod p (non-canonical y accepted),
                   "negative zero" x accepted (dalek CompressedEdwardsY::decompress);
                   k = SHA-512(R_bytes || A_bytes || M) mod l over the ORIGINAL bytes;
                   accept iff [8]([s]B - [k]A - R) is the identity (cofactored equation).
  shredder.rs:199-216          SliceCommitment::new: slot u64 LE || slice_index u64 LE ||
                               is_last u8 || slice_root (49 bytes) -- the signed message.
  shredder/validated_shred.rs:52-81
                               ValidatedShred::try_new: root from the shred's Merkle path,
                               commitment, then the cached-commitment short cut /
                               Equivocation / InvalidSignature rules.
  shredder.rs:540              the shred side: sk.sign_bytes(SliceCommitment(header, root)).

Parity pins: RFC 8032 §7.1 TESTs 1-3 (secret key -> public key -> signature, byte-exact;
tests/golden/ed25519_rfc8032.json) plus the group-law identities checked in
tests/test_ed25519.py.  The ZIP-215 acceptance rules for malformed encodings have no
known-answer vectors in the reference: those cases are "parity unpinned" against the
crate and pinned only to the rules above.
"""

from __future__ import annotations

import hashlib

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
SQRT_M1 = pow(2, (P - 1) // 4, P)

# base point: y = 4/5, x even
_BY = (4 * pow(5, P - 2, P)) % P


def _recover_x(y: int, sign: int):
    """x with x^2 = (y^2-1)/(d y^2+1), x's parity = sign; None if not a square.
    Like dalek's decompress, sign=1 with x=0 is NOT rejected (ZIP-215)."""
    u = (y * y - 1) % P
    v = (D * y * y + 1) % P
    x = (u * pow(v, 3, P) * pow(u * pow(v, 7, P), (P - 5) // 8, P)) % P
    vx2 = (v * x * x) % P
    if vx2 == u:
        pass
    elif vx2 == (-u) % P:
        x = (x * SQRT_M1) % P
    else:
        return None
    if x & 1:
        x = P - x  # nonnegative root (even), then apply the sign bit
    if sign:
        x = (-x) % P
    return x


_BX = _recover_x(_BY, 0)
B = (_BX, _BY, 1, (_BX * _BY) % P)  # extended (X, Y, Z, T)
IDENTITY = (0, 1, 1, 0)


def point_add(p, q):
    """add-2008-hwcd-3 (a = -1) in extended coordinates."""
    x1, y1, z1, t1 = p
    x2, y2, z2, t2 = q
    a = ((y1 - x1) * (y2 - x2)) % P
    b = ((y1 + x1) * (y2 + x2)) % P
    c = (t1 * 2 * D * t2) % P
    d = (z1 * 2 * z2) % P
    e, f, g, h = b - a, d - c, d + c, b + a
    return ((e * f) % P, (g * h) % P, (f * g) % P, (e * h) % P)


def point_neg(p):
    x, y, z, t = p
    return ((-x) % P, y, z, (-t) % P)


def scalar_mult(s: int, p):
    q = IDENTITY
    while s > 0:
        if s & 1:
            q = point_add(q, p)
        p = point_add(p, p)
        s >>= 1
    return q


def is_identity(p) -> bool:
    x, y, z, _ = p
    return x % P == 0 and (y - z) % P == 0


def point_equal(p, q) -> bool:
    x1, y1, z1, _ = p
    x2, y2, z2, _ = q
    return (x1 * z2 - x2 * z1) % P == 0 and (y1 * z2 - y2 * z1) % P == 0


def compress(p) -> bytes:
    x, y, z, _ = p
    zi = pow(z, P - 2, P)
    x, y = (x * zi) % P, (y * zi) % P
    return int.to_bytes(y | ((x & 1) << 255), 32, "little")


def decompress(s: bytes):
    """CompressedEdwardsY::decompress (curve25519-dalek 4.1): 255-bit y reduced mod p."""
    if len(s) != 32:
        return None
    v = int.from_bytes(s, "little")
    sign = v >> 255
    y = (v & ((1 << 255) - 1)) % P
    x = _recover_x(y, sign)
    if x is None:
        return None
    return (x, y, 1, (x * y) % P)


def sha512(*parts) -> bytes:
    h = hashlib.sha512()
    for p in parts:
        h.update(p)
    return h.digest()


def _expand(seed: bytes):
    h = sha512(seed)
    a = int.from_bytes(h[:32], "little")
    a &= (1 << 254) - 8
    a |= 1 << 254
    return a, h[32:]


def secret_to_public(seed: bytes) -> bytes:
    """SecretKey::to_pk (signature.rs:54-58): A = [a]B, RFC 8032 §5.1.5."""
    a, _ = _expand(seed)
    return compress(scalar_mult(a, B))


def sign(seed: bytes, msg: bytes) -> bytes:
    """SecretKey::sign_bytes (signature.rs:69-72): RFC 8032 §5.1.6."""
    a, prefix = _expand(seed)
    A = compress(scalar_mult(a, B))
    r = int.from_bytes(sha512(prefix, msg), "little") % L
    R = compress(scalar_mult(r, B))
    k = int.from_bytes(sha512(R, A, msg), "little") % L
    s = (r + k * a) % L
    return R + int.to_bytes(s, 32, "little")


def verify(pk: bytes, msg: bytes, sig: bytes) -> bool:
    """Signature::verify_bytes (signature.rs:100-103) = ed25519-zebra verify (ZIP-215)."""
    if len(sig) != 64 or len(pk) != 32:
        return False
    A = decompress(pk)
    if A is None:
        return False
    s = int.from_bytes(sig[32:], "little")
    if s >= L:
        return False
    R = decompress(sig[:32])
    if R is None:
        return False
    k = int.from_bytes(sha512(sig[:32], pk, msg), "little") % L
    # R' = [s]B - [k]A ; accept iff [8](R - R') == identity
    rp = point_add(scalar_mult(s, B), point_neg(scalar_mult(k, A)))
    diff = point_add(R, point_neg(rp))
    for _ in range(3):
        diff = point_add(diff, diff)
    return is_identity(diff)


# ---- shreds (shredder.rs, shredder/validated_shred.rs) ----------------------------------

SLICE_COMMITMENT_LEN = 8 + 8 + 1 + 32

OK, INVALID_SIGNATURE, EQUIVOCATION = 0, 1, 2


def slice_commitment(slot: int, slice_index: int, is_last: bool, slice_root: bytes) -> bytes:
    """SliceCommitment::new (shredder.rs:206-215)."""
    assert len(slice_root) == 32
    return (int(slot).to_bytes(8, "little") + int(slice_index).to_bytes(8, "little") +
            bytes([1 if is_last else 0]) + bytes(slice_root))


def validate_shred(commitment: bytes, sig: bytes, pk: bytes, cached: bytes | None) -> int:
    """ValidatedShred::try_new's decision (validated_shred.rs:52-81) once the commitment
    (header + root derived from the Merkle path) is known."""
    if cached is not None:
        if cached == commitment:
            return OK
        return EQUIVOCATION if verify(pk, commitment, sig) else INVALID_SIGNATURE
    return OK if verify(pk, commitment, sig) else INVALID_SIGNATURE


# small-order points (the torsion subgroup E[8]) in compressed form, for edge-case tests
def small_order_encodings():
    """The 8 points of order dividing 8, canonical encodings (x sign as computed)."""
    pts = set()
    # order-2: (0,-1); order-4: (+-sqrt(-1)... on a=-1 curve: (x, 0) with x^2 = -1)
    # enumerate by multiplying a random point by l: [l]Q lies in E[8]
    seed = 1
    while len(pts) < 8:
        y = seed
        seed += 1
        x = _recover_x(y % P, 0)
        if x is None:
            continue
        q = scalar_mult(L, (x, y, 1, (x * y) % P))
        for i in range(8):
            pts.add(compress(scalar_mult(i, q)))
    return sorted(pts)
