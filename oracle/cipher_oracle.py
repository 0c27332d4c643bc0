"""CPU restatement of the AONT / PETS shredders' payload transforms -- TEST INFRASTRUCTURE
ONLY (tests/, bench cpu_baseline legs); the product path is libalpenglow_rs.so (ag_aon_*).

Follows /root/reference/src:
  crypto/cipher.rs:25-30   apply_keystream: ctr::Ctr64LE<aes::Aes128>, all-zero IV
  crypto/hash.rs:64-67     hash: SHA-256 (sha2 crate) -> hashlib
  shredder.rs:414-418      PetsShredder::shred: ciphertext || key
  shredder.rs:463-470      AontShredder::shred: ciphertext || key ^ SHA-256(ciphertext)[..16]
  shredder.rs:509-528      decrypt_payload (+ the derive_key closures :430, :481-488)

AES-128 is FIPS-197, written out here (no AES library is installed); pinned by the
FIPS-197 Appendix C.1 and NIST SP 800-38A F.1.1 known-answer vectors in the tests.  The
CTR flavour is recalled from the ctr crate (Ctr64LE: the first 8 counter-block bytes are a
little-endian u64 block counter; the zero IV leaves the other 8 bytes zero): the aes / ctr
crates are not vendored, so that detail is "parity unpinned" (the reference's own cipher
tests are round trips only, crypto/cipher.rs:42-66).
"""

from __future__ import annotations

import hashlib

KEY_BYTES = 16


def _gmul(a: int, b: int) -> int:
    p = 0
    for _ in range(8):
        if b & 1:
            p ^= a
        hi = a & 0x80
        a = (a << 1) & 0xFF
        if hi:
            a ^= 0x1B
        b >>= 1
    return p


def _sbox():
    inv = [0] * 256
    for a in range(1, 256):
        for b in range(1, 256):
            if _gmul(a, b) == 1:
                inv[a] = b
                break
    out = []
    for i in range(256):
        b = inv[i]
        s = b
        for k in range(1, 5):
            s ^= ((b << k) | (b >> (8 - k))) & 0xFF
        out.append(s ^ 0x63)
    return out


SBOX = _sbox()
RCON = [0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x1B, 0x36]


def expand_key(key: bytes):
    """FIPS-197 §5.2: 11 round keys of 16 bytes."""
    w = [list(key[4 * i: 4 * i + 4]) for i in range(4)]
    for i in range(4, 44):
        t = list(w[i - 1])
        if i % 4 == 0:
            t = t[1:] + t[:1]
            t = [SBOX[x] for x in t]
            t[0] ^= RCON[i // 4 - 1]
        w.append([w[i - 4][j] ^ t[j] for j in range(4)])
    return [sum(w[4 * r: 4 * r + 4], []) for r in range(11)]


def aes128_encrypt_block(key: bytes, block: bytes, rks=None) -> bytes:
    rks = rks or expand_key(key)
    s = [block[i] ^ rks[0][i] for i in range(16)]  # column-major state, byte i = row i%4, col i//4
    for r in range(1, 11):
        s = [SBOX[x] for x in s]
        s = [s[(i + 4 * (i % 4)) % 16] for i in range(16)]  # ShiftRows
        if r != 10:
            t = []
            for c in range(4):
                a = s[4 * c: 4 * c + 4]
                t += [_gmul(a[0], 2) ^ _gmul(a[1], 3) ^ a[2] ^ a[3],
                      a[0] ^ _gmul(a[1], 2) ^ _gmul(a[2], 3) ^ a[3],
                      a[0] ^ a[1] ^ _gmul(a[2], 2) ^ _gmul(a[3], 3),
                      _gmul(a[0], 3) ^ a[1] ^ a[2] ^ _gmul(a[3], 2)]
            s = t
        s = [s[i] ^ rks[r][i] for i in range(16)]
    return bytes(s)


def apply_keystream(key: bytes, buf: bytes) -> bytes:
    """cipher::apply_keystream (Ctr64LE, zero IV): block i = AES(LE64(i) || 0^8)."""
    rks = expand_key(key)
    out = bytearray(buf)
    for i in range(0, len(buf), 16):
        ks = aes128_encrypt_block(key, (i // 16).to_bytes(8, "little") + bytes(8), rks)
        for j in range(min(16, len(buf) - i)):
            out[i + j] ^= ks[j]
    return bytes(out)


def sha256(data: bytes) -> bytes:
    return hashlib.sha256(data).digest()


def aont_encrypt(payload: bytes, key: bytes) -> bytes:
    ct = apply_keystream(key, payload)
    return ct + bytes(k ^ h for k, h in zip(key, sha256(ct)))


def pets_encrypt(payload: bytes, key: bytes) -> bytes:
    return apply_keystream(key, payload) + bytes(key)


def decrypt_payload(buf: bytes, aont: bool):
    """decrypt_payload: None for a buffer shorter than the key (DeshredError::BadEncoding)."""
    if len(buf) < KEY_BYTES:
        return None
    ct, tail = buf[:-KEY_BYTES], buf[-KEY_BYTES:]
    key = bytes(t ^ h for t, h in zip(tail, sha256(ct))) if aont else tail
    return apply_keystream(key, ct)
