"""Slice payload framing oracle.

TEST INFRASTRUCTURE ONLY -- imported by tests/; never by the product package.

Restates /root/reference/src/types/slice.rs:
  Slice::payload_bytes          slice.rs:73-84   wincode(parent: Option<BlockId>) || wincode(data: Vec<u8>)
  SlicePayload::try_from(&[u8]) slice.rs:211-218 TooLarge if len > MAX_DATA_PER_SLICE; wincode
                                                 deserialize_exact with preallocation capped at
                                                 MAX_DATA_PER_SLICE, any failure -> BadEncoding
with BlockId = (Slot, BlockHash) (lib.rs:65; Slot(u64) slot.rs:22, BlockHash =
DoubleMerkleRoot(Hash([u8; 32])) merkle.rs:212, hash.rs:17) and wincode's default config
(fixed-width little-endian integers, Option tag byte 0/1, Vec = u64 length + elements).
The wincode crate (Cargo.lock: wincode 0.6) is not vendored: its encoding rules are recalled
(consistent with the reference's own comment at slice.rs:77 "8-byte `data` length prefix
(wincode fixint)"); the behaviours are pinned by the reference's slice.rs tests (:267-332),
restated in tests/test_slice.py.
"""

from __future__ import annotations

import struct

MAX_DATA_PER_SLICE = 32 * 1024 - 1   # shredder.rs:54 (MAX_DATA_PER_SLICE_AFTER_PADDING - 1)
BLOCK_ID_BYTES = 8 + 32              # (Slot u64, BlockHash [u8; 32])

OK, TOO_LARGE, BAD_ENCODING = 0, 1, 2


def header_len(parent) -> int:
    return 1 + (BLOCK_ID_BYTES if parent is not None else 0) + 8


def payload_bytes(parent, data: bytes) -> bytes:
    """Slice::payload_bytes: parent = None or (slot: int, block_hash: 32 bytes)."""
    if parent is None:
        head = b"\x00"
    else:
        slot, h = parent
        if len(h) != 32:
            raise ValueError("block hash must be 32 bytes")
        head = b"\x01" + struct.pack("<Q", slot) + bytes(h)
    return head + struct.pack("<Q", len(data)) + bytes(data)


def try_from(payload: bytes):
    """SlicePayload::try_from -> (status, parent, data); parent/data None unless OK."""
    n = len(payload)
    if n > MAX_DATA_PER_SLICE:
        return TOO_LARGE, None, None
    if n < 1:
        return BAD_ENCODING, None, None
    tag = payload[0]
    if tag == 0:
        parent, off = None, 1
    elif tag == 1:
        if n < 1 + BLOCK_ID_BYTES:
            return BAD_ENCODING, None, None
        parent = (struct.unpack_from("<Q", payload, 1)[0], bytes(payload[9:41]))
        off = 41
    else:
        return BAD_ENCODING, None, None
    if n < off + 8:
        return BAD_ENCODING, None, None
    length = struct.unpack_from("<Q", payload, off)[0]
    off += 8
    # preallocation cap, then exact consumption (no trailing bytes, no truncation)
    if length > MAX_DATA_PER_SLICE or off + length != n:
        return BAD_ENCODING, None, None
    return OK, parent, bytes(payload[off:off + length])
