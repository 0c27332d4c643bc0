"""CPU restatement of the shred wire format -- TEST INFRASTRUCTURE ONLY.

Only tests/ and bench_wire.py's cpu_baseline leg use this module, as the checker; the
product path (ag_shred_serialize_batch / ag_shred_deserialize_batch) never calls it.

The reference sends a `Shred` (shredder.rs:113-127) as one UDP datagram, encoded with
wincode 0.6.0 (Cargo.lock:3170-3173; not vendored) and decoded by network::deserialize
(network.rs:52-64: wincode's default configuration with preallocation capped at
MTU_BYTES = 1500, all bytes consumed).  wincode is bincode-compatible (fixed-width
little-endian integers, u32 enum discriminants, u64 sequence lengths, bool as one byte 0/1),
so a Shred is:

  u32  variant             ShredPayloadType::{Data = 0, Coding = 1}      shredder.rs:113-117
  u64  slot                SliceHeader.slot (Slot(u64))                  types/slice.rs:153-160
  u64  slice_index         usize, raw 8 bytes; read rejects >= MAX_SLICES_PER_BLOCK = 1024
                           (types/slice_index.rs:15,115-132)
  u8   is_last             bool
  u64  shred_index         usize; read rejects >= TOTAL_SHREDS = 64 (shred_index.rs:91-108)
  u64  len, len bytes      ShredPayload.data (Vec<u8>)                   shredder.rs:177-186
  64 B slice_sig           Signature (pod wrapper)                       crypto/signature.rs:31-39
  u64  len, len x 32 B     merkle_path: SliceProof(Vec<Hash>)            crypto/merkle.rs:199

Parity unpinned: the reference holds no serialized Shred bytes; the layout follows the
derives above and wincode's published bincode-compatible encoding.
"""

from __future__ import annotations

import struct

MTU_BYTES = 1500
MAX_SLICES_PER_BLOCK = 1024
TOTAL_SHREDS = 64
DATA, CODING = 0, 1
OK, MALFORMED = 0, 1


def serialize(kind: int, slot: int, slice_index: int, is_last: bool, shred_index: int, data: bytes, sig: bytes,
              proof: list[bytes]) -> bytes:
    assert kind in (DATA, CODING) and len(sig) == 64 and all(len(h) == 32 for h in proof)
    return (struct.pack("<IQQBQQ", kind, slot, slice_index, 1 if is_last else 0, shred_index, len(data)) +
            bytes(data) + bytes(sig) + struct.pack("<Q", len(proof)) + b"".join(proof))


def deserialize(buf: bytes):
    """network::deserialize::<Shred>: a tuple (kind, slot, slice_index, is_last, shred_index,
    data, sig, proof) or None when wincode would reject the bytes."""
    try:
        kind, slot, slice_index, is_last, shred_index, n = struct.unpack_from("<IQQBQQ", buf, 0)
    except struct.error:
        return None
    o = struct.calcsize("<IQQBQQ")
    if kind not in (DATA, CODING) or is_last > 1 or slice_index >= MAX_SLICES_PER_BLOCK or \
            shred_index >= TOTAL_SHREDS or n > MTU_BYTES or o + n > len(buf):
        return None
    data = bytes(buf[o:o + n])
    o += n
    if o + 64 + 8 > len(buf):
        return None
    sig = bytes(buf[o:o + 64])
    o += 64
    (h,) = struct.unpack_from("<Q", buf, o)
    o += 8
    if h * 32 > MTU_BYTES or o + 32 * h > len(buf):
        return None
    proof = [bytes(buf[o + 32 * i:o + 32 * i + 32]) for i in range(h)]
    o += 32 * h
    if o != len(buf):  # deserialize_exact: trailing bytes rejected
        return None
    return kind, slot, slice_index, bool(is_last), shred_index, data, sig, proof
