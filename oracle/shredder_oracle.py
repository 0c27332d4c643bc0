"""CPU composition of the reference's RegularShredder (TEST INFRASTRUCTURE ONLY: imported by
tests/ as the checker of ag_shredder_shred_batch / ag_shredder_deshred_batch; never by the
product path).

Follows /root/reference/src/shredder.rs:
  RegularShredder::shred (:337-345) = ReedSolomonCoder::shred(slice.payload_bytes())
    -> data_and_coding_to_output_shreds (:533-542): build_merkle_tree (:628-632),
       sign(SliceCommitment(header, root)) (:540, :206-222), assemble_output_shreds /
       fill_missing_shreds (:551-611): shred j carries the header, index j, its raw shred,
       the slice signature and tree.create_proof(j); data shreds first.
  Shredder::deshred (:282-311): ValidatedShreds layout -> ReedSolomonCoder::deshred ->
    check_merkle_tree (:616-625) -> SlicePayload::try_from -> fill_missing_shreds.
Datagrams are network::serialize(&Shred) (shred_wire_oracle).  Each stage is the pinned or
restated oracle of its own row (slice_oracle, rs_oracle, merkle_oracle, ed25519_oracle,
shred_wire_oracle); this module only composes them.
"""

import ed25519_oracle as ed
import merkle_oracle as mk
import rs_oracle as o
import shred_wire_oracle as wire
import slice_oracle as so

DATA_SHREDS, TOTAL_SHREDS = 32, 64


def datagrams(raw_data, raw_coding, slot: int, slice_index: int, is_last: bool, seed: bytes):
    """data_and_coding_to_output_shreds + serialization: the 64 datagrams of one slice whose
    raw shreds are given (a leader may sign any bytes, consistent or not)."""
    tree = mk.slice_tree(raw_data, raw_coding)
    root = tree.root()
    sig = ed.sign(seed, ed.slice_commitment(slot, slice_index, is_last, root))
    raw = list(raw_data) + list(raw_coding)
    pkts = [wire.serialize(wire.DATA if j < len(raw_data) else wire.CODING, slot, slice_index, is_last, j, raw[j], sig,
                           tree.create_proof(j)) for j in range(len(raw))]
    return pkts, root, sig


def shred(parent, data: bytes, slot: int, slice_index: int, is_last: bool, seed: bytes):
    """RegularShredder::shred of one slice -> (datagrams, RawShreds, root, sig)."""
    raw = o.coder_shred(so.payload_bytes(parent, data), TOTAL_SHREDS - DATA_SHREDS)
    pkts, root, sig = datagrams(raw.data, raw.coding, slot, slice_index, is_last, seed)
    return pkts, raw, root, sig
