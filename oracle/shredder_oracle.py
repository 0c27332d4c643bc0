"""CPU composition of the reference's four shredders (TEST INFRASTRUCTURE ONLY: imported by
tests/ as the checker of ag_shredder_shred_batch(_kind) / ag_shredder_deshred_batch(_kind);
never by the product path).

Follows /root/reference/src/shredder.rs:
  RegularShredder::shred (:337-345) = ReedSolomonCoder::shred(slice.payload_bytes())
    -> data_and_coding_to_output_shreds (:533-542): build_merkle_tree (:628-632),
       sign(SliceCommitment(header, root)) (:540, :206-222), assemble_output_shreds /
       fill_missing_shreds (:551-611): shred j carries the header, index j, its raw shred,
       the slice signature and tree.create_proof(j); data shreds first.
  Shredder::deshred (:282-311): ValidatedShreds layout -> ReedSolomonCoder::deshred (the
    crate's decoder over EVERY kept shred, reed_solomon.rs:154-166: rs_oracle.decode) ->
    check_merkle_tree (:616-625) -> SlicePayload::try_from -> fill_missing_shreds (:576-611).
  The receiver in front of it (`receive`): network::deserialize, the datagram's slot
    (shred index, kind, shred size, path length), ValidatedShred::try_new
    (validated_shred.rs:52-81) with the blockstore's cached commitment -- the first fitting
    shred of a slice is checked by signature and caches its commitment -- and the shreds kept
    for the slice: the valid ones with the first valid one's commitment.  This is the
    receive model ag_shredder_deshred_batch documents (include/alpenglow_rs.h section 9).
  CodingOnlyShredder / PetsShredder / AontShredder (:361-500, deshred_validated_shreds
    :512-528): shred_kind / deshred_kind -- the same composition with the coder's coding count
    (64 / 33 / 32), the output data shreds (0 / 31 / 32) and PETS / AONT encryption
    (cipher_oracle, pinned separately).
Datagrams are network::serialize(&Shred) (shred_wire_oracle).  Each stage is the pinned or
restated oracle of its own row (slice_oracle, rs_oracle, merkle_oracle, ed25519_oracle,
shred_wire_oracle); this module only composes them.
"""

import cipher_oracle as ci
import ed25519_oracle as ed
import merkle_oracle as mk
import rs_oracle as o
import shred_wire_oracle as wire
import slice_oracle as so

DATA_SHREDS, TOTAL_SHREDS = 32, 64

# The four shredders of shredder.rs (include/alpenglow_rs.h AG_SHREDDER_*): the coder's coding
# shreds m and the data output shreds (DATA_OUTPUT_SHREDS)
REGULAR, CODING_ONLY, PETS, AONT = 0, 1, 2, 3
CODING = {REGULAR: 32, CODING_ONLY: 64, PETS: 33, AONT: 32}
DATA_OUT = {REGULAR: 32, CODING_ONLY: 0, PETS: 31, AONT: 32}


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


def output_raw(kind: int, raw):
    """The output raw shreds of the coder's RawShreds: CodingOnly drops the data shreds
    (shredder.rs:372-373, 385-386), PETS the data shred holding the key (:420-421, 432-433)."""
    if kind == CODING_ONLY:
        return o.RawShreds(data=[], coding=list(raw.coding))
    if kind == PETS:
        return o.RawShreds(data=list(raw.data[:-1]), coding=list(raw.coding))
    return raw


def shred_kind(kind: int, parent, data: bytes, slot: int, slice_index: int, is_last: bool, seed: bytes,
               key: bytes = None):
    """Shredder::shred of RegularShredder / CodingOnlyShredder / PetsShredder / AontShredder
    (shredder.rs:336-500) for one slice; PETS / AONT take the key encrypt_with_random_key would
    draw.  -> (datagrams, output RawShreds, root, sig); raises RSError(TooMuchData)."""
    payload = so.payload_bytes(parent, data)
    if kind == PETS:
        payload = ci.pets_encrypt(payload, key)   # :414-418
    elif kind == AONT:
        payload = ci.aont_encrypt(payload, key)   # :463-469
    raw = output_raw(kind, o.coder_shred(payload, CODING[kind]))
    pkts, root, sig = datagrams(raw.data, raw.coding, slot, slice_index, is_last, seed)
    return pkts, raw, root, sig


# ---- the receive side ---------------------------------------------------------------------

HEIGHT = 6  # Merkle path length of a 64-leaf slice tree

# per-slice results (AG_RS_OK / AG_RS_ERR_* of include/alpenglow_rs.h)
OK, NOT_ENOUGH_SHARDS, TOO_MUCH_DATA, BAD_ENCODING, INVALID_MERKLE_TREE = 0, 9, 20, 23, 24


def receive(rows, pk: bytes, shred_bytes: int, num_data: int = DATA_SHREDS):
    """The shreds a receiver keeps for one slice from its 64 datagram slots (bytes or None):
    a list of 64 entries, None or dict(kind, slot, slice_index, is_last, data, sig, root).
    num_data: the shredder's data output shreds (slot j < num_data holds a Data shred)."""
    parsed = [wire.deserialize(p) if p else None for p in rows]

    def fits(j):
        x = parsed[j]
        return (x is not None and x[4] == j and x[0] == (wire.CODING if j >= num_data else wire.DATA) and
                len(x[5]) == shred_bytes and len(x[7]) == HEIGHT)

    commit, root = [None] * TOTAL_SHREDS, [None] * TOTAL_SHREDS
    for j in range(TOTAL_SHREDS):
        if fits(j):
            _, slot, si, last, _, data, _, proof = parsed[j]
            root[j] = mk.derive_root(data, j, proof)  # Shred::slice_root (shredder.rs:169-175)
            commit[j] = ed.slice_commitment(slot, si, last, root[j])
    fitting = [j for j in range(TOTAL_SHREDS) if commit[j] is not None]
    if not fitting:
        return [None] * TOTAL_SHREDS
    first = fitting[0]
    cached = commit[first] if ed.validate_shred(commit[first], parsed[first][6], pk, None) == ed.OK else None
    valid = [j for j in fitting if ed.validate_shred(commit[j], parsed[j][6], pk, cached) == ed.OK]
    out = [None] * TOTAL_SHREDS
    for j in valid:
        if commit[j] == commit[valid[0]]:
            kind, slot, si, last, _, data, sig, _ = parsed[j]
            out[j] = dict(kind=kind, slot=slot, slice_index=si, is_last=last, data=data, sig=sig, root=root[j])
    return out


def deshred(kept):
    """Shredder::deshred (shredder.rs:282-311) for RegularShredder on the kept shreds.
    Returns (status, result): result = dict(payload parse, raw shreds, the 64 datagrams with
    the missing ones filled in) for OK, else None."""
    if all(x is None for x in kept):
        return NOT_ENOUGH_SHARDS, None
    shreds = [(j < DATA_SHREDS, x["data"]) if x is not None else None for j, x in enumerate(kept)]
    try:
        payload, raw = o.coder_deshred(shreds, DATA_SHREDS, TOTAL_SHREDS - DATA_SHREDS)
    except o.RSError as e:
        return {"NotEnoughShreds": NOT_ENOUGH_SHARDS, "TooMuchData": TOO_MUCH_DATA,
                "InvalidPadding": BAD_ENCODING}[e.kind], None
    any_shred = next(x for x in kept if x is not None)
    tree = mk.slice_tree(raw.data, raw.coding)
    if tree.root() != any_shred["root"]:
        return INVALID_MERKLE_TREE, None
    st, parent, data = so.try_from(payload)
    if st != so.OK:
        return (TOO_MUCH_DATA if st == so.TOO_LARGE else BAD_ENCODING), None
    shards = raw.data + raw.coding
    dgrams = [wire.serialize(wire.DATA if j < DATA_SHREDS else wire.CODING, any_shred["slot"],
                             any_shred["slice_index"], any_shred["is_last"], j, shards[j], any_shred["sig"],
                             tree.create_proof(j)) for j in range(TOTAL_SHREDS)]
    return OK, dict(parent=parent, data=data, raw=raw, header=(any_shred["slot"], any_shred["slice_index"],
                                                               any_shred["is_last"]), datagrams=dgrams)


def deshred_kind(kept, kind: int):
    """Shredder::deshred (shredder.rs:282-311) of the shredder `kind`: ValidatedShreds with its
    layout, deshred_validated_shreds (the coder over every kept shred, then decrypt_payload for
    PETS / AONT, :512-528), check_merkle_tree over the output raw shreds, SlicePayload, and the
    64 datagrams with the missing ones filled in.  (status, result) as deshred."""
    if kind == REGULAR:
        return deshred(kept)
    if all(x is None for x in kept):
        return NOT_ENOUGH_SHARDS, None
    nd = DATA_OUT[kind]
    shreds = [(j < nd, x["data"]) if x is not None else None for j, x in enumerate(kept)]
    try:
        buf, raw = o.coder_deshred(shreds, nd, CODING[kind])
    except o.RSError as e:
        return {"NotEnoughShreds": NOT_ENOUGH_SHARDS, "TooMuchData": TOO_MUCH_DATA,
                "InvalidPadding": BAD_ENCODING}[e.kind], None
    raw = output_raw(kind, raw)
    payload = buf
    if kind in (PETS, AONT):
        payload = ci.decrypt_payload(buf, kind == AONT)
        if payload is None:
            return BAD_ENCODING, None
    any_shred = next(x for x in kept if x is not None)
    tree = mk.slice_tree(raw.data, raw.coding)
    if tree.root() != any_shred["root"]:
        return INVALID_MERKLE_TREE, None
    st, parent, data = so.try_from(payload)
    if st != so.OK:
        return (TOO_MUCH_DATA if st == so.TOO_LARGE else BAD_ENCODING), None
    shards = raw.data + raw.coding
    dgrams = [wire.serialize(wire.DATA if j < nd else wire.CODING, any_shred["slot"], any_shred["slice_index"],
                             any_shred["is_last"], j, shards[j], any_shred["sig"], tree.create_proof(j))
              for j in range(TOTAL_SHREDS)]
    return OK, dict(parent=parent, data=data, raw=raw, header=(any_shred["slot"], any_shred["slice_index"],
                                                               any_shred["is_last"]), datagrams=dgrams)
