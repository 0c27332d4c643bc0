"""CPU restatement of the reference's slice Merkle tree -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module, as
the checker; the product path (libalpenglow_rs.so, ag_merkle_*) never calls it.

Follows /root/reference/src/crypto/merkle.rs:
  labels                  :42-44
  MerkleTree::new         :281-333  (odd node at height h pairs with EMPTY_ROOTS[h])
  get_root / height       :337-345
  create_proof            :351-370
  check_proof             :374-387
  check_proof_last        :394-407, derive_hash_root_last :436-452
  derive_root             :411-428
  hash_leaf / hash_pair   :457-468
and crypto/hash.rs:64-79 (hash_all = SHA-256 of the concatenation; sha2 crate).
The slice tree's leaves are the raw shreds, data then coding (shredder.rs:628-632).

Parity pin: EMPTY_ROOTS recomputed here must equal the 32 digests the reference holds
(merkle.rs:62-157; tests/golden/merkle_empty_roots.json, tests/golden/make_merkle_golden.py).
"""

from __future__ import annotations

import hashlib

LEAF_LABEL = b"ALPENGLOW-MERKLE-TREE  LEAF-NODE"
LEFT_LABEL = b"ALPENGLOW-MERKLE-TREE  LEFT-NODE"
RIGHT_LABEL = b"ALPENGLOW-MERKLE-TREE RIGHT-NODE"
MAX_MERKLE_TREE_HEIGHT = 32

assert len(LEAF_LABEL) == len(LEFT_LABEL) == len(RIGHT_LABEL) == 32


def hash_all(parts) -> bytes:
    h = hashlib.sha256()
    for p in parts:
        h.update(p)
    return h.digest()


def hash_leaf(data: bytes) -> bytes:
    return hash_all([LEAF_LABEL, data])


def hash_pair(left: bytes, right: bytes) -> bytes:
    return hash_all([LEFT_LABEL, left, RIGHT_LABEL, right])


def _empty_roots():
    out, node = [], hash_leaf(b"")
    for _ in range(MAX_MERKLE_TREE_HEIGHT):
        out.append(node)
        node = hash_pair(node, node)
    return out


EMPTY_ROOTS = _empty_roots()


class MerkleTree:
    """nodes: leaf hashes, then each level; levels: (offset, len) per level."""

    def __init__(self, leaves):
        nodes = [hash_leaf(bytes(x)) for x in leaves]
        assert nodes, "empty tree"
        levels = [(0, len(nodes))]
        left, right = 0, len(nodes)
        length, h = right - left, 0
        while length > 1:
            for i in range(left, right, 2):
                if i + 1 == right:
                    nodes.append(hash_pair(nodes[i], EMPTY_ROOTS[h]))
                    break
                nodes.append(hash_pair(nodes[i], nodes[i + 1]))
            length = (length + 1) // 2
            left, right = right, right + length
            h += 1
            levels.append((left, length))
        self.nodes, self.levels = nodes, levels

    def root(self) -> bytes:
        return self.nodes[-1]

    def height(self) -> int:
        return len(self.levels) - 1

    def create_proof(self, index: int) -> list[bytes]:
        assert index < (1 << self.height()) or self.height() == 0
        assert index < self.levels[0][1]
        proof, i = [], index
        for h, (off, length) in enumerate(self.levels[: self.height()]):
            proof.append(EMPTY_ROOTS[h] if (i ^ 1) >= length else self.nodes[off + (i ^ 1)])
            i //= 2
        return proof


def derive_root(data: bytes, index: int, proof) -> bytes:
    node, i = hash_leaf(data), index
    for h in proof:
        node = hash_pair(node, h) if i % 2 == 0 else hash_pair(h, node)
        i //= 2
    return node


def check_proof(data: bytes, index: int, root: bytes, proof) -> bool:
    return len(proof) <= len(EMPTY_ROOTS) and derive_root(data, index, proof) == root


def check_proof_last(data: bytes, index: int, root: bytes, proof) -> bool:
    if len(proof) > len(EMPTY_ROOTS):
        return False
    node, i = hash_leaf(data), index
    for height, h in enumerate(proof):
        if i % 2 == 0:
            if h != EMPTY_ROOTS[height]:
                return False
            node = hash_pair(node, EMPTY_ROOTS[height])
        else:
            node = hash_pair(h, node)
        i //= 2
    return node == root


def slice_tree(data_shreds, coding_shreds) -> MerkleTree:
    """build_merkle_tree (shredder.rs:628-632): leaves = data shreds then coding shreds."""
    return MerkleTree(list(data_shreds) + list(coding_shreds))
