// Slice Merkle trees (merkle.hip): parameter blocks and launchers.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace ag {

// TOTAL_SHREDS (shredder.rs:47): every shredder's slice tree has 64 leaves.
constexpr uint32_t kMerkleMaxLeaves = 64;

// Row t of a per-shred table (data rows, leaves): t * stride, or -- with group_stride set --
// grouped by slice: row j of slice g = t / 64 at g * group_stride + (j + (j >= skip)) * stride
// (skip 0: none).  The composed shredders address their output shreds in the caller's codeword
// buffer this way (CodingOnly: the coding rows; PETS: every row but the withheld data shard).
__host__ __device__ inline uint64_t grouped_row_offset(uint64_t t, uint64_t stride, uint64_t group_stride,
                                                       uint32_t skip) {
  if (!group_stride) return t * stride;
  const uint64_t j = t & (kMerkleMaxLeaves - 1);
  return (t / kMerkleMaxLeaves) * group_stride + (j + (skip && j >= skip ? 1u : 0u)) * stride;
}
// MAX_MERKLE_TREE_HEIGHT (merkle.rs:33)
constexpr int kMerkleMaxHeight = 32;

// nslices trees of n_leaves leaves; leaf j of slice s: leaves + s*slice_stride + j*leaf_stride,
// leaf_bytes long.  Outputs (device): roots[s] (32 B); nodes (optional) = the reference's
// `nodes` vector (leaf hashes, then each level); proofs (optional) = create_proof(j) for
// every leaf, height digests each.
struct MerkleBuildParams {
  const uint8_t* leaves;
  uint64_t leaf_stride;
  uint64_t slice_stride;
  uint32_t leaf_bytes;
  uint32_t n_leaves;
  uint64_t nslices;
  const uint32_t* empty_roots;  // device [32][8] big-endian words (EMPTY_ROOTS)
  uint8_t* roots;
  uint8_t* proofs;  // may be null
  uint64_t proofs_stride;
  // nullable pair: hash only the leaves t (slice-major, t = slice * n_leaves + j) with
  // hash_leaf[t] != 0, compacted into list (nslices * n_leaves + 1 words of scratch); the other
  // leaves' digests must already be in nodes (a proof check's leaf_nodes, same bytes)
  const uint8_t* hash_leaf;
  uint32_t* list;
  uint32_t skip_leaf;  // > 0: leaf j >= skip_leaf sits at (j + 1) * leaf_stride (a withheld row)
};
// nodes: the node digests (reference order, nodes_stride per slice; the caller's buffer or
// scratch) -- the levels are built there.
hipError_t launch_merkle_build(const MerkleBuildParams& p, uint8_t* nodes, uint64_t nodes_stride,
                               hipStream_t stream);

// check_proof for n leaves (or, with roots_out set, derive_root: the root each proof yields): leaf t at leaves + t*leaf_stride, its index index[t], the root
// roots + t*roots_stride, height proof digests at proofs + t*proofs_stride; ok[t] = 0/1.
struct MerkleVerifyParams {
  const uint8_t* leaves;
  uint64_t leaf_stride;
  uint32_t leaf_bytes;
  uint32_t height;
  const uint32_t* index;
  const uint8_t* roots;
  uint64_t roots_stride;
  const uint8_t* proofs;
  uint64_t proofs_stride;
  uint64_t n;
  uint8_t* ok;
  uint8_t* roots_out;  // derive_root mode (merkle.rs:411-428): root digests out, 32 B each; ok unused
  const uint8_t* active;  // nullable: leaves with active[t] == 0 are skipped (nothing written)
  uint32_t* list;         // nullable, n + 1 words of device scratch: with `active`, the active
                          // leaves are compacted first so that no lane idles on a skipped one
  uint8_t* leaf_nodes;    // nullable: leaf t's digest also to leaf_nodes + (t / leaves_per_tree) *
  uint64_t leaf_nodes_stride;  // leaf_nodes_stride + 32 (t % leaves_per_tree) (a later build's
  uint32_t leaves_per_tree;    // level 0, launch_merkle_build's nodes layout)
  uint64_t group_stride;       // leaf t at leaves + grouped_row_offset(t, leaf_stride, group_stride,
  uint32_t skip_row;           // skip_row) (group_stride 0: t * leaf_stride)
};
hipError_t launch_merkle_verify(const MerkleVerifyParams& p, hipStream_t stream);

// EMPTY_ROOTS[h] as big-endian words (host; the same SHA-256 code as the kernels).
void merkle_empty_roots(uint32_t out[kMerkleMaxHeight][8]);

}  // namespace ag
