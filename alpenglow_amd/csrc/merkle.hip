// Slice Merkle trees on the GPU.
//
// What it replaces: the reference builds one SHA-256 Merkle tree per slice over its 64
// shreds (data shreds, then coding shreds; shredder.rs:628-632 build_merkle_tree) with
// MerkleTree::new (crypto/merkle.rs:281-333), takes the root (:337) and one proof per shred
// (create_proof, :351-370); receivers check proofs (check_proof / derive_root, :374-425)
// and rebuild the tree after decoding (check_merkle_tree, shredder.rs:616-626).
//   leaf  = SHA-256(LEAF_LABEL || shred bytes)                      (merkle.rs:457-460)
//   inner = SHA-256(LEFT_LABEL || left || RIGHT_LABEL || right)     (merkle.rs:466-468)
//   an odd node at height h pairs with EMPTY_ROOTS[h]               (merkle.rs:312-315)
// SHA-256 is the sha2 crate's (crypto/hash.rs:64-79); here it is a plain FIPS 180-4
// implementation shared by host and device.
//
// Kernels
//   merkle_leaf_kernel    one thread per leaf (all slices): SHA-256 of label || shred.
//                         Integer VALU-bound (~1.2k VALU per 64-byte SHA-256 block and
//                         lane: v_alignbit rotations, v_bitop3 sigma XORs / ch / maj, v_add3)
//   merkle_level_kernel   one launch per tree level, one thread per (slice, pair)
//   merkle_proof_kernel   one thread per leaf: its create_proof siblings
//   merkle_verify_kernel  one thread per (leaf, index, root, proof): derive_root == root.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>

#include "merkle.hpp"
#include "sha256.hpp"

namespace ag {

namespace {

using sha::hash_pair;

// SHA-256(LEAF_LABEL || data[0..len)).  A4: data is 16-byte aligned (vector loads).
// The blocks made only of data bytes (b = 1 .. T/64 - 1, T = 32 + len) are software-pipelined:
// block b + 1's four 16-byte loads are issued before block b's compression, so each lane's
// HBM latency (its leaf is 1 KiB away from its neighbours', one cache line per lane and
// instruction) hides under ~1.2k VALU of rounds instead of stalling every block.
template <bool A4>
__device__ __forceinline__ void leaf_hash(const uint8_t* __restrict__ data, uint32_t len, uint32_t out[8]) {
  uint32_t st[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) st[i] = sha::kIv[i];
  const uint32_t T = 32 + len, nblk = (T + 9 + 63) / 64;
  auto word = [&](uint32_t j) -> uint32_t {
    if constexpr (A4) {
      return reinterpret_cast<const uint32_t*>(data)[j];
    } else {
      return uint32_t(data[4 * j]) | (uint32_t(data[4 * j + 1]) << 8) | (uint32_t(data[4 * j + 2]) << 16) |
             (uint32_t(data[4 * j + 3]) << 24);
    }
  };
  auto byte = [&](uint32_t i) -> uint32_t { return data[i]; };
  auto generic = [&](uint32_t b) __attribute__((always_inline)) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = sha::leaf_msg_word(16 * b + i, len, nblk, word, byte);
    sha::compress(st, w);
  };
  if constexpr (A4) {
    const uint32_t nd = T / 64;  // blocks 1 .. nd - 1 are data only (words 16 b - 8 ..)
    uint4 nx[4];
    auto fetch = [&](uint32_t b) __attribute__((always_inline)) {
#pragma unroll
      for (int q = 0; q < 4; ++q) nx[q] = *reinterpret_cast<const uint4*>(data + 64 * b - 32 + 16 * q);
    };
    if (nd > 1) fetch(1);
    generic(0);
    for (uint32_t b = 1; b < nd; ++b) {
      uint32_t w[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        w[4 * q] = sha::bswap(nx[q].x);
        w[4 * q + 1] = sha::bswap(nx[q].y);
        w[4 * q + 2] = sha::bswap(nx[q].z);
        w[4 * q + 3] = sha::bswap(nx[q].w);
      }
      if (b + 1 < nd) fetch(b + 1);
      sha::compress(st, w);
    }
    for (uint32_t b = nd > 1 ? nd : 1; b < nblk; ++b) generic(b);
  } else {
    for (uint32_t b = 0; b < nblk; ++b) {
      uint32_t w[16];
      const uint32_t o0 = 64 * b;
      if (b > 0 && o0 + 64 <= T) {  // a block of data only: words j0 .. j0 + 15
        const uint32_t j0 = (o0 - 32) >> 2;
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = sha::bswap(word(j0 + i));
        sha::compress(st, w);
      } else {
        generic(b);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) out[i] = st[i];
}

// Digests are stored as 8 big-endian words -> 32 bytes in the crate's byte order.
__device__ __forceinline__ void store_digest(uint8_t* dst, const uint32_t h[8]) {
  uint4* d = reinterpret_cast<uint4*>(dst);
  d[0] = make_uint4(sha::bswap(h[0]), sha::bswap(h[1]), sha::bswap(h[2]), sha::bswap(h[3]));
  d[1] = make_uint4(sha::bswap(h[4]), sha::bswap(h[5]), sha::bswap(h[6]), sha::bswap(h[7]));
}
__device__ __forceinline__ void load_digest(const uint8_t* src, uint32_t h[8]) {
  const uint4* s = reinterpret_cast<const uint4*>(src);
  const uint4 a = s[0], b = s[1];
  h[0] = sha::bswap(a.x);
  h[1] = sha::bswap(a.y);
  h[2] = sha::bswap(a.z);
  h[3] = sha::bswap(a.w);
  h[4] = sha::bswap(b.x);
  h[5] = sha::bswap(b.y);
  h[6] = sha::bswap(b.z);
  h[7] = sha::bswap(b.w);
}

// Build = one kernel per tree level, every launch fully parallel over all slices (a fused
// one-wave-per-slice build left 50..98% of the lanes idle in its 6 dependent levels of 3
// compressions each: as long as the 17-block leaf phase).
//   level 0: thread (slice, leaf) hashes the leaf into nodes[slice][leaf]
//   level h: thread (slice, j) hashes nodes[off + 2j], nodes[off + 2j + 1] (or EMPTY_ROOTS[h]
//            past the end) into nodes[off + len + j]; the last level also writes the root
//   proofs:  thread (slice, leaf) copies its siblings (create_proof)
// LIST: thread i hashes leaf list[i] for i < list[nslices * n_leaves] (hash_leaf compacted)
template <bool A4, bool LIST = false>
__global__ __launch_bounds__(256) void merkle_leaf_kernel(const MerkleBuildParams p, uint8_t* nodes,
                                                          uint64_t nodes_stride) {
  uint64_t t = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if constexpr (LIST) {
    if (t >= p.list[p.nslices * p.n_leaves]) return;
    t = p.list[t];
  } else {
    if (t >= p.nslices * p.n_leaves) return;
  }
  const uint64_t s = t / p.n_leaves, j = t - s * p.n_leaves;
  uint32_t h[8];
  const uint64_t jr = j + (p.skip_leaf && j >= p.skip_leaf ? 1u : 0u);
  leaf_hash<A4>(p.leaves + s * p.slice_stride + jr * p.leaf_stride, p.leaf_bytes, h);
  store_digest(nodes + s * nodes_stride + 32 * j, h);
  if (p.n_leaves == 1) store_digest(p.roots + 32 * s, h);  // a one-leaf tree's root is the leaf
}

__global__ __launch_bounds__(256) void merkle_level_kernel(const MerkleBuildParams p, uint8_t* nodes,
                                                           uint64_t nodes_stride, uint32_t off, uint32_t len,
                                                           uint32_t height) {
  const uint32_t nlen = (len + 1) / 2;
  const uint64_t t = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= p.nslices * nlen) return;
  const uint64_t s = t / nlen, j = t - s * nlen;
  uint8_t* nd = nodes + s * nodes_stride;
  uint32_t l[8], r[8], h[8];
  load_digest(nd + 32 * (off + 2 * j), l);
  if (2 * j + 1 < len) {
    load_digest(nd + 32 * (off + 2 * j + 1), r);
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = p.empty_roots[8 * height + i];
  }
  hash_pair(l, r, h);
  store_digest(nd + 32 * (off + len + j), h);
  if (nlen == 1) store_digest(p.roots + 32 * s, h);
}

// One wave per slice: the slice's proofs are one contiguous run of n_leaves * height digests, so
// lane-consecutive 16-byte pieces make every store instruction one contiguous 1 KiB (a thread
// per leaf wrote 16 bytes per lane at a 32 * height-byte stride: 1.1 TB/s of proof bytes)
__global__ __launch_bounds__(256) void merkle_proof_kernel(const MerkleBuildParams p, const uint8_t* nodes,
                                                           uint64_t nodes_stride, uint32_t height) {
  const uint64_t s = static_cast<uint64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (s >= p.nslices) return;
  const uint32_t lane = threadIdx.x & 63;
  const uint8_t* nd = nodes + s * nodes_stride;
  uint8_t* dst = p.proofs + s * p.proofs_stride;
  const uint32_t pieces = p.n_leaves * height * 2;  // 16-byte halves of the digests
  for (uint32_t i = lane; i < pieces; i += 64) {
    const uint32_t j = i / (2 * height), r = i - j * 2 * height, h = r >> 1, half = r & 1;
    // level h starts at node offset off_h; its length l_h
    uint32_t off = 0, l = p.n_leaves;
    for (uint32_t g = 0; g < h; ++g) {
      off += l;
      l = (l + 1) / 2;
    }
    const uint32_t sib = (j >> h) ^ 1;
    uint4 v;
    if (sib >= l) {
      const uint32_t* e = p.empty_roots + 8 * h + 4 * half;
      v = make_uint4(sha::bswap(e[0]), sha::bswap(e[1]), sha::bswap(e[2]), sha::bswap(e[3]));
    } else {
      v = *reinterpret_cast<const uint4*>(nd + 32 * (off + sib) + 16 * half);
    }
    *reinterpret_cast<uint4*>(dst + 16 * static_cast<uint64_t>(i)) = v;
  }
}

// check_proof (merkle.rs:374-387, 417-428) for one leaf per thread; derive_root (:411-428)
// when roots_out is set.
// LIST: thread i verifies leaf list[i] for i < list[n] (the compacted active leaves).
template <bool A4, bool LIST>
__global__ __launch_bounds__(256) void merkle_verify_kernel(const MerkleVerifyParams p) {
  uint64_t t = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if constexpr (LIST) {
    if (t >= p.list[p.n]) return;
    t = p.list[t];
  } else {
    if (t >= p.n || (p.active && !p.active[t])) return;
  }
  uint32_t node[8];
  leaf_hash<A4>(p.leaves + grouped_row_offset(t, p.leaf_stride, p.group_stride, p.skip_row), p.leaf_bytes, node);
  if (p.leaf_nodes)
    store_digest(p.leaf_nodes + (t / p.leaves_per_tree) * p.leaf_nodes_stride + 32 * (t % p.leaves_per_tree), node);
  uint32_t idx = p.index[t];
  const uint8_t* pr = p.proofs + t * p.proofs_stride;
  for (uint32_t h = 0; h < p.height; ++h) {
    uint32_t s[8], nn[8];
    load_digest(pr + 32 * h, s);
    if (idx & 1) hash_pair(s, node, nn); else hash_pair(node, s, nn);
#pragma unroll
    for (int i = 0; i < 8; ++i) node[i] = nn[i];
    idx >>= 1;
  }
  if (p.roots_out) {  // derive_root: the root digest bytes (big-endian words)
    uint32_t* o = reinterpret_cast<uint32_t*>(p.roots_out + 32 * t);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = sha::bswap(node[i]);
    return;
  }
  uint32_t root[8];
  load_digest(p.roots + t * p.roots_stride, root);
  bool ok = true;
#pragma unroll
  for (int i = 0; i < 8; ++i) ok = ok && node[i] == root[i];
  p.ok[t] = ok ? 1 : 0;
}

// list[0 .. *count) = the t < n with active[t] != 0 (in no particular order): per 1024-thread
// workgroup one atomic on the counter (a per-wave atomic serialises 65 536 of them, 0.75 ms).
__global__ __launch_bounds__(1024) void compact_active_kernel(const uint8_t* __restrict__ active, uint64_t n,
                                                              uint32_t* count, uint32_t* __restrict__ list) {
  __shared__ uint32_t wcnt[16];
  __shared__ uint32_t base;
  const uint64_t t = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool a = t < n && active[t] != 0;
  const uint64_t m = __builtin_amdgcn_ballot_w64(a);
  if (lane == 0) wcnt[wave] = static_cast<uint32_t>(__builtin_popcountll(m));
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t tot = 0;
    for (int w = 0; w < 16; ++w) {
      const uint32_t c = wcnt[w];
      wcnt[w] = tot;
      tot += c;
    }
    base = tot ? atomicAdd(count, tot) : 0;
  }
  __syncthreads();
  if (a) list[base + wcnt[wave] + __builtin_popcountll(m & ((uint64_t{1} << lane) - 1))] = static_cast<uint32_t>(t);
}

}  // namespace

hipError_t launch_merkle_build(const MerkleBuildParams& p, uint8_t* nodes, uint64_t nodes_stride,
                               hipStream_t stream) {
  if (p.nslices == 0) return hipSuccess;
  if (p.n_leaves == 0 || p.n_leaves > kMerkleMaxLeaves || !nodes || nodes_stride % 16) return hipErrorInvalidValue;
  auto grid_of = [](uint64_t threads) { return dim3(static_cast<unsigned>((threads + 255) / 256)); };
  if ((p.nslices * p.n_leaves + 255) / 256 > 0x7FFFFFFFull) return hipErrorInvalidValue;
  const bool a16 = (reinterpret_cast<uintptr_t>(p.leaves) | p.leaf_stride | p.slice_stride) % 16 == 0;
  const dim3 g0 = grid_of(p.nslices * p.n_leaves);
  if (p.hash_leaf && p.list) {  // only the flagged leaves: compacted, so no lane idles on a known one
    const uint64_t nl = p.nslices * p.n_leaves;
    if (nl >= 0xFFFFFFFFull || hipMemsetAsync(p.list + nl, 0, 4, stream) != hipSuccess) return hipErrorInvalidValue;
    hipLaunchKernelGGL(compact_active_kernel, dim3(static_cast<unsigned>((nl + 1023) / 1024)), dim3(1024), 0, stream,
                       p.hash_leaf, nl, p.list + nl, p.list);
    if (a16) hipLaunchKernelGGL((merkle_leaf_kernel<true, true>), g0, dim3(256), 0, stream, p, nodes, nodes_stride);
    else hipLaunchKernelGGL((merkle_leaf_kernel<false, true>), g0, dim3(256), 0, stream, p, nodes, nodes_stride);
  } else if (a16) {
    hipLaunchKernelGGL((merkle_leaf_kernel<true>), g0, dim3(256), 0, stream, p, nodes, nodes_stride);
  } else {
    hipLaunchKernelGGL((merkle_leaf_kernel<false>), g0, dim3(256), 0, stream, p, nodes, nodes_stride);
  }
  uint32_t off = 0, len = p.n_leaves, height = 0;
  while (len > 1) {
    const uint32_t nlen = (len + 1) / 2;
    hipLaunchKernelGGL(merkle_level_kernel, grid_of(p.nslices * nlen), dim3(256), 0, stream, p, nodes, nodes_stride,
                       off, len, height);
    off += len;
    len = nlen;
    ++height;
  }
  if (p.proofs && height)
    hipLaunchKernelGGL(merkle_proof_kernel, grid_of(p.nslices * 64) , dim3(256), 0, stream, p, nodes, nodes_stride,
                       height);
  return hipGetLastError();
}

hipError_t launch_merkle_verify(const MerkleVerifyParams& p, hipStream_t stream) {
  if (p.n == 0) return hipSuccess;
  const uint64_t groups = (p.n + 255) / 256;
  if (groups > 0x7FFFFFFFull) return hipErrorInvalidValue;
  const bool a16 = (reinterpret_cast<uintptr_t>(p.leaves) | p.leaf_stride | p.group_stride) % 16 == 0;
  const dim3 grid(static_cast<unsigned>(groups));
  if (p.active && p.list && p.n < 0xFFFFFFFFull) {
    if (hipMemsetAsync(p.list + p.n, 0, 4, stream) != hipSuccess) return hipErrorInvalidValue;
    hipLaunchKernelGGL(compact_active_kernel, dim3(static_cast<unsigned>((p.n + 1023) / 1024)), dim3(1024), 0, stream,
                       p.active, p.n, p.list + p.n, p.list);
    if (a16) hipLaunchKernelGGL((merkle_verify_kernel<true, true>), grid, dim3(256), 0, stream, p);
    else hipLaunchKernelGGL((merkle_verify_kernel<false, true>), grid, dim3(256), 0, stream, p);
  } else if (a16) {
    hipLaunchKernelGGL((merkle_verify_kernel<true, false>), grid, dim3(256), 0, stream, p);
  } else {
    hipLaunchKernelGGL((merkle_verify_kernel<false, false>), grid, dim3(256), 0, stream, p);
  }
  return hipGetLastError();
}

// EMPTY_ROOTS (merkle.rs:62-157): hash_leaf([]) then hash_pair(node, node) per height.
void merkle_empty_roots(uint32_t out[kMerkleMaxHeight][8]) {
  uint32_t st[8], w[16];
  for (int i = 0; i < 8; ++i) st[i] = sha::kIv[i];
  for (int i = 0; i < 8; ++i) w[i] = sha::kLeafLabel.w[i];
  w[8] = 0x80000000u;
  for (int i = 9; i < 15; ++i) w[i] = 0;
  w[15] = 32 * 8;
  sha::compress(st, w);
  for (int i = 0; i < 8; ++i) out[0][i] = st[i];
  for (int h = 1; h < kMerkleMaxHeight; ++h) sha::hash_pair(out[h - 1], out[h - 1], out[h]);
}

}  // namespace ag
