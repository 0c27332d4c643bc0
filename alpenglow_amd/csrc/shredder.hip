// Glue kernels of the composed Shredder pipeline (gfx950).
//
// What they replace: the per-slice bookkeeping around the batched stages in the
// reference's RegularShredder::shred (shredder.rs:337-345 -> data_and_coding_to_output_shreds
// :533-560) and Shredder::deshred (:282-311 -> check_merkle_tree :616-625,
// fill_missing_shreds :576-611), plus the receiver's per-shred checks
// (ValidatedShred::try_new with the blockstore's cached commitment,
// validated_shred.rs:52-81).  The stages themselves (framing, RS, Merkle, Ed25519, wire) are
// the library's other kernels; ag_shredder_*_batch in rs_api.cpp chains them.
#include <hip/hip_runtime.h>

#include "shredder.hpp"

namespace ag {
namespace {

__global__ __launch_bounds__(256) void pipe_expand_kernel(const PipeExpandParams p) {
  const uint64_t t = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= p.nslices * kPipeShreds) return;
  const uint64_t s = t / kPipeShreds;
  const uint32_t j = static_cast<uint32_t>(t % kPipeShreds);
  const bool skip = (p.skip && ((p.skip[s] >> j) & 1)) || (p.slice_ok && !p.slice_ok[s]);
  p.kind[t] = j >= p.num_data ? 1 : 0;
  p.shred_index[t] = j;
  p.data_len[t] = skip ? 0xFFFFFFFFu : p.shred_bytes;
  p.height[t] = kPipeHeight;
}

// shred t fits slot j of its slice: parsed, index j, Data for j < num_data, S bytes, 6 digests
__device__ __forceinline__ bool plausible(const ShredColumns& c, const uint8_t* wire_status, uint64_t t, uint32_t j,
                                          uint32_t S, uint32_t num_data) {
  return wire_status[t] == kWireOk && c.shred_index[t] == j && c.kind[t] == (j >= num_data ? 1 : 0) &&
         c.data_len[t] == S && c.height[t] == kPipeHeight;
}

// one 64-lane wave per slice; lane j looks at shred j
__global__ __launch_bounds__(64) void pipe_pick_kernel(const PipePickParams p) {
  const uint64_t s = blockIdx.x;
  const uint32_t j = threadIdx.x;
  const uint64_t t = s * kPipeShreds + j;
  const bool fits = plausible(p.cols, p.wire_status, t, j, p.shred_bytes, p.num_data);
  p.plausible[t] = fits ? 1 : 0;
  const uint64_t ok = __builtin_amdgcn_ballot_w64(fits);
  const uint32_t pick = ok ? static_cast<uint32_t>(__builtin_ctzll(ok)) : kPipeNone;
  if (j == 0) p.pick[s] = static_cast<uint8_t>(pick);
  if (pick == kPipeNone) return;
  const uint64_t r = s * kPipeShreds + pick;
  // payload row (2-byte aligned: S is only even), proof, signature, header
  const uint16_t* src = reinterpret_cast<const uint16_t*>(p.cols.data + data_row_offset(p.cols, r));
  uint16_t* dst = reinterpret_cast<uint16_t*>(p.g_data + s * p.shred_bytes);
  for (uint32_t i = j; i < p.shred_bytes / 2; i += kPipeShreds) dst[i] = src[i];
  const uint8_t* pp = p.cols.proof + r * p.cols.proof_stride;
  for (uint32_t i = j; i < 32 * kPipeHeight; i += kPipeShreds) p.g_proof[s * 32 * kPipeHeight + i] = pp[i];
  p.g_sig[64 * s + j] = p.cols.sig[64 * r + j];
  if (j == 0) {
    p.g_slot[s] = p.cols.slot[r];
    p.g_slice_index[s] = p.cols.slice_index[r];
    p.g_is_last[s] = p.cols.is_last[r];
    p.g_shred_index[s] = pick;
  }
}

__global__ __launch_bounds__(256) void pipe_cache_kernel(const uint8_t* pick, const uint8_t* pick_status,
                                                         uint64_t nslices, uint8_t* has_cached) {
  const uint64_t s = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (s >= nslices) return;
  has_cached[s] = pick[s] != kPipeNone && pick_status[s] == 0 ? 1 : 0;  // kShredOk
}

__global__ __launch_bounds__(64) void pipe_check_kernel(const PipeCheckParams p) {
  const uint64_t s = blockIdx.x;
  const uint32_t j = threadIdx.x;
  const uint64_t t = s * kPipeShreds + j;
  const bool valid = plausible(p.cols, p.wire_status, t, j, p.shred_bytes, p.num_data) && p.val_status[t] == 0;
  const uint64_t v = __builtin_amdgcn_ballot_w64(valid);
  if (v == 0) {
    if (j == 0) p.present[s] = 0;
    return;
  }
  const uint32_t r0 = static_cast<uint32_t>(__builtin_ctzll(v));
  const uint64_t r = s * kPipeShreds + r0;
  // keep the shreds whose commitment (header + root) equals the first kept one's
  bool same = valid && p.cols.slot[t] == p.cols.slot[r] && p.cols.slice_index[t] == p.cols.slice_index[r] &&
              p.cols.is_last[t] == p.cols.is_last[r];
  if (same) {
    const uint32_t* a = reinterpret_cast<const uint32_t*>(p.roots + 32 * t);
    const uint32_t* b = reinterpret_cast<const uint32_t*>(p.roots + 32 * r);
    for (int i = 0; i < 8; ++i) same = same && a[i] == b[i];
  }
  const uint64_t keep = __builtin_amdgcn_ballot_w64(same);
  if (j == 0) {
    p.present[s] = keep;
    p.slot[s] = p.cols.slot[r];
    p.slice_index[s] = p.cols.slice_index[r];
    p.is_last[s] = p.cols.is_last[r];
  }
  if (j < 32) p.root[32 * s + j] = p.roots[32 * r + j];
  p.sig[64 * s + j] = p.cols.sig[64 * r + j];
}

__global__ __launch_bounds__(256) void pipe_root_cmp_kernel(const uint8_t* a, const uint8_t* b, uint64_t nslices,
                                                            uint8_t* same) {
  const uint64_t s = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (s >= nslices) return;
  const uint32_t* x = reinterpret_cast<const uint32_t*>(a + 32 * s);
  const uint32_t* y = reinterpret_cast<const uint32_t*>(b + 32 * s);
  uint32_t d = 0;
  for (int i = 0; i < 8; ++i) d |= x[i] ^ y[i];
  same[s] = d == 0 ? 1 : 0;
}

__global__ __launch_bounds__(256) void pipe_merge_kernel(const uint32_t* fresh, const uint64_t* present,
                                                         const uint8_t* slice_ok, uint64_t nslices,
                                                         uint32_t* packet_lens) {
  const uint64_t t = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= nslices * kPipeShreds) return;
  const uint64_t s = t / kPipeShreds;
  const uint32_t j = static_cast<uint32_t>(t % kPipeShreds);
  if (slice_ok[s] && !((present[s] >> j) & 1)) packet_lens[t] = fresh[t];
}

dim3 grid256(uint64_t n) { return dim3(static_cast<unsigned>((n + 255) / 256)); }

// The lowest `budget` set bits of b: one step per kept bit (the host's window masks do the same,
// rs_patterns.cpp window64_masks)
__device__ __forceinline__ uint64_t keep_lowest(uint64_t b, uint32_t budget) {
  uint64_t keep = 0;
  for (uint32_t i = 0; i < budget && b; ++i, b &= b - 1) keep |= b & (~b + 1);
  return keep;
}

// ANY_K survivors of one slice's kept shreds in the W = 64 window (decode_device's rule).
// fuse: slices with exactly k = 32 kept shreds (every successful deshred of the reference's
// follower, slot_block_data.rs:343-355) also restore their absent coding shreds in the same
// window decode (decode_pk<-1>): the 32 survivors fix the codeword, so the decoder's values at
// the absent recovery positions are exactly the re-encode of the restored data
// (reed_solomon.rs:206) -- few[s] bit 1 marks them, and the separate re-encode skips them.
// Slices with surplus kept shreds keep the re-encode (present-but-unused recovery shreds are
// rewritten only when the slice succeeds).  few[s] bit 0: fewer than k kept shreds.
__global__ __launch_bounds__(256) void pipe_patterns_kernel(const uint64_t* __restrict__ present, uint64_t n,
                                                            uint64_t* __restrict__ xm, uint8_t* __restrict__ few,
                                                            uint32_t fuse) {
  const uint64_t s = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (s >= n) return;
  const uint64_t pr = present[s];
  const uint64_t ob = pr & 0xFFFFFFFFull;
  uint64_t rb = pr >> 32;
  const uint32_t cnt = static_cast<uint32_t>(__builtin_popcountll(pr));
  uint64_t in = 0, out = 0, e = 0;
  uint8_t f = cnt < kPipeData ? 1 : 0;
  if (cnt >= kPipeData && ob != 0xFFFFFFFFull) {
    rb = keep_lowest(rb, kPipeData - static_cast<uint32_t>(__builtin_popcountll(ob)));
    in = rb | (ob << 32);
    out = (~ob & 0xFFFFFFFFull) << 32;
    e = (~rb & 0xFFFFFFFFull) | out;
    if (fuse && cnt == kPipeData) {  // no surplus: every erased position is an absent shred
      out = e;
      f = 2;
    }
  }
  xm[s] = e;
  xm[n + 2 * s] = in;
  xm[n + 2 * s + 1] = out;
  few[s] = f;
}

// ANY_K survivors of one CodingOnly slice (LowRate 32:64) in the W = 128 window, decode_device's
// class-8 rule: originals i at i, recovery j at 32 + j (half 0 holds recovery 0..31, half 1
// recovery 32..63 at 64..95), the present originals then recovery shards in index order up
// to 32 survivors.  present[2 s] = data bits | coding 0..31 << 32, present[2 s + 1] = coding
// 32..63.
__global__ __launch_bounds__(256) void pipe_patterns128_kernel(const uint64_t* __restrict__ present, uint64_t n,
                                                               uint64_t* __restrict__ xm, uint8_t* __restrict__ few) {
  const uint64_t s = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (s >= n) return;
  const uint64_t p0 = present[2 * s], p1 = present[2 * s + 1] & 0xFFFFFFFFull;
  const uint64_t ob = p0 & 0xFFFFFFFFull;
  uint64_t rb = (p0 >> 32) | (p1 << 32);  // coding 0..63
  const uint32_t cnt = static_cast<uint32_t>(__builtin_popcountll(p0) + __builtin_popcountll(p1));
  uint64_t e0 = 0, e1 = 0, in0 = 0, in1 = 0, out0 = 0;
  if (cnt >= kPipeData && ob != 0xFFFFFFFFull) {
    rb = keep_lowest(rb, kPipeData - static_cast<uint32_t>(__builtin_popcountll(ob)));
    in0 = ob | ((rb & 0xFFFFFFFFull) << 32);
    in1 = rb >> 32;
    out0 = ~ob & 0xFFFFFFFFull;
    e0 = out0 | (~in0 & ~0xFFFFFFFFull);  // lost / surplus recovery 0..31
    e1 = ~in1;                            // lost / surplus recovery 32..63, positions past 95
  }
  uint64_t* q = xm + 6 * s;  // m6: erased, present, restored as (half 0, half 1) pairs
  q[0] = e0;
  q[1] = e1;
  q[2] = in0;
  q[3] = in1;
  q[4] = out0;
  q[5] = 0;
  xm[6 * n + 2 * s] = in1;      // pass 1: the other half's survivors
  xm[6 * n + 2 * s + 1] = out0;
  xm[8 * n + 2 * s] = in0;      // pass 2: the output half's survivors
  xm[8 * n + 2 * s + 1] = out0;
  few[s] = cnt < kPipeData ? 1 : 0;
}

__global__ __launch_bounds__(256) void pipe_store_mask_kernel(const uint8_t* __restrict__ few,
                                                              int64_t* __restrict__ strip,
                                                              const uint64_t* __restrict__ present, uint32_t wps,
                                                              uint64_t n, uint64_t* __restrict__ mask,
                                                              int64_t err_few, int64_t err_padding) {
  const uint64_t s = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (s >= n) return;
  uint64_t m = 0;
  const int64_t len = strip[s];
  if (!(few[s] & 1) && len >= 0) {
    // exactly k kept shreds fix the codeword: the received coding shreds are its own, so only
    // the absent ones are written (none when the decode restored them: few 2); with surplus
    // shreds every coding shred is re-encoded
    const uint64_t p0 = present[wps * s], p1 = wps == 2 ? present[wps * s + 1] : 0;
    const uint32_t cnt = static_cast<uint32_t>(__builtin_popcountll(p0) + __builtin_popcountll(p1));
    const uint64_t coding = (p0 >> 32) | (p1 << 32);  // coding shreds 0..63 present
    m = few[s] ? 0 : cnt == kPipeData ? ~coding : ~uint64_t{0};
  }
  mask[s] = m;
  // the slice's result in place: payload length, or the crate's error (too few shreds first)
  strip[s] = (few[s] & 1) ? err_few : len < 0 ? err_padding : len;
}

// Rebuild leaves of the composed deshred's check_merkle_tree: leaf (s, j) is hashed again iff
// shred j of slice s was not kept (restored by the decode), or it is a coding shred the coder
// may have rewritten (all: a slice with surplus shreds, or every slice when reencode_all).  The
// kept rows are the bytes the proof check hashed.
__global__ __launch_bounds__(256) void pipe_leaf_flags_kernel(const uint64_t* __restrict__ present, uint64_t n,
                                                              uint32_t reencode_all, uint8_t* __restrict__ flags) {
  const uint64_t t = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= n * kPipeShreds) return;
  const uint64_t s = t / kPipeShreds;
  const uint32_t j = static_cast<uint32_t>(t - s * kPipeShreds);
  const uint64_t pr = present[s];
  const bool coding_rewritten = reencode_all || __builtin_popcountll(pr) > static_cast<int>(kPipeData);
  flags[t] = (!((pr >> j) & 1) || (j >= kPipeData && coding_rewritten)) ? 1 : 0;
}

}  // namespace

hipError_t launch_pipe_expand(const PipeExpandParams& p, hipStream_t stream) {
  const uint64_t n = p.nslices * kPipeShreds;
  if (n == 0) return hipSuccess;
  if (n > 0x7FFFFFFFull * 256) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pipe_expand_kernel, grid256(n), dim3(256), 0, stream, p);
  return hipGetLastError();
}

hipError_t launch_pipe_pick(const PipePickParams& p, hipStream_t stream) {
  if (p.nslices == 0) return hipSuccess;
  if (p.nslices > 0x7FFFFFFFull || p.cols.proof_stride < 32 * kPipeHeight) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pipe_pick_kernel, dim3(static_cast<unsigned>(p.nslices)), dim3(64), 0, stream, p);
  return hipGetLastError();
}

hipError_t launch_pipe_cache_flags(const uint8_t* pick, const uint8_t* pick_status, uint64_t nslices,
                                   uint8_t* has_cached, hipStream_t stream) {
  if (nslices == 0) return hipSuccess;
  hipLaunchKernelGGL(pipe_cache_kernel, grid256(nslices), dim3(256), 0, stream, pick, pick_status, nslices,
                     has_cached);
  return hipGetLastError();
}

hipError_t launch_pipe_check(const PipeCheckParams& p, hipStream_t stream) {
  if (p.nslices == 0) return hipSuccess;
  if (p.nslices > 0x7FFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pipe_check_kernel, dim3(static_cast<unsigned>(p.nslices)), dim3(64), 0, stream, p);
  return hipGetLastError();
}

hipError_t launch_pipe_root_cmp(const uint8_t* a, const uint8_t* b, uint64_t nslices, uint8_t* same,
                                hipStream_t stream) {
  if (nslices == 0) return hipSuccess;
  hipLaunchKernelGGL(pipe_root_cmp_kernel, grid256(nslices), dim3(256), 0, stream, a, b, nslices, same);
  return hipGetLastError();
}

hipError_t launch_pipe_merge_lens(const uint32_t* fresh, const uint64_t* present, const uint8_t* slice_ok,
                                  uint64_t nslices, uint32_t* packet_lens, hipStream_t stream) {
  const uint64_t n = nslices * kPipeShreds;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(pipe_merge_kernel, grid256(n), dim3(256), 0, stream, fresh, present, slice_ok, nslices,
                     packet_lens);
  return hipGetLastError();
}

hipError_t launch_pipe_patterns(const uint64_t* present, uint64_t nslices, uint64_t* xm, uint8_t* few, bool fuse,
                                hipStream_t stream) {
  if (nslices == 0) return hipSuccess;
  hipLaunchKernelGGL(pipe_patterns_kernel, grid256(nslices), dim3(256), 0, stream, present, nslices, xm, few,
                     fuse ? 1u : 0u);
  return hipGetLastError();
}

hipError_t launch_pipe_patterns128(const uint64_t* present, uint64_t nslices, uint64_t* xm, uint8_t* few,
                                   hipStream_t stream) {
  if (nslices == 0) return hipSuccess;
  hipLaunchKernelGGL(pipe_patterns128_kernel, grid256(nslices), dim3(256), 0, stream, present, nslices, xm, few);
  return hipGetLastError();
}

hipError_t launch_pipe_store_masks(const uint8_t* few, int64_t* strip, const uint64_t* present, uint32_t wps,
                                   uint64_t nslices, uint64_t* mask, int64_t err_few, int64_t err_padding,
                                   hipStream_t stream) {
  if (nslices == 0) return hipSuccess;
  hipLaunchKernelGGL(pipe_store_mask_kernel, grid256(nslices), dim3(256), 0, stream, few, strip, present, wps, nslices,
                     mask, err_few, err_padding);
  return hipGetLastError();
}

hipError_t launch_pipe_leaf_flags(const uint64_t* present, uint64_t nslices, bool reencode_all, uint8_t* flags,
                                  hipStream_t stream) {
  if (nslices == 0) return hipSuccess;
  hipLaunchKernelGGL(pipe_leaf_flags_kernel, grid256(nslices * kPipeShreds), dim3(256), 0, stream, present, nslices,
                     reencode_all ? 1u : 0u, flags);
  return hipGetLastError();
}

}  // namespace ag
