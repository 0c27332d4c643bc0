// Slice payload framing kernels (gfx950).
//
// What they replace: Slice::payload_bytes (/root/reference/src/types/slice.rs:73-84), the
// bytes RegularShredder::shred hands to ReedSolomonCoder::shred (shredder.rs:337-345), and
// SlicePayload::try_from (slice.rs:211-218), which Shredder::deshred applies to the coder's
// output (shredder.rs:282-311).  wincode default config: Option tag byte, fixed-width LE
// integers, Vec<u8> = u64 length + bytes.  Both run in place on the batched coder's
// codeword buffers, so framing + padding + encode and deshred + parse never leave HBM.
#include <hip/hip_runtime.h>

#include "../../include/alpenglow_rs.h"
#include "slice.hpp"

namespace ag {
namespace {

// One 256-thread workgroup per slice; each thread writes whole dwords of the framed
// payload (header bytes, data bytes, and zeros past the end up to the next dword), four at
// a time where they are all data.
__global__ __launch_bounds__(256) void slice_frame_kernel(const SliceFrameParams p) {
  const uint64_t b = blockIdx.x;
  if (b >= p.n) return;
  const uint32_t has_parent = p.parent_flags[b] != 0;
  const uint32_t hdr = 1 + (has_parent ? kBlockIdBytes : 0) + 8;
  const uint32_t len = p.data_lens[b];
  const uint32_t total = hdr + len;
  const uint8_t* id = p.parent_ids + b * kBlockIdBytes;
  const uint8_t* src = p.data + b * p.data_stride;
  uint32_t* dst = reinterpret_cast<uint32_t*>(p.cw + b * p.cw_stride);
  auto byte_at = [&](uint32_t i) -> uint32_t {
    if (i >= hdr) return i < total ? src[i - hdr] : 0u;
    if (i == 0) return has_parent;
    if (has_parent && i <= kBlockIdBytes) return id[i - 1];
    const uint32_t k = i - (hdr - 8);  // byte k of the u64 LE length
    return k < 4 ? (len >> (8 * k)) & 0xFFu : 0u;
  };
  auto word_at = [&](uint32_t w) {
    const uint32_t i = 4 * w;
    return byte_at(i) | (byte_at(i + 1) << 8) | (byte_at(i + 2) << 16) | (byte_at(i + 3) << 24);
  };
  // Groups of four destination words.  A group wholly inside the data, with its source words
  // inside the data row, is five aligned source words funnel-shifted by the header length
  // (v_alignbyte); the rest (header, the last words) go byte by byte.
  const bool wsrc = ((reinterpret_cast<uintptr_t>(p.data) | p.data_stride) & 3) == 0;
  const uint32_t nwords = (total + 3) / 4;
  const uint32_t* sw = reinterpret_cast<const uint32_t*>(src);
  for (uint32_t g = threadIdx.x; 4 * g < nwords; g += blockDim.x) {
    const uint32_t w0 = 4 * g, i0 = 4 * w0;
    if (wsrc && i0 >= hdr && i0 + 16 <= total && (i0 - hdr) + 20 <= p.data_stride) {
      const uint32_t j = i0 - hdr, sh = j & 3, q = j >> 2;
      const uint4 x = *reinterpret_cast<const uint4*>(sw + q);  // 4-byte aligned: fine for dwordx4
      uint4 o = x;
      if (sh) {  // the fifth word holds a valid data byte only when sh != 0
        const uint32_t e = sw[q + 4];
        o.x = __builtin_amdgcn_alignbyte(x.y, x.x, sh);
        o.y = __builtin_amdgcn_alignbyte(x.z, x.y, sh);
        o.z = __builtin_amdgcn_alignbyte(x.w, x.z, sh);
        o.w = __builtin_amdgcn_alignbyte(e, x.w, sh);
      }
      *reinterpret_cast<uint4*>(dst + w0) = o;
    } else {
      for (uint32_t w = w0; w < w0 + 4 && w < nwords; ++w) dst[w] = word_at(w);
    }
  }
}

__device__ __forceinline__ uint64_t ld_u64_bytes(const uint8_t* q) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; --i) v = (v << 8) | q[i];
  return v;
}

// One thread per slice: the header is at most 49 bytes; the data stays in place.
__global__ __launch_bounds__(256) void slice_parse_kernel(const SliceParseParams p) {
  const uint64_t b = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b >= p.n) return;
  const int64_t n = p.payload_lens[b];
  const uint8_t* q = p.cw + b * p.cw_stride;
  uint8_t st = AG_SLICE_OK, flag = 0;
  uint32_t off = 0, dlen = 0;
  if (n < 0) {
    st = AG_SLICE_NO_PAYLOAD;
  } else if (n > static_cast<int64_t>(kSliceMaxData)) {
    st = AG_SLICE_TOO_LARGE;  // checked before decoding (slice.rs:212-214)
  } else if (n < 1 || q[0] > 1) {
    st = AG_SLICE_BAD_ENCODING;  // Option tag must be 0 or 1
  } else {
    flag = q[0];
    off = 1 + (flag ? kBlockIdBytes : 0);
    if (static_cast<uint64_t>(n) < off + 8) {
      st = AG_SLICE_BAD_ENCODING;
    } else {
      const uint64_t l = ld_u64_bytes(q + off);
      off += 8;
      // preallocation capped at MAX_DATA_PER_SLICE, then exact consumption (slice.rs:215-216)
      if (l > kSliceMaxData || off + l != static_cast<uint64_t>(n)) st = AG_SLICE_BAD_ENCODING;
      else dlen = static_cast<uint32_t>(l);
    }
  }
  p.status[b] = st;
  p.parent_flags[b] = st == AG_SLICE_OK ? flag : 0;
  for (uint32_t i = 0; i < kBlockIdBytes; ++i)
    p.parent_ids[b * kBlockIdBytes + i] = (st == AG_SLICE_OK && flag) ? q[1 + i] : 0;
  p.data_offsets[b] = st == AG_SLICE_OK ? off : 0;
  p.data_lens[b] = dlen;
}

}  // namespace

hipError_t launch_slice_frame(const SliceFrameParams& p, hipStream_t stream) {
  if (p.n == 0) return hipSuccess;
  if (p.n > 0x7FFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(slice_frame_kernel, dim3(static_cast<unsigned>(p.n)), dim3(256), 0, stream, p);
  return hipGetLastError();
}

hipError_t launch_slice_parse(const SliceParseParams& p, hipStream_t stream) {
  if (p.n == 0) return hipSuccess;
  const uint64_t groups = (p.n + 255) / 256;
  if (groups > 0x7FFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(slice_parse_kernel, dim3(static_cast<unsigned>(groups)), dim3(256), 0, stream, p);
  return hipGetLastError();
}

}  // namespace ag
