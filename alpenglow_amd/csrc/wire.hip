// Shred wire format on the device.
//
// A received datagram is one wincode-encoded `Shred` (shredder.rs:113-186; decoded by
// network::deserialize, network.rs:52-64: DefaultConfig with preallocation capped at
// MTU_BYTES, exact consumption).  Layout (bincode-compatible wincode 0.6):
//   u32 variant | u64 slot | u64 slice_index | u8 is_last | u64 shred_index |
//   u64 data_len | data | 64 B slice_sig | u64 proof_len | proof_len x 32 B
// (oracle/shred_wire_oracle.py restates it; parity unpinned -- the reference holds no
// serialized bytes).
//
// Kernels: one wave per packet.  Lane 0 reads the fixed fields and the two lengths (the
// offsets depend on data_len), the wave then copies the data, signature and proof bytes
// lane-parallel: deserialize moves the data (at packet offset 37, unaligned) as 16-byte groups
// of words funnel-shifted with v_alignbyte, the signature and proof bytes singly; serialize
// stores 16 bytes per lane at the rows' unaligned offsets (copy16_any).  The packet bytes are
// read once and the columns written once: ~1.3 KB per shred each way.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "unaligned.hpp"
#include "wire.hpp"

namespace ag {

namespace {

__device__ __forceinline__ uint64_t ld_u64(const uint8_t* p) {
  uint64_t v = 0;
#pragma unroll
  for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
  return v;
}
__device__ __forceinline__ uint32_t ld_u32(const uint8_t* p) {
  return uint32_t(p[0]) | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 24);
}
__device__ __forceinline__ void st_u64(uint8_t* p, uint64_t v) {
#pragma unroll
  for (int i = 0; i < 8; ++i) p[i] = static_cast<uint8_t>(v >> (8 * i));
}

// Destination words [0, nw) from a source whose word w is (sw[w], sw[w + 1]) shifted right by
// sh bytes (sh = 0: sw[w] itself; sw[nw] is read only when sh != 0).  Four words per lane
// per step (dwordx4 accesses need only 4-byte alignment), the last partial group word by word.
__device__ __forceinline__ void shift_words(uint32_t* __restrict__ dw, const uint32_t* __restrict__ sw, uint32_t nw,
                                            uint32_t sh, int lane) {
  for (uint32_t w = 4 * lane; w < nw; w += 256) {
    if (w + 4 <= nw) {
      const uint4 x = ld16u(sw + w);
      uint4 o = x;
      if (sh) {
        const uint32_t e = sw[w + 4];
        o.x = __builtin_amdgcn_alignbyte(x.y, x.x, sh);
        o.y = __builtin_amdgcn_alignbyte(x.z, x.y, sh);
        o.z = __builtin_amdgcn_alignbyte(x.w, x.z, sh);
        o.w = __builtin_amdgcn_alignbyte(e, x.w, sh);
      }
      st16u(dw + w, o);
    } else {
      for (uint32_t v = w; v < nw; ++v) dw[v] = sh ? __builtin_amdgcn_alignbyte(sw[v + 1], sw[v], sh) : sw[v];
    }
  }
}
// dst[0, len) = src[0, len) for a 4-byte-aligned dst and any src whose aligned base is
// readable through src + len + 3 (the packet row continues past the data): whole words
// funnel-shifted, the tail bytes singly.  Lane-parallel.
__device__ __forceinline__ void copy_to_aligned(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
                                                uint32_t len, int lane) {
  const uint32_t mis = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(src) & 3);
  const uint32_t nw = len >> 2;
  shift_words(reinterpret_cast<uint32_t*>(dst), reinterpret_cast<const uint32_t*>(src - mis), nw, mis, lane);
  for (uint32_t i = 4 * nw + lane; i < len; i += 64) dst[i] = src[i];
}
// dst[0, len) = src[0, len) at any alignment of either: 16-byte lane accesses (gfx950 runs
// global memory in unaligned mode), the last len % 16 bytes singly.  Lane-parallel.
__device__ __forceinline__ void copy16_any(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, uint32_t len,
                                           int lane) {
  const uint32_t n16 = len >> 4;
  for (uint32_t i = lane; i < n16; i += 64)
    st16u(dst + 16 * i, ld16u(src + 16 * i));
  for (uint32_t i = 16 * n16 + lane; i < len; i += 64) dst[i] = src[i];
}
// the data rows are 4-byte aligned (every row, so word copies never leave a row)
__device__ __forceinline__ bool word_rows(const ShredColumns& c) {
  return ((reinterpret_cast<uintptr_t>(c.data) | c.data_stride | c.group_stride) & 3) == 0;
}

__global__ __launch_bounds__(256) void shred_deserialize_kernel(const uint8_t* __restrict__ packets,
                                                                uint64_t packet_stride,
                                                                const uint32_t* __restrict__ packet_lens, uint64_t n,
                                                                const ShredColumns c, uint8_t* __restrict__ status) {
  const uint64_t t = static_cast<uint64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= n) return;
  const uint8_t* pk = packets + t * packet_stride;
  // Speculation: a call's datagrams carry data_stride data bytes and a full-capacity proof (the
  // composed deshreds' rows: S bytes, 6 digests).  Their data, signature, proof length and proof
  // are loaded now, in the same round trip as the length and the header, where that layout fits
  // the packet row; the copy below uses them only if the parsed header matches (otherwise the
  // dependent loads run as before).  Every speculative access stays inside the packet row.
  const uint32_t E = static_cast<uint32_t>(c.data_stride);
  const uint32_t e_sig = kShredHeadBytes + E;
  const bool spec = E <= 1024 && c.proof_stride <= 256 && c.proof_stride % 16 == 0 &&
                    uint64_t{e_sig} + 72 + c.proof_stride <= packet_stride;
  const uint32_t len = packet_lens[t];
  uint32_t st = kWireOk;
  uint64_t dlen = 0, plen = 0;
  if (len > packet_stride) st = kWireTooLarge;  // the caller's row cannot hold it: never read past it
  else if (len < kShredHeadBytes) st = kWireMalformed;  // (an absent slot: length 0)
  uint4 s_data = make_uint4(0u, 0u, 0u, 0u), s_tail = make_uint4(0u, 0u, 0u, 0u);
  uint64_t s_plen = 0;
  if (spec && st == kWireOk && len == e_sig + 72 + c.proof_stride) {  // (loaded with the header)
    if (16u * lane < E && kShredHeadBytes + 16u * lane + 16u <= packet_stride) s_data = ld16u(pk + kShredHeadBytes + 16 * lane);
    if (lane < 4) s_tail = ld16u(pk + e_sig + 16 * lane);                                  // signature
    else if (16u * (lane - 4) < c.proof_stride) s_tail = ld16u(pk + e_sig + 72 + 16 * (lane - 4));  // proof
    s_plen = ld_u64(pk + e_sig + 64);
  }
  // header parse (wave-uniform values; every lane reads the same bytes)
  uint32_t kind = 0, is_last = 0;
  uint64_t slot = 0, si = 0, idx = 0;
  if (st == kWireOk) {
    kind = ld_u32(pk);
    slot = ld_u64(pk + 4);
    si = ld_u64(pk + 12);
    is_last = pk[20];
    idx = ld_u64(pk + 21);
    dlen = ld_u64(pk + 29);
    if (kind > 1 || is_last > 1 || si >= kMaxSlicesPerBlock || idx >= kTotalShreds || dlen > kMtuBytes ||
        kShredHeadBytes + dlen + 64 + 8 > len)
      st = kWireMalformed;
  }
  const uint32_t o_sig = kShredHeadBytes + static_cast<uint32_t>(dlen);
  const bool hit = spec && dlen == E && len == e_sig + 72 + c.proof_stride;  // the speculative loads are its fields
  if (st == kWireOk) {
    plen = hit ? s_plen : ld_u64(pk + o_sig + 64);
    // bound plen before any multiply: 32 * plen wraps in u64 for plen >= 2^59
    if (plen > kMtuBytes / 32 || o_sig + 72 + 32 * plen != len) st = kWireMalformed;  // exact consumption
  }
  if (st == kWireOk && (dlen > c.data_stride || 32 * plen > c.proof_stride)) st = kWireTooLarge;
  if (lane == 0) {
    status[t] = static_cast<uint8_t>(st);
    if (st == kWireOk) {
      c.kind[t] = static_cast<uint8_t>(kind);
      c.slot[t] = slot;
      c.slice_index[t] = si;
      c.is_last[t] = static_cast<uint8_t>(is_last);
      c.shred_index[t] = static_cast<uint32_t>(idx);
      c.data_len[t] = static_cast<uint32_t>(dlen);
      c.height[t] = static_cast<uint32_t>(plen);
    }
  }
  if (st != kWireOk) return;
  uint8_t* dd = c.data + data_row_offset(c, t);
  uint8_t* pp = c.proof + t * c.proof_stride;
  if (hit && 32 * plen == c.proof_stride) {
    // the registers hold it all: data chunk `lane`, signature pieces (lanes 0..3), proof pieces
    const uint32_t o = 16u * lane;
    if (o + 16 <= E) {
      st16u(dd + o, s_data);
    } else if (o < E) {  // the last partial chunk (E even): its bytes singly
      const uint32_t w[4] = {s_data.x, s_data.y, s_data.z, s_data.w};
      for (uint32_t i = 0; i < E - o; ++i) dd[o + i] = static_cast<uint8_t>(w[i >> 2] >> (8 * (i & 3)));
    }
    if (lane < 4) st16u(c.sig + 64 * t + 16 * lane, s_tail);
    else if (16u * (lane - 4) < c.proof_stride) st16u(pp + 16 * (lane - 4), s_tail);
    return;
  }
  if (word_rows(c)) copy_to_aligned(dd, pk + kShredHeadBytes, static_cast<uint32_t>(dlen), lane);
  else for (uint32_t i = lane; i < dlen; i += 64) dd[i] = pk[kShredHeadBytes + i];
  c.sig[64 * t + lane] = pk[o_sig + lane];
  for (uint32_t i = lane; i < 32 * plen; i += 64) pp[i] = pk[o_sig + 72 + i];
}

__global__ __launch_bounds__(256) void shred_serialize_kernel(const ShredColumns c, uint64_t n,
                                                              uint8_t* __restrict__ packets, uint64_t packet_stride,
                                                              uint32_t* __restrict__ packet_lens) {
  const uint64_t t = static_cast<uint64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= n) return;
  uint8_t* pk = packets + t * packet_stride;
  const uint32_t dlen = c.data_len[t], plen = c.height[t];
  const uint32_t o_sig = kShredHeadBytes + dlen;
  if (dlen > c.data_stride || 32ull * plen > c.proof_stride || uint64_t{o_sig} + 72 + 32ull * plen > packet_stride) {
    if (lane == 0) packet_lens[t] = 0;  // does not fit the caller's rows: nothing written
    return;
  }
  const uint64_t h = c.hdr_group > 1 ? t / c.hdr_group : t;  // header row
  if (lane == 0) {
    // the 37 header bytes as words (unaligned 16-, 4- and 1-byte stores) and the proof length
    // as 8 bytes: 5 store instructions where byte stores took 45
    const uint64_t slot = c.slot[h], si = c.slice_index[h];
    const uint32_t idx = c.shred_index[t], last = c.is_last[h] ? 1u : 0u;
    st16u(pk, make_uint4(c.kind[t], static_cast<uint32_t>(slot), static_cast<uint32_t>(slot >> 32),
                         static_cast<uint32_t>(si)));
    st16u(pk + 16, make_uint4(static_cast<uint32_t>(si >> 32), last | (idx << 8), idx >> 24,
                              dlen << 8));  // idx and dlen as u64: high bytes 0
    st4u(pk + 32, dlen >> 24);
    pk[36] = 0;
    st8u(pk + o_sig + 64, make_uint2(plen, 0));
    packet_lens[t] = o_sig + 72 + 32 * plen;
  }
  const uint8_t* dd = c.data + data_row_offset(c, t);
  // unaligned 16-byte stores (the datagram rows sit at any byte offset)
  copy16_any(pk + kShredHeadBytes, dd, dlen, lane);
  if (!c.skip_sig) copy16_any(pk + o_sig, c.sig + 64 * h, 64, lane);
  copy16_any(pk + o_sig + 72, c.proof + t * c.proof_stride, 32 * plen, lane);
}

__global__ __launch_bounds__(256) void shred_sig_patch_kernel(const ShredColumns c, uint64_t n,
                                                              uint8_t* __restrict__ packets, uint64_t packet_stride,
                                                              const uint32_t* __restrict__ packet_lens) {
  const uint64_t t = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= n || packet_lens[t] == 0) return;
  const uint64_t h = c.hdr_group > 1 ? t / c.hdr_group : t;
  uint8_t* dst = packets + t * packet_stride + kShredHeadBytes + c.data_len[t];
  const uint8_t* src = c.sig + 64 * h;
#pragma unroll
  for (int q = 0; q < 4; ++q) st16u(dst + 16 * q, ld16u(src + 16 * q));
}

}  // namespace

hipError_t launch_shred_deserialize(const uint8_t* packets, uint64_t packet_stride, const uint32_t* packet_lens,
                                    uint64_t n, const ShredColumns& c, uint8_t* status, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  if ((n + 3) / 4 > 0x7FFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(shred_deserialize_kernel, dim3(static_cast<unsigned>((n + 3) / 4)), dim3(256), 0, stream,
                     packets, packet_stride, packet_lens, n, c, status);
  return hipGetLastError();
}

hipError_t launch_shred_serialize(const ShredColumns& c, uint64_t n, uint8_t* packets, uint64_t packet_stride,
                                  uint32_t* packet_lens, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  if ((n + 3) / 4 > 0x7FFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(shred_serialize_kernel, dim3(static_cast<unsigned>((n + 3) / 4)), dim3(256), 0, stream, c, n,
                     packets, packet_stride, packet_lens);
  return hipGetLastError();
}

hipError_t launch_shred_sig_patch(const ShredColumns& c, uint64_t n, uint8_t* packets, uint64_t packet_stride,
                                  const uint32_t* packet_lens, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  if ((n + 255) / 256 > 0x7FFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(shred_sig_patch_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, stream, c, n,
                     packets, packet_stride, packet_lens);
  return hipGetLastError();
}

}  // namespace ag
