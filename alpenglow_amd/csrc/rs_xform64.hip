// xform_h8: the bitsliced 64-point transform FFT_64,DOUT(IFFT_64,DIN(in)) -- HighRate encode
// and full-recovery decode for chunk 64 (64:64, k <= 64), LowRate encode per 64-point recovery
// chunk.  Replaces the crate's 64-point FFT/IFFT calls behind
// /root/reference/src/shredder/reed_solomon.rs:121-125 (encode) and :166 (decode).  gfx950.
#include <hip/hip_runtime.h>

#include "rs_device.hpp"
#include "rs_launch.hpp"
#include "rs_xform.hpp"

namespace ag {
namespace {

using dev::static_for;

// =====================================================================================
// xform_h8: the 64-point transform on 32-column tiles with the lane half as a position bit
// (decode_h8's layouts without the locator products and the derivative): 8 waves x 4 slots x 2
// lane halves, 64 KiB of swap buffer, so two 512-thread workgroups share a CU and one's loads,
// swaps and stores overlap the other's arithmetic (the round-2 xform16 ran one 1024-thread
// workgroup per CU, its load -> swaps -> store sequence exposed between tiles; removed).  Loads and
// stores are lane-linear (tile_io_l32 + quad_exchange).  The default 64-point kernel: 4.81-4.91
// vs 4.23-4.41 TB/s encode, 4.55-4.60 vs 4.22-4.37 reconstruct against xform16 on 64 KiB - 4
// MiB blocks (profiles/r03_ab_xform_h8.txt).  A first version that gave each lane one whole
// chunk (its four 16-byte pieces 64 bytes apart in every wave access) ran 2.8-3.4 TB/s
// (profiles/r03_ab_xform_h8_rejected.txt).
// Layouts (slot bits | lane half | waves):
//   A  slots p0 p1 | h p2 | waves p3 p4 p5   loads, IFFT b0; FFT b0, stores
//   B  slots p2 p1 | h p0 | waves p3 p4 p5   IFFT b1 b2 / FFT b1
//   C  slots p2 p3 | h p0 | waves p1 p4 p5   IFFT b3 / FFT b2
//   D  slots p4 p3 | h p0 | waves p1 p2 p5   IFFT b4 / FFT b3
//   E  slots p4 p5 | h p0 | waves p1 p2 p3   IFFT b5, FFT b5 b4
// =====================================================================================
// HALF: every stored shard is < 32 (position bit 5 clear; a reconstruct whose erased originals
// all lie in shards 0..31): after FFT layer 4 the waves whose slots would hold p5 = 1 hand
// over their live slots and retire (decode_h8's OUTH pruning).
// LR2: two LowRate recovery chunks of a 32-point code (k <= 32) in one launch.  The crate's
// chunk j is FFT_32,32(j+1)(IFFT_32,0(data)); FFT_64,δ of (u, 0) is (FFT_32,δ(u),
// FFT_32,δ+32(u)) because its top layer maps (u, 0) to (u, u) for any skew.  So with the data in
// positions 0..31 and nothing in 32..63, the IFFT stops before its top layer (layers 0-4 are
// the 32-point IFFT of each half; the empty half stays zero, and its waves skip them) and the
// FFT_64 at δ = 32(2i + 1) yields chunks 2i and 2i + 1 as positions 0..63: the data is read
// once and its IFFT computed once for both chunks.
template <int DIN, int DOUT, bool HALF = false, bool LR2 = false>
__global__ __launch_bounds__(512, 4) void xform_h8_kernel(const XformParams p) {
  using LB = X8Lay<2, 1, 3, 4, 5>;
  using LC = X8Lay<2, 3, 1, 4, 5>;
  using LD = X8Lay<4, 3, 1, 2, 5>;
  using LE = X8Lay<4, 5, 1, 2, 3>;
  __shared__ uint4 lds[16 * 4 * kXfLanes];  // 8 waves x 2 slots x 4 KiB
  __shared__ X8Flags flags;
  const int lane = threadIdx.x & 63;
  const int h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (threadIdx.x < 16) reinterpret_cast<uint32_t*>(&flags)[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t tile = dev::xcd_tile(blockIdx.x, gridDim.x);
  const TileIO io = tile_io_l32(p.total_columns, p.chunks_per_shard, tile, lane, p.in_block_stride);
  Regs4 r;
  static_for<4>([&](auto T) {
    constexpr int t = decltype(T)::value;
    const uint32_t s = t | (h << 2) | (wave << 3);  // layout A position
    if (s < p.n_in) {
      const uint8_t* base = p.in + s * p.in_shard_stride;
      static_for<4>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        const uint4 x = ld_piece(base + io.off[q]);
        r[t][4 * q] = x.x;
        r[t][4 * q + 1] = x.y;
        r[t][4 * q + 2] = x.z;
        r[t][4 * q + 3] = x.w;
      });
    } else {
      static_for<16>([&](auto P) { r[t][decltype(P)::value] = 0; });
    }
  });
  static_for<4>([&](auto T) {
    quad_exchange(r[decltype(T)::value], lane);
    dev::planes_from_raw(r[decltype(T)::value]);
  });
  // IFFT_64 (skew delta DIN); LR2: the waves of the empty half (p5 = wave bit 2 in A-D) hold
  // zeros through layer 4, and the top layer is not applied
  const bool ifft = !LR2 || !((wave >> 2) & 1);
  if (ifft) {
    h8_layer0<true, DIN>(wave, h, r);
    h8_relayout(r);
    x8_layer_t<LB, 1, true, DIN>(wave, r);
    x8_layer_t<LB, 2, true, DIN>(wave, r);
  }
  x8_swap<1, 0, 1>(wave, lane, lds, &flags, r);
  if (ifft) x8_layer_t<LC, 3, true, DIN>(wave, r);
  x8_swap<0, 1, 2>(wave, lane, lds, &flags, r);
  if (ifft) x8_layer_t<LD, 4, true, DIN>(wave, r);
  x8_swap<1, 2, 3>(wave, lane, lds, &flags, r);
  if constexpr (!LR2) x8_layer_t<LE, 5, true, DIN>(wave, r);
  // FFT_64 (skew delta DOUT), ending in A
  x8_layer_t<LE, 5, false, DOUT>(wave, r);
  x8_layer_t<LE, 4, false, DOUT>(wave, r);
  if constexpr (!HALF) {
    x8_swap<1, 2, 4>(wave, lane, lds, &flags, r);
  } else {
    // E -> D: slot bit 1 (p5) <-> wave bit 2 (p3).  After it a wave's slots all have p5 = its
    // wave bit 2; the waves of the p5 = 1 half only send the slots their live partner needs.
    const int partner = wave ^ 4;
    if ((wave >> 2) & 1) {
      x8_wait_ge(&flags.done[partner], 3);
      static_for<4>([&](auto T) {
        constexpr int t = decltype(T)::value;
        if constexpr (((t >> 1) & 1) == 0) {
          lds_put(lds, 2 * partner + (t & 1), lane, r[t]);
          __asm__ volatile("; xh8 put %0" ::"n"(t));
        }
      });
      x8_signal(&flags.ready[wave], 4, lane);
      return;
    }
    x8_wait_ge(&flags.ready[partner], 4);
    static_for<4>([&](auto T) {
      constexpr int t = decltype(T)::value;
      if constexpr (((t >> 1) & 1) != 0) {
        lds_get(lds, 2 * wave + (t & 1), lane, r[t]);
        __asm__ volatile("; xh8 get %0" ::"n"(t));
      }
    });
    x8_signal(&flags.done[wave], 4, lane);
  }
  x8_layer_t<LD, 3, false, DOUT>(wave, r);
  x8_swap<0, 1, 5>(wave, lane, lds, &flags, r);
  x8_layer_t<LC, 2, false, DOUT>(wave, r);
  x8_swap<1, 0, 6>(wave, lane, lds, &flags, r);
  x8_layer_t<LB, 1, false, DOUT>(wave, r);
  // store addresses computed only now; the empty asm keeps the compiler from keeping the
  // load-time divisions live across the transform (VGPR pressure)
  uint32_t tile_late = tile;
  int lane_late = lane;
  __asm__ volatile("" : "+s"(tile_late), "+v"(lane_late));
  const TileIO out_io = tile_io_l32(p.total_columns, p.chunks_per_shard, tile_late, lane_late, p.out_block_stride);
  // Every store predicate of the wave, packed before the first store (bit 4 t + q: piece q of
  // slot t): the store loop then reads no mask word.  With per-block masks re-read between
  // the slots' stores, whole lane classes of a slot intermittently skipped their stores.
  uint32_t qall = 0;
  {
    uint64_t mask[4] = {~0ull, ~0ull, ~0ull, ~0ull};
    if (p.out_mask) {
      if (!p.pattern_per_block) {
        const uint64_t m = p.out_mask[0];
        mask[0] = mask[1] = mask[2] = mask[3] = m;
      } else {
        static_for<4>([&](auto Q) { mask[decltype(Q)::value] = p.out_mask[out_io.blk[decltype(Q)::value]]; });
      }
    }
    static_for<4>([&](auto T) {
      constexpr int t = decltype(T)::value;
      const uint32_t s = t | (h << 2) | (wave << 3);
      if (s < p.n_out) qall |= store_qmask(out_io, mask, s) << (4 * t);
    });
  }
  // a wave's partner-swap duties are done: it may retire when it stores nothing
  if (__builtin_amdgcn_ballot_w64(qall != 0) == 0) return;
  h8_relayout(r);
  h8_layer0<false, DOUT>(wave, h, r);
  static_for<4>([&](auto T) {
    constexpr int t = decltype(T)::value;
    const uint32_t s = t | (h << 2) | (wave << 3);
    // the quad partners' quarters belong to the same shard: both lanes take part in the
    // exchange, each stores only its own pieces
    uint32_t v[16];
    static_for<16>([&](auto P) { v[decltype(P)::value] = r[t][decltype(P)::value]; });
    dev::transpose8(v);
    dev::transpose8(v + 8);
    quad_exchange(v, lane);
    uint8_t* base = p.out + s * p.out_shard_stride;
    static_for<4>([&](auto Q) {
      constexpr int q = decltype(Q)::value;
      if ((qall >> (4 * t + q)) & 1) st_piece(base + out_io.off[q], v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
    });
  });
}

}  // namespace

hipError_t launch_xform64(unsigned din, unsigned dout, const XformParams& p, hipStream_t stream) {
  if (p.total_columns == 0) return hipSuccess;
  const uint64_t t32 = (p.total_columns + 31) / 32;
  if (t32 > 0x7FFFFFFFull) return hipErrorInvalidValue;
  const dim3 g32(static_cast<unsigned>(t32));
  if (din == 64 && dout == 0) hipLaunchKernelGGL((xform_h8_kernel<64, 0>), g32, dim3(512), 0, stream, p);
  else if (din == 0 && dout == 64 && p.out_low_half)
    hipLaunchKernelGGL((xform_h8_kernel<0, 64, true>), g32, dim3(512), 0, stream, p);
  else if (din == 0 && dout == 64) hipLaunchKernelGGL((xform_h8_kernel<0, 64>), g32, dim3(512), 0, stream, p);
  else if (din == 0 && dout == 128) hipLaunchKernelGGL((xform_h8_kernel<0, 128>), g32, dim3(512), 0, stream, p);
  else if (din == 0 && dout == 192) hipLaunchKernelGGL((xform_h8_kernel<0, 192>), g32, dim3(512), 0, stream, p);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_xform_lowrate2(unsigned pair, const XformParams& p, hipStream_t stream) {
  if (p.total_columns == 0) return hipSuccess;
  if (p.n_in > 32 || p.n_out > 64) return hipErrorInvalidValue;
  const uint64_t t32 = (p.total_columns + 31) / 32;
  if (t32 > 0x7FFFFFFFull) return hipErrorInvalidValue;
  const dim3 g32(static_cast<unsigned>(t32));
  if (pair == 0) hipLaunchKernelGGL((xform_h8_kernel<0, 32, false, true>), g32, dim3(512), 0, stream, p);
  else if (pair == 1) hipLaunchKernelGGL((xform_h8_kernel<0, 96, false, true>), g32, dim3(512), 0, stream, p);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace ag
