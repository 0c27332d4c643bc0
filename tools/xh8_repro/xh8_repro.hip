// DIAGNOSTIC ONLY (not part of the library): a reconstruction of the first xform_h8, whose
// store loop re-derived each slot's store predicate from the per-block mask words and which
// intermittently skipped whole lane classes' stores.  Built by
// tools/xh8_repro/build.sh into tools/xh8_repro/_build/libxh8_repro.so and driven by
// tools/xh8_repro/run.py: MODE 0 = that store loop; MODE 1 = the same with s_waitcnt(0) after
// every store; MODE 2 = the same with one s_waitcnt(0) before the first store (every older load
// retired, the stores still back to back and followed by EXEC writes).  The product kernel (rs_xform64.hip) packs the predicates before the first store.
#include <hip/hip_runtime.h>

#include "rs_device.hpp"
#include "rs_launch.hpp"
#include "rs_xform.hpp"

namespace ag {
namespace {
using dev::static_for;

template <int DIN, int DOUT, int MODE>
__global__ __launch_bounds__(512, 4) void xh8_repro_kernel(const XformParams p) {
  constexpr bool HALF = false;
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
  // IFFT_64 (skew delta DIN)
  h8_layer0<true, DIN>(wave, h, r);
  h8_relayout(r);
  x8_layer_t<LB, 1, true, DIN>(wave, r);
  x8_layer_t<LB, 2, true, DIN>(wave, r);
  x8_swap<1, 0, 1>(wave, lane, lds, &flags, r);
  x8_layer_t<LC, 3, true, DIN>(wave, r);
  x8_swap<0, 1, 2>(wave, lane, lds, &flags, r);
  x8_layer_t<LD, 4, true, DIN>(wave, r);
  x8_swap<1, 2, 3>(wave, lane, lds, &flags, r);
  x8_layer_t<LE, 5, true, DIN>(wave, r);
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
  uint64_t mask[4] = {~0ull, ~0ull, ~0ull, ~0ull};
  if (p.out_mask) {
    if (!p.pattern_per_block) {
      const uint64_t m = p.out_mask[0];
      mask[0] = mask[1] = mask[2] = mask[3] = m;
    } else {
      static_for<4>([&](auto Q) { mask[decltype(Q)::value] = p.out_mask[out_io.blk[decltype(Q)::value]]; });
    }
  }
  uint32_t need = 0;
  static_for<4>([&](auto T) {
    const uint32_t s = decltype(T)::value | (h << 2) | (wave << 3);
    if (s < p.n_out) need |= store_qmask(out_io, mask, s);
  });
  if (__builtin_amdgcn_ballot_w64(need != 0) == 0) return;
  h8_relayout(r);
  h8_layer0<false, DOUT>(wave, h, r);
  if constexpr (MODE == 2) __builtin_amdgcn_s_waitcnt(0);  // the mask loads retired before the first store
  static_for<4>([&](auto T) {
    constexpr int t = decltype(T)::value;
    const uint32_t s = t | (h << 2) | (wave << 3);
    // MODE 0: the slot's predicate re-derived from the mask words here (the first xform_h8)
    const uint32_t qm = s < p.n_out ? store_qmask(out_io, mask, s) : 0u;
    uint32_t v[16];
    static_for<16>([&](auto P) { v[decltype(P)::value] = r[t][decltype(P)::value]; });
    dev::transpose8(v);
    dev::transpose8(v + 8);
    quad_exchange(v, lane);
    uint8_t* base = p.out + s * p.out_shard_stride;
    static_for<4>([&](auto Q) {
      constexpr int q = decltype(Q)::value;
      if ((qm >> q) & 1) {
        st_piece(base + out_io.off[q], v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
        if constexpr (MODE == 1) __builtin_amdgcn_s_waitcnt(0);  // every store retired before the next exec change
      }
    });
  });
}

}  // namespace
}  // namespace ag

extern "C" int xh8_repro_decode(int mode, const ag::XformParams* p, void* stream) {
  const uint64_t t32 = (p->total_columns + 31) / 32;
  const dim3 g(static_cast<unsigned>(t32));
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (mode == 0) hipLaunchKernelGGL((ag::xh8_repro_kernel<0, 64, 0>), g, dim3(512), 0, s, *p);
  else if (mode == 1) hipLaunchKernelGGL((ag::xh8_repro_kernel<0, 64, 1>), g, dim3(512), 0, s, *p);
  else hipLaunchKernelGGL((ag::xh8_repro_kernel<0, 64, 2>), g, dim3(512), 0, s, *p);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
