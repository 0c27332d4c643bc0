// xform16: the bitsliced 64-point transform FFT_64,DOUT(IFFT_64,DIN(in)) -- HighRate encode
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
// xform16: the 64-point transform with xform8's scheme widened to 16 waves x 4 slots
// (64-column tiles, 1024 threads, one workgroup per CU: the swaps move 2 of 4 slots per
// wave through 128 KiB of LDS).  Every butterfly is in-lane -- no lane-half duplication
// as in xform64h -- and the per-wave state is xform8's (4 waves/SIMD).  Layouts:
//   G0 slots p0 p1 | waves p2 p3 p4 p5   IFFT b0 b1   (loads; FFT b0, stores)
//   G1 slots p2 p1 | waves p0 p3 p4 p5   IFFT b2      (FFT b1)
//   G2 slots p2 p3 | waves p0 p1 p4 p5   IFFT b3      (FFT b2)
//   G3 slots p4 p3 | waves p0 p1 p2 p5   IFFT b4      (FFT b3)
//   G4 slots p4 p5 | waves p0 p1 p2 p3   IFFT b5, FFT b5 b4
// =====================================================================================
template <int DIN, int DOUT>
__global__ __launch_bounds__(1024, 4) void xform16_kernel(const XformParams p) {
  using G0 = X8Lay<0, 1, 2, 3, 4, 5>;
  using G1 = X8Lay<2, 1, 0, 3, 4, 5>;
  using G2 = X8Lay<2, 3, 0, 1, 4, 5>;
  using G3 = X8Lay<4, 3, 0, 1, 2, 5>;
  using G4 = X8Lay<4, 5, 0, 1, 2, 3>;
  __shared__ uint4 lds[32 * 4 * kXfLanes];  // 16 waves x 2 slots x 4 KiB
  __shared__ XFlags<16> flags;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (threadIdx.x < 32) reinterpret_cast<uint32_t*>(&flags)[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t tile = dev::xcd_tile(blockIdx.x, gridDim.x);
  const TileIO io = tile_io(p, tile, lane, p.in_block_stride);
  Regs4 r;
  static_for<4>([&](auto T) {
    constexpr int t = decltype(T)::value;
    const uint32_t sh = 4 * wave + t;  // G0: wave-uniform
    if (sh < p.n_in) {
      const uint8_t* base = p.in + sh * p.in_shard_stride;
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
    swap_halves(r[decltype(T)::value]);
    dev::planes_from_raw(r[decltype(T)::value]);
  });
  x8_layer_t<G0, 0, true, DIN>(wave, r);
  x8_layer_t<G0, 1, true, DIN>(wave, r);
  x8_swap<0, 0, 1>(wave, lane, lds, &flags, r);
  x8_layer_t<G1, 2, true, DIN>(wave, r);
  x8_swap<1, 1, 2>(wave, lane, lds, &flags, r);
  x8_layer_t<G2, 3, true, DIN>(wave, r);
  x8_swap<0, 2, 3>(wave, lane, lds, &flags, r);
  x8_layer_t<G3, 4, true, DIN>(wave, r);
  x8_swap<1, 3, 4>(wave, lane, lds, &flags, r);
  x8_layer_t<G4, 5, true, DIN>(wave, r);
  x8_layer_t<G4, 5, false, DOUT>(wave, r);
  x8_layer_t<G4, 4, false, DOUT>(wave, r);
  x8_swap<1, 3, 5>(wave, lane, lds, &flags, r);
  x8_layer_t<G3, 3, false, DOUT>(wave, r);
  x8_swap<0, 2, 6>(wave, lane, lds, &flags, r);
  x8_layer_t<G2, 2, false, DOUT>(wave, r);
  x8_swap<1, 1, 7>(wave, lane, lds, &flags, r);
  x8_layer_t<G1, 1, false, DOUT>(wave, r);
  x8_swap<0, 0, 8>(wave, lane, lds, &flags, r);
  const TileIO out_io = tile_io(p, tile, lane, p.out_block_stride);
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
    const uint32_t sh = 4 * wave + decltype(T)::value;
    if (sh < p.n_out && store_qmask(out_io, mask, sh)) need = 1;
  });
  if (__builtin_amdgcn_ballot_w64(need != 0) == 0) return;
  x8_layer_t<G0, 0, false, DOUT>(wave, r);
  static_for<4>([&](auto T) {
    constexpr int t = decltype(T)::value;
    const uint32_t sh = 4 * wave + t;  // wave-uniform
    if (sh < p.n_out) store_shard(p.out + sh * p.out_shard_stride, out_io, store_qmask(out_io, mask, sh), r[t]);
  });
}

}  // namespace

hipError_t launch_xform16(unsigned din, unsigned dout, const XformParams& p, hipStream_t stream) {
  if (p.total_columns == 0) return hipSuccess;
  const uint64_t tiles = (p.total_columns + kXfLanes - 1) / kXfLanes;
  if (tiles > 0x7FFFFFFFull) return hipErrorInvalidValue;
  const dim3 grid(static_cast<unsigned>(tiles));
  if (din == 64 && dout == 0) hipLaunchKernelGGL((xform16_kernel<64, 0>), grid, dim3(1024), 0, stream, p);
  else if (din == 0 && dout == 64) hipLaunchKernelGGL((xform16_kernel<0, 64>), grid, dim3(1024), 0, stream, p);
  else if (din == 0 && dout == 128) hipLaunchKernelGGL((xform16_kernel<0, 128>), grid, dim3(1024), 0, stream, p);
  else if (din == 0 && dout == 192) hipLaunchKernelGGL((xform16_kernel<0, 192>), grid, dim3(1024), 0, stream, p);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace ag
