// decode_c: the correction decoder for 32-point full-window geometries with lost recovery
// shards (gfx950 / CDNA4).
//
// What it replaces: the crate decoder behind ReedSolomonCoder::deshred
// (/root/reference/src/shredder/reed_solomon.rs:150-180) for HighRate k <= 32, m = 32
// when some coding shreds are missing -- the pattern a follower sees whenever a coding
// shred is lost.  Any k survivors determine the originals (MDS), so the restored bytes equal
// the crate decoder's on every valid codeword (ANY_K mode).
//
// Algorithm (rs_launch.hpp, CorrPattern): the xform8 full-recovery transform runs on the
// present recovery shards with the lost ones read as zero; at |L| known original-coset
// points (present originals, or virtual zeros past k) the difference between the transform
// output and the known value is a syndrome s_b; the erased originals are then the transform
// outputs plus K s, K = X[E, L] N^-1 built per pattern on the host.  The |E| x |L| runtime
// products run by four Russians: per syndrome and pair of 4-plane groups, the two 16-entry
// XOR tables are built once (22 VALU) and every output plane takes one wave-uniform pick
// from each (v_mov in gpr-index mode) and one 3-input XOR.
//
// Layout: xform8's (8 waves x 4 slots, 64-column tiles, two workgroups per CU), except that
// the FFT ends in layout H0 (slots p4 p0 | waves p1 p2 p3), so the restored originals of
// the usual patterns (runs of erased data shreds) spread over all eight waves.  The
// syndromes go through the 64 KiB exchange buffer (16 slots of 4 KiB) once the transform's
// swaps are done.
#include <hip/hip_runtime.h>

#include "rs_device.hpp"
#include "rs_launch.hpp"
#include "rs_xform.hpp"

namespace ag {
namespace {

// The 16 XOR combinations of planes a, b, c, d (entry n = XOR of the planes selected by n).
__device__ __forceinline__ void corr_table(uint32_t* t, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  t[0] = 0;
  t[1] = a;
  t[2] = b;
  t[3] = a ^ b;
  t[4] = c;
  t[5] = a ^ c;
  t[6] = b ^ c;
  t[7] = dev::xor3(a, b, c);
  t[8] = d;
  t[9] = a ^ d;
  t[10] = b ^ d;
  t[11] = dev::xor3(a, b, d);
  t[12] = c ^ d;
  t[13] = dev::xor3(a, c, d);
  t[14] = dev::xor3(b, c, d);
  t[15] = dev::xor3(t[3], c, d);
}

// The pattern table is read-only for the whole launch: reading it through the constant
// address space lets its wave-uniform loads be scalar (s_load) even though the kernel
// stores to global memory.
using ConstU32 = __attribute__((address_space(4))) const uint32_t;
using ConstPat = __attribute__((address_space(4))) const CorrPattern;

// acc[o] ^= (K s)[o] restricted to input groups G0, G0 + 1 (tables t0, t1); k8 = the 8
// packed row dwords of K[a][b] (wave-uniform: scalar loads).
template <int G0>
__device__ __forceinline__ void corr_acc(uint32_t* acc, const uint32_t* t0, const uint32_t* t1, ConstU32* k8) {
  static_for<8>([&](auto Q) {
    constexpr int q = decltype(Q)::value;
    const uint32_t w = k8[q];
    static_for<2>([&](auto H) {
      constexpr int o = 2 * q + decltype(H)::value;
      constexpr int sh = 16 * decltype(H)::value + 4 * G0;
      acc[o] = dev::xor3(acc[o], t0[(w >> sh) & 15], t1[(w >> (sh + 4)) & 15]);
    });
  });
}

using H3 = X8Lay<4, 3, 0, 1, 2>;
using H2 = X8Lay<4, 2, 0, 1, 3>;
using H1 = X8Lay<4, 1, 0, 2, 3>;
using H0 = X8Lay<4, 0, 1, 2, 3>;
static_assert(std::is_same_v<H3, X8Layout<3>>, "H3 is layout L3");

__global__ __launch_bounds__(512, AG_X8_WAVES_PER_EU) void decode_c_kernel(const DecodeCParams p) {
  __shared__ uint4 lds[16 * 4 * kXfLanes];  // xform8 exchange, then kCorrMaxSyn syndrome slots
  __shared__ X8Flags flags;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (threadIdx.x < 16) reinterpret_cast<uint32_t*>(&flags)[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t tile = dev::xcd_tile(blockIdx.x, gridDim.x);
  uint64_t vtile = tile, pat = 0;
  if (p.per_block) {
    const uint64_t bi = tile / p.tiles_per_block;
    const uint64_t blk = p.block_ids ? p.block_ids[bi] : bi;
    vtile = blk * p.tiles_per_block + (tile - bi * p.tiles_per_block);
    pat = blk;
  }
  // wave-uniform pattern: the mask words and K rows become scalar loads
  ConstPat* cp = (ConstPat*)(p.pat) + __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(pat));
  const uint64_t rmask = cp->rmask;
  const TileIO io_r = tile_io_g(p.total_columns, p.chunks_per_shard, vtile, lane, p.rec_block_stride);
  Regs4 r;
  static_for<4>([&](auto T) {
    constexpr int t = decltype(T)::value;
    const uint32_t sh = 4 * wave + t;  // layout L0: wave-uniform
    if ((rmask >> sh) & 1) {
      const uint8_t* base = p.rec + sh * p.rec_shard_stride;
      static_for<4>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        const uint4 x = *reinterpret_cast<const uint4*>(base + io_r.off[q]);
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
  // IFFT_32 (skew delta 0), then FFT_32 (delta 32) ending in layout H0
  x8_layer<0, 0, true, 0>(wave, r);
  x8_layer<0, 1, true, 0>(wave, r);
  x8_swap<0, 0, 1>(wave, lane, lds, &flags, r);
  x8_layer<1, 2, true, 0>(wave, r);
  x8_swap<1, 1, 2>(wave, lane, lds, &flags, r);
  x8_layer<2, 3, true, 0>(wave, r);
  x8_swap<0, 2, 3>(wave, lane, lds, &flags, r);
  x8_layer<3, 4, true, 0>(wave, r);
  x8_layer<3, 4, false, 32>(wave, r);
  x8_layer_lay<H3, 3, 32, 0xF>(wave, r);
  x8_swap<1, 2, 4>(wave, lane, lds, &flags, r);
  x8_layer_lay<H2, 2, 32, 0xF>(wave, r);
  x8_swap<1, 1, 5>(wave, lane, lds, &flags, r);
  x8_layer_lay<H1, 1, 32, 0xF>(wave, r);
  x8_swap<1, 0, 6>(wave, lane, lds, &flags, r);
  x8_layer_lay<H0, 0, 32, 0xF>(wave, r);

  const uint64_t emask = cp->emask, smask = cp->smask;
  const uint32_t ns = cp->ns;
  const TileIO io_o = tile_io_g(p.total_columns, p.chunks_per_shard, vtile, lane, p.orig_block_stride);
  __syncthreads();  // every wave's last swap reads are done: the exchange buffer is free
  // syndromes s_b = d_a - (X r')_a at the syndrome points a (rank b), into LDS slot b
  static_for<4>([&](auto T) {
    constexpr int t = decltype(T)::value;
    const uint32_t a = H0::pos(wave, t);  // wave-uniform
    if ((smask >> a) & 1) {
      if (a < p.k) {  // a present original (a virtual zero point adds nothing)
        const uint8_t* base = p.orig + a * p.orig_shard_stride;
        uint32_t d[16];
        static_for<4>([&](auto Q) {
          constexpr int q = decltype(Q)::value;
          const uint4 x = *reinterpret_cast<const uint4*>(base + io_o.off[q]);
          d[4 * q] = x.x;
          d[4 * q + 1] = x.y;
          d[4 * q + 2] = x.z;
          d[4 * q + 3] = x.w;
        });
        swap_halves(d);
        dev::planes_from_raw(d);
        dev::xor_planes(r[t], d);
      }
      const uint32_t b = static_cast<uint32_t>(__builtin_popcountll(smask & ((uint64_t{1} << a) - 1)));
      lds_put(lds, static_cast<int>(b), lane, r[t]);
    }
  });
  __syncthreads();
  uint32_t emine = 0;  // slots holding restored originals (wave-uniform)
  static_for<4>([&](auto T) {
    constexpr int t = decltype(T)::value;
    if ((emask >> H0::pos(wave, t)) & 1) emine |= 1u << t;
  });
  if (emine == 0) return;
  for (uint32_t b = 0; b < ns; ++b) {
    static_for<2>([&](auto GP) {
      constexpr int gp = decltype(GP)::value;
      uint32_t s[8];
      static_for<2>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        const uint4 x = lds[(b * 4 + 2 * gp + q) * kXfLanes + lane];
        s[4 * q] = x.x;
        s[4 * q + 1] = x.y;
        s[4 * q + 2] = x.z;
        s[4 * q + 3] = x.w;
      });
      uint32_t t0[16], t1[16];
      corr_table(t0, s[0], s[1], s[2], s[3]);
      corr_table(t1, s[4], s[5], s[6], s[7]);
      static_for<4>([&](auto T) {
        constexpr int t = decltype(T)::value;
        if ((emine >> t) & 1) {
          const uint32_t a = H0::pos(wave, t);
          const uint32_t ea = static_cast<uint32_t>(__builtin_popcountll(emask & ((uint64_t{1} << a) - 1)));
          corr_acc<2 * gp>(r[t], t0, t1, cp->kmat + 8 * (ea * ns + b));
        }
      });
    });
  }
  static_for<4>([&](auto T) {
    constexpr int t = decltype(T)::value;
    if ((emine >> t) & 1) {
      const uint32_t a = H0::pos(wave, t);
      store_shard(p.orig + a * p.orig_shard_stride, io_o, io_o.valid, r[t]);
    }
  });
}

}  // namespace

hipError_t launch_decode_c(const DecodeCParams& p, hipStream_t stream) {
  if (p.ntiles == 0) return hipSuccess;
  if (p.ntiles > 0x7FFFFFFFull || p.k > 32) return hipErrorInvalidValue;
  hipLaunchKernelGGL(decode_c_kernel, dim3(static_cast<unsigned>(p.ntiles)), dim3(512), 0, stream, p);
  return hipGetLastError();
}

}  // namespace ag
