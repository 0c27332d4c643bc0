// HIP kernels for the Reed-Solomon shredder path (gfx950 / CDNA4).
//
// What they replace: the reed-solomon-simd 3.1.0 calls inside ReedSolomonCoder
// (/root/reference/src/shredder/reed_solomon.rs:96-125 encode, :150-180 decode,
// :211-231 re-encode).  Arithmetic: GF(2^16) Leopard additive FFT.
//
// Kernels
//   xform_kernel<NW>  bitsliced IFFT-N + FFT-N over one N = 32 or 64 point block; HighRate
//                     encode (k <= m, next_pow2(m) = N) and decode-from-a-full-recovery-set
//                     (m = N).  HBM-bound.
//   generic_*         table-driven crate algorithm for every geometry (correctness path:
//                     multi-chunk HighRate, LowRate, exact decode with any erasures).
//   locator_kernel    erasure-locator logs (crate eval_poly: FWHT over 65536 in LDS).
//   fill_splitmix     synthetic input blocks (bench / tests), generated on the device.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "rs_device.hpp"
#include "rs_launch.hpp"
#include "rs_xform.hpp"


namespace ag {
namespace {

using dev::static_for;


// One 64-chunk tile per workgroup of NW waves.  N = 32: 64 KiB LDS, two workgroups per
// CU; N = 64: 128 KiB LDS, one workgroup (8 waves) per CU.
// TAIL 1: shards end in the crate's split tail chunk (XformParams::tail_bytes, rs_xform.hpp).
template <int NW, int DIN, int DOUT, int TAIL = 0>
__global__ __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) void xform_kernel(const XformParams p) {
  __shared__ uint4 lds[4 * NW * 4 * kXfLanes];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t tile = dev::xcd_tile(blockIdx.x, gridDim.x);
  if (p.skip_idle) {  // per-block masks: a tile none of whose blocks stores anything exits
    const uint64_t col = static_cast<uint64_t>(tile) * kXfLanes + lane;
    const uint64_t m = col < p.total_columns ? p.out_mask[col / p.chunks_per_shard] : 0;
    if (__builtin_amdgcn_ballot_w64(m != 0) == 0) return;
  }
  Regs8 ra;
  xf_load_raw<TAIL>(p, tile_io<TAIL>(p, tile, lane, p.in_block_stride), wave, ra);
  // Store-mask words, fetched now so their latency hides under the data loads.  With
  // one pattern for the batch the word is wave-uniform (scalar load).
  uint64_t mask[4] = {~0ull, ~0ull, ~0ull, ~0ull};
  if (p.out_mask) {
    if (!p.pattern_per_block) {
      const uint64_t m = p.out_mask[0];
      mask[0] = mask[1] = mask[2] = mask[3] = m;
    } else {
      const TileIO io = tile_io<TAIL>(p, tile, lane, p.out_block_stride);  // the stores' column order
      static_for<4>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        mask[q] = p.out_mask[io.blk[q]];
      });
    }
  }

  if constexpr (TAIL == 1) {
    const TileIO in_io = tile_io<TAIL>(p, tile, lane, p.in_block_stride);
    static_for<8>([&](auto T) { tail_fix_all<TAIL>(in_io, ra[decltype(T)::value]); });
  }
  static_for<8>([&](auto T) {
    swap_halves(ra[decltype(T)::value]);
    dev::planes_from_raw(ra[decltype(T)::value]);
  });
  xf_pass_a<NW, DIN>(wave, ra);
  Regs8 rb;
  xf_exchange_ab<NW>(wave, lane, lds, ra, rb);
  xf_pass_b<NW, DIN, DOUT>(rb);
  xf_exchange_bc<NW>(wave, lane, lds, rb, ra);

  // pass C only where some lane of the wave stores one of its 8 shards (a decode restores
  // only the erased originals)
  const TileIO out_io = tile_io<TAIL>(p, tile, lane, p.out_block_stride);
  const uint32_t qall = qmask_all<8>(out_io, mask, 8 * wave, p.n_out);  // 32 bits: 8 shards x 4 pieces
  if (__builtin_amdgcn_ballot_w64(qall != 0) == 0) return;
  xf_pass_c<NW, DOUT>(wave, ra);
  static_for<8>([&](auto T) {
    constexpr int t = decltype(T)::value;
    const uint32_t s = 8 * wave + t;  // wave-uniform
    const uint32_t q = (qall >> (4 * t)) & 15u;
    // a slot no lane stores skips its planes -> bytes conversion (a decode restores a subset)
    if (s < p.n_out && __builtin_amdgcn_ballot_w64(q != 0) != 0)
      store_shard<false, TAIL>(p.out + s * p.out_shard_stride, out_io, q, ra[t]);
  });
}

// HALF: every stored output has position bit 4 clear (a decode whose erased originals all
// lie in shards 0..15).  After FFT layer 4 only the x halves are needed (no y update),
// and the remaining 16-point FFT runs on the two live slots per wave (slot bit 0 = p4 = 0)
// with one slot moved per exchange; the stores are two shards per wave:
//   H3 slots p4 p3 | waves p0 p1 p2   FFT b4 (x only), b3
//   H2 slots p4 p2 | waves p0 p1 p3   FFT b2
//   H1 slots p4 p1 | waves p0 p2 p3   FFT b1
//   H0 slots p4 p0 | waves p1 p2 p3   FFT b0, store shards 2w, 2w + 1
// One tile (flags zeroed by the caller, every wave of the 512-thread workgroup calls it):
// xform8_kernel's grid and the per-call server's jobs (latency_server_kernel).
template <int DIN, int DOUT, bool HALF = false, int TAIL = 0>
__device__ __forceinline__ void xform8_tile(const XformParams& p, uint32_t tile, uint4* lds, X8Flags* fl) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const TileIO io = tile_io<TAIL>(p, tile, lane, p.in_block_stride);
  Regs4 r;
  // a tile past the batch's last column (one slice per call: 16 of 64 columns) loads only
  // its existing pieces -- over PCIe from mapped host memory, the idle re-reads were 3/4 of
  // the per-call server's input traffic
  const bool whole = p.total_columns >= (static_cast<uint64_t>(tile) + 1) * kXfLanes;
  static_for<4>([&](auto T) {
    constexpr int t = decltype(T)::value;
    const uint32_t sh = 4 * wave + t;  // LA: wave-uniform
    if (sh < p.n_in) {
      const uint8_t* base = p.in + sh * p.in_shard_stride;
      static_for<4>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        uint4 x = make_uint4(0, 0, 0, 0);
        if (whole || ((io.valid >> q) & 1)) x = ld_piece_io<TAIL>(base, io, q);
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
    tail_fix_all<TAIL>(io, r[decltype(T)::value]);
    swap_halves(r[decltype(T)::value]);
    dev::planes_from_raw(r[decltype(T)::value]);
  });
  x8_layer<0, 0, true, DIN>(wave, r);
  x8_layer<0, 1, true, DIN>(wave, r);
  x8_swap<0, 0, 1>(wave, lane, lds, fl, r);
  x8_layer<1, 2, true, DIN>(wave, r);
  x8_swap<1, 1, 2>(wave, lane, lds, fl, r);
  x8_layer<2, 3, true, DIN>(wave, r);
  x8_swap<0, 2, 3>(wave, lane, lds, fl, r);
  if constexpr (HALF) {
    using H3 = X8Lay<4, 3, 0, 1, 2>;
    using H2 = X8Lay<4, 2, 0, 1, 3>;
    using H1 = X8Lay<4, 1, 0, 2, 3>;
    using H0 = X8Lay<4, 0, 1, 2, 3>;
    static_assert(std::is_same_v<H3, X8Layout<3>>, "H3 is layout L3");
    x8_layer<3, 4, true, DIN>(wave, r);
    x8_layer<3, 4, false, DOUT, 0x5, false>(wave, r);
    x8_layer_lay<H3, 3, DOUT, 0x5>(wave, r);
    x8_swap<1, 2, 4, 0x5>(wave, lane, lds, fl, r);
    x8_layer_lay<H2, 2, DOUT, 0x5>(wave, r);
    x8_swap<1, 1, 5, 0x5>(wave, lane, lds, fl, r);
    x8_layer_lay<H1, 1, DOUT, 0x5>(wave, r);
    x8_swap<1, 0, 6, 0x5>(wave, lane, lds, fl, r);
    const TileIO out_io = tile_io<TAIL>(p, tile, lane, p.out_block_stride);
    uint64_t mask[4] = {~0ull, ~0ull, ~0ull, ~0ull};
    if (p.out_mask) {
      if (!p.pattern_per_block) {
        const uint64_t m = p.out_mask[0];
        mask[0] = mask[1] = mask[2] = mask[3] = m;
      } else {
        static_for<4>([&](auto Q) { mask[decltype(Q)::value] = p.out_mask[out_io.blk[decltype(Q)::value]]; });
      }
    }
    // store predicates packed before the first store (bits 4 u + q; see qmask_all)
    const uint32_t qall = qmask_all<2>(out_io, mask, 2 * wave, p.n_out);
    if (__builtin_amdgcn_ballot_w64(qall != 0) == 0) return;
    x8_layer_lay<H0, 0, DOUT, 0x5>(wave, r);
    static_for<2>([&](auto U) {
      constexpr int t = 2 * decltype(U)::value;
      const uint32_t sh = 2 * wave + (t >> 1);  // H0 position of live slot t
      if (sh < p.n_out) store_shard<false, TAIL>(p.out + sh * p.out_shard_stride, out_io, (qall >> (4 * (t >> 1))) & 15u, r[t]);
    });
    return;
  }
  x8_layer<3, 4, true, DIN>(wave, r);
  x8_layer<3, 4, false, DOUT>(wave, r);
  x8_layer<3, 3, false, DOUT>(wave, r);
  x8_swap<0, 2, 4>(wave, lane, lds, fl, r);
  x8_layer<2, 2, false, DOUT>(wave, r);
  x8_swap<1, 1, 5>(wave, lane, lds, fl, r);
  x8_layer<1, 1, false, DOUT>(wave, r);
  x8_swap<0, 0, 6>(wave, lane, lds, fl, r);
  // store masks fetched only now: live across the transform they cost registers (spills)
  const TileIO out_io = tile_io<TAIL>(p, tile, lane, p.out_block_stride);
  uint64_t mask[4] = {~0ull, ~0ull, ~0ull, ~0ull};
  if (p.out_mask) {
    if (!p.pattern_per_block) {
      const uint64_t m = p.out_mask[0];
      mask[0] = mask[1] = mask[2] = mask[3] = m;
    } else {
      static_for<4>([&](auto Q) { mask[decltype(Q)::value] = p.out_mask[out_io.blk[decltype(Q)::value]]; });
    }
  }
  const uint32_t qall = qmask_all<4>(out_io, mask, 4 * wave, p.n_out);
  // slots some lane stores (wave-uniform): a decode restores only the erased originals, so
  // the last FFT layer skips butterflies with no stored output (y not updated where only x is
  // stored) and unstored slots skip their planes -> bytes conversion
  uint32_t need = 0;
  static_for<4>([&](auto T) {
    constexpr int t = decltype(T)::value;
    if (__builtin_amdgcn_ballot_w64(((qall >> (4 * t)) & 15u) != 0) != 0) need |= 1u << t;
  });
  if (need == 0) return;
  {
    using L0 = X8Layout<0>;
    const int v = x8_compress<L0::rel(0)>(wave);
    if (need & 3u) x8_bfly_w<L0, 0, false, DOUT, 0>(v, r[0], r[1], (need & 2u) != 0);
    if (need & 12u) x8_bfly_w<L0, 0, false, DOUT, 2>(v, r[2], r[3], (need & 8u) != 0);
  }
  static_for<4>([&](auto T) {
    constexpr int t = decltype(T)::value;
    const uint32_t sh = 4 * wave + t;  // wave-uniform
    if (((need >> t) & 1u) && sh < p.n_out)
      store_shard<false, TAIL>(p.out + sh * p.out_shard_stride, out_io, (qall >> (4 * t)) & 15u, r[t]);
  });
}

template <int DIN, int DOUT, bool HALF = false, int TAIL = 0>
__global__ __launch_bounds__(512, 4) void xform8_kernel(const XformParams p) {
  __shared__ uint4 lds[16 * 4 * kXfLanes];  // 8 waves x 2 slots x 4 KiB
  __shared__ X8Flags flags;
  if (threadIdx.x < 16) reinterpret_cast<uint32_t*>(&flags)[threadIdx.x] = 0;
  __syncthreads();
  xform8_tile<DIN, DOUT, HALF, TAIL>(p, dev::xcd_tile(blockIdx.x, gridDim.x), lds, &flags);
}

// =====================================================================================
// decode_x<NW>: the crate's HighRate decoder for any erasure
// pattern, bitsliced, over a W = 8*NW point window (W = next_pow2(chunk + k) in {32, 64}):
//   pass A : load present positions (recovery j < chunk, original chunk + i), multiply by
//            the pattern's locator constant (runtime 16x16 GF(2) matrix), IFFT dist 1..4
//   pass B : IFFT dist 8.., formal derivative, FFT ..8
//   pass C : FFT dist 4..1, multiply erased originals by the inverse locator, store
// Position j sits where shard j sits in xform<NW>.  The formal derivative
//   w'[j] = w[j] ^ XOR_{b : bit b of j clear} w[j | 2^b]     (all terms pre-derivative)
// splits in layout B into slot bits (in-lane) and wave bits (partner waves through LDS).
// Pattern constants come from decode_rows_kernel; one pattern per tile (either one
// pattern for the batch, or tiles that never straddle blocks).
// =====================================================================================

// x <- M x for a runtime 16x16 GF(2) matrix (rows[o] bit i = M[o][i], wave-uniform rows) by
// four Russians: per group of 4 input planes, the 16 XOR combinations (11 XORs); output plane
// o is then the XOR of 4 combinations picked by the row's nibbles.  The nibbles are
// wave-uniform, so each pick is one v_movrels (M0 index) instead of 4 bitop3s: 44 + 16 * 5
// VALU per multiply instead of 256 masked XORs (+ the mask extraction).
__device__ __forceinline__ void mul_rt4(uint32_t* x, const uint32_t* __restrict__ rows) {
  uint32_t t0[16], t1[16], t2[16], t3[16];
  auto build = [&](uint32_t* t, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
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
  };
  build(t0, x[0], x[1], x[2], x[3]);
  build(t1, x[4], x[5], x[6], x[7]);
  build(t2, x[8], x[9], x[10], x[11]);
  build(t3, x[12], x[13], x[14], x[15]);
  static_for<16>([&](auto O) {
    constexpr int o = decltype(O)::value;
    const uint32_t r = __builtin_amdgcn_readfirstlane(rows[o]);
    x[o] = dev::xor3(t0[r & 15], t1[(r >> 4) & 15], t2[(r >> 8) & 15]) ^ t3[(r >> 12) & 15];
  });
}

__device__ __forceinline__ void lds_get_xor(const uint4* lds, int slot, int lane, uint32_t* v) {
  static_for<4>([&](auto Q) {
    constexpr int q = decltype(Q)::value;
    const uint4 x = lds[(slot * 4 + q) * kXfLanes + lane];
    v[4 * q] ^= x.x;
    v[4 * q + 1] ^= x.y;
    v[4 * q + 2] ^= x.z;
    v[4 * q + 3] ^= x.w;
  });
}

// Formal derivative in layout B (slot t of wave w = position w + NW*t).
template <int NW>
__device__ __forceinline__ void xf_derivative(int wave, int lane, uint4* lds, Regs8& r) {
  constexpr int LNW = NW == 4 ? 2 : 3;
  static_for<2>([&](auto Rho) {
    constexpr int rho = decltype(Rho)::value;
    static_for<4>([&](auto U) { lds_put(lds, 4 * wave + decltype(U)::value, lane, r[4 * rho + decltype(U)::value]); });
    __syncthreads();
    // slot bits, ascending t: partners t | 2^tb > t still hold pre-derivative values
    static_for<4>([&](auto U) {
      constexpr int t = 4 * rho + decltype(U)::value;
      static_for<3>([&](auto TB) {
        constexpr int tb = decltype(TB)::value;
        if constexpr (!((t >> tb) & 1)) dev::xor_planes(r[t], r[t | (1 << tb)]);
      });
    });
    // wave bits: partner waves' pre-derivative slots from LDS
    static_for<LNW>([&](auto B) {
      constexpr int b = decltype(B)::value;
      if (!((wave >> b) & 1)) {
        const int pw = wave | (1 << b);
        static_for<4>([&](auto U) { lds_get_xor(lds, 4 * pw + decltype(U)::value, lane, r[4 * rho + decltype(U)::value]); });
      }
    });
    __syncthreads();
  });
}

// PL: per-lane patterns (tiles straddle blocks: shard sizes below 4 KiB, e.g. the 1 KiB
// shreds of the reference's slices).  Every lane then owns one whole 64-byte chunk of one
// block (four 16-byte loads of its own chunk, no lane exchange), reads its block's pattern
// masks and matrices, and multiplies with mul_rt_lane; the transform itself is unchanged
// (its skew constants never depend on the pattern).
template <int NW, bool PL = false>
__global__ __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) void decode_x_kernel(const DecodeXParams p) {
  constexpr int W = 8 * NW;
  __shared__ uint4 lds[4 * NW * 4 * kXfLanes];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t tile = dev::xcd_tile(blockIdx.x, gridDim.x);
  uint64_t in_mask, out_mask;
  const uint32_t* rows;
  TileIO io_r, io_o;
  uint64_t off_r = 0, off_o = 0;
  if constexpr (PL) {
    const uint64_t g0 = static_cast<uint64_t>(tile) * kXfLanes;  // wave-uniform: one scalar division
    const uint64_t b0 = g0 / p.chunks_per_shard;
    const uint32_t cc = static_cast<uint32_t>(g0 - b0 * p.chunks_per_shard) + lane;
    const bool ok = g0 + lane < p.total_columns;
    const uint32_t d = ok ? cc / p.chunks_per_shard : 0;
    const uint64_t blk = ok ? b0 + d : 0;
    const uint64_t col = ok ? cc - d * p.chunks_per_shard : 0;
    in_mask = ok ? p.pmask[2 * blk] : 0;
    out_mask = ok ? p.pmask[2 * blk + 1] : 0;
    rows = p.rows + blk * W;  // polynomial-basis constants, one word per position
    off_r = blk * p.rec_block_stride + col * 64;
    off_o = blk * p.orig_block_stride + col * 64;
  } else {
    // tile -> (pattern, address tile)
    uint64_t vtile = tile, pat = 0;
    if (p.per_block) {
      const uint64_t bi = tile / p.tiles_per_block;
      const uint64_t blk = p.block_ids ? p.block_ids[bi] : bi;
      vtile = blk * p.tiles_per_block + (tile - bi * p.tiles_per_block);
      pat = blk;
    }
    in_mask = p.pmask[2 * pat];
    out_mask = p.pmask[2 * pat + 1];
    rows = p.rows + pat * (W * 16);
    io_r = tile_io_g(p.total_columns, p.chunks_per_shard, vtile, lane, p.rec_block_stride);
    io_o = tile_io_g(p.total_columns, p.chunks_per_shard, vtile, lane, p.orig_block_stride);
  }

  Regs8 ra;
  static_for<8>([&](auto T) {
    constexpr int t = decltype(T)::value;
    const uint32_t j = 8 * wave + t;  // wave-uniform
    if ((in_mask >> j) & 1) {          // PL: per lane
      const uint32_t opos = p.low_rate ? 0 : p.chunk, rpos = p.low_rate ? p.chunk : 0;
      const bool is_rec = p.low_rate ? j >= p.chunk : j < p.chunk;
      const uint8_t* base = is_rec ? p.rec + (j - rpos) * p.rec_shard_stride : p.orig + (j - opos) * p.orig_shard_stride;
      static_for<4>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        const uint8_t* src;
        if constexpr (PL) src = base + (is_rec ? off_r : off_o) + 16 * q;
        else src = base + (is_rec ? io_r.off[q] : io_o.off[q]);
        const uint4 x = ld_piece(src);
        ra[t][4 * q] = x.x;
        ra[t][4 * q + 1] = x.y;
        ra[t][4 * q + 2] = x.z;
        ra[t][4 * q + 3] = x.w;
      });
    } else {
      static_for<16>([&](auto P) { ra[t][decltype(P)::value] = 0; });
    }
  });
  static_for<8>([&](auto T) {
    constexpr int t = decltype(T)::value;
    const uint32_t j = 8 * wave + t;
    if ((in_mask >> j) & 1) {
      if constexpr (!PL) swap_halves(ra[t]);
      dev::planes_from_raw(ra[t]);
      if constexpr (PL) dev::mul_rt_poly(ra[t], rows[j]); else mul_rt4(ra[t], rows + j * 16);
    }
  });
  xf_pass_a<NW, 0>(wave, ra);
  Regs8 rb;
  xf_exchange_ab<NW>(wave, lane, lds, ra, rb);
  xf_pass_b_ifft<NW, 0>(rb);
  xf_derivative<NW>(wave, lane, lds, rb);
  xf_pass_b_fft<NW, 0>(rb);
  xf_exchange_bc<NW>(wave, lane, lds, rb, ra);
  const uint32_t mine = static_cast<uint32_t>(out_mask >> (8 * wave)) & 0xFF;
  if constexpr (PL) {
    if (__builtin_amdgcn_ballot_w64(mine != 0) == 0) return;  // nothing to restore in this wave
  } else {
    if (mine == 0) return;
  }
  xf_pass_c<NW, 0>(wave, ra);
  static_for<8>([&](auto T) {
    constexpr int t = decltype(T)::value;
    const uint32_t j = 8 * wave + t;
    if ((out_mask >> j) & 1) {
      uint8_t* dst = p.orig + (j - (p.low_rate ? 0 : p.chunk)) * p.orig_shard_stride;
      if constexpr (PL) {
        dev::mul_rt_poly(ra[t], rows[j]);
        dev::store_chunk(dst + off_o, ra[t]);
      } else {
        mul_rt4(ra[t], rows + j * 16);
        store_shard(dst, io_o, io_o.valid, ra[t]);
      }
    }
  });
}

// =====================================================================================
// decode_x16<PASS, DIN, DOUT>: the window decoder (decode_x's algorithm) on the 16-wave
// layout: 16 waves x 4 slots, one 1024-thread workgroup per CU at 4 waves/SIMD (decode_x<8>
// keeps 8 slots per lane at 216 VGPRs: 2 waves/SIMD, latency-bound).
// Positions by layout (X8Lay: slot bits | wave bits):
//   G0 slots p0 p1 | waves p2 p3 p4 p5   loads + locator multiplies, IFFT b0 b1; FFT b0, stores
//   G1 slots p2 p1 | waves p0 p3 p4 p5   IFFT b2 / FFT b1
//   G2 slots p2 p3 | waves p0 p1 p4 p5   IFFT b3 / FFT b2
//   G3 slots p4 p3 | waves p0 p1 p2 p5   IFFT b4 / FFT b3
//   G4 slots p4 p5 | waves p0 p1 p2 p3   IFFT b5, formal derivative, FFT b5 b4
// The derivative w'[j] = w[j] ^ XOR_{b : bit b of j clear} w[j | 2^b] (pre-derivative terms)
// in G4: slot bits in-lane, wave bits from the partner waves' pre-derivative copies in LDS,
// two slots per round (2 x 128 KiB would not fit).
//
// PASS 0: the W <= 64 window (DIN = DOUT = 0).
// PASS 1 / 2: the W = 128 window as two 64-point passes.  With u_h = IFFT_64 of window half h
// (skew delta 64 h) and P = the derivative without its self term (D = I + P), the crate's
// IFFT_128 -> derivative -> FFT_128 gives output half o as FFT_64,64o(P u_o ^ u_{1-o}): the
// size-128 layer's skew factor (index 63) is zero, so the halves meet only there
// (tests/test_oracle.py pins the identity against the oracle's 128-point decoder).  Pass 1
// (DIN = the other half, DOUT = the output half): IFFT, no derivative, FFT, the partial
// stored unmultiplied.  Pass 2 (DIN = DOUT = the output half): IFFT, P, FFT, + the stored
// partial (in planes), output multiply (linear: one product per restored original).  Loads
// and masks are the pass's loaded half (window positions DIN + j); outputs are window
// positions DOUT + j.  One pattern per tile (tiles never straddle blocks): the constants are
// wave-uniform words, multiplied by the Horner scheme in the polynomial basis with the
// coefficient bits tested on the scalar unit (mul_rt_poly_u: a clear bit costs no VALU).
// Per-lane patterns run on decode_h8.
// =====================================================================================
template <int PASS, int DIN, int DOUT>
__global__ __launch_bounds__(1024, 4) void decode_x16_kernel(const DecodeXParams p) {
  using G0 = X8Lay<0, 1, 2, 3, 4, 5>;
  using G1 = X8Lay<2, 1, 0, 3, 4, 5>;
  using G2 = X8Lay<2, 3, 0, 1, 4, 5>;
  using G3 = X8Lay<4, 3, 0, 1, 2, 5>;
  using G4 = X8Lay<4, 5, 0, 1, 2, 3>;
  static_assert(PASS != 0 || (DIN == 0 && DOUT == 0), "the one-pass window starts at 0");
  static_assert(PASS != 2 || DIN == DOUT, "pass 2 loads its output half");
  __shared__ uint4 lds[32 * 4 * kXfLanes];  // 16 waves x 2 slots x 4 KiB
  __shared__ XFlags<16> flags;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t tile = dev::xcd_tile(blockIdx.x, gridDim.x);
  const uint32_t rw = p.rows_w;  // constants per pattern (64 or 128)
  if (threadIdx.x < 32) reinterpret_cast<uint32_t*>(&flags)[threadIdx.x] = 0;
  __syncthreads();
  uint64_t vtile = tile, pat = 0;
  if (p.per_block) {
    const uint64_t bi = tile / p.tiles_per_block;
    const uint64_t blk = p.block_ids ? p.block_ids[bi] : bi;
    vtile = blk * p.tiles_per_block + (tile - bi * p.tiles_per_block);
    pat = blk;
  }
  const uint64_t in_mask = p.pmask[2 * pat];
  const uint64_t out_mask = p.pmask[2 * pat + 1];
  const uint32_t* coef = p.rows + pat * rw + DIN;
  const uint32_t* coef_out = p.rows + pat * rw + DOUT;
  const TileIO io_r = tile_io_g(p.total_columns, p.chunks_per_shard, vtile, lane, p.rec_block_stride);
  const TileIO io_o = tile_io_g(p.total_columns, p.chunks_per_shard, vtile, lane, p.orig_block_stride);
  const uint32_t opos = p.low_rate ? 0 : p.chunk, rpos = p.low_rate ? p.chunk : 0;
  Regs4 r;
  static_for<4>([&](auto T) {
    constexpr int t = decltype(T)::value;
    const uint32_t j = 4 * wave + t;  // G0 position in the pass (wave-uniform)
    if ((in_mask >> j) & 1) {
      const uint32_t g = DIN + j;  // window position (recovery shards below the originals in HighRate)
      const bool is_rec = p.low_rate ? g >= p.chunk : g < p.chunk;
      const uint8_t* base = is_rec ? p.rec + (g - rpos) * p.rec_shard_stride : p.orig + (g - opos) * p.orig_shard_stride;
      static_for<4>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        const uint4 x = ld_piece(base + (is_rec ? io_r.off[q] : io_o.off[q]));
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
    constexpr int t = decltype(T)::value;
    const uint32_t j = 4 * wave + t;
    if ((in_mask >> j) & 1) {
      swap_halves(r[t]);
      dev::planes_from_raw(r[t]);
      dev::mul_rt_poly_u(r[t], coef[j]);  // wave-uniform constant: scalar-branch Horner
    }
  });
  // IFFT_64 (skew delta DIN)
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
  if constexpr (PASS != 1) {
    // formal derivative in G4 (slot t: position bits p4 = t & 1, p5 = t >> 1; wave bits p0..p3)
    __syncthreads();  // every wave's swap reads are done: the exchange buffer is free
    static_for<2>([&](auto Rho) {
      constexpr int rho = decltype(Rho)::value;
      // slot = 2 * wave + u holds this wave's pre-derivative slot 2 rho + u
      static_for<2>([&](auto U) { lds_put(lds, 2 * wave + decltype(U)::value, lane, r[2 * rho + decltype(U)::value]); });
      // slot-bit terms of slots 2 rho, 2 rho + 1 from pre-derivative partners (ascending t: a
      // partner t | 2^i > t is unmodified; slots 2, 3 are untouched until round 1)
      static_for<2>([&](auto U) {
        constexpr int t = 2 * rho + decltype(U)::value;
        if constexpr (PASS == 2) {
          // P = D ^ I: the partner terms only (the slot's own value stays in LDS for the
          // partner waves; lower slots never need a higher slot's register after this)
          static_for<16>([&](auto P) {
            constexpr int q = decltype(P)::value;
            if constexpr (!(t & 1) && !(t & 2)) r[t][q] = r[t | 1][q] ^ r[t | 2][q];
            else if constexpr (!(t & 1)) r[t][q] = r[t | 1][q];
            else if constexpr (!(t & 2)) r[t][q] = r[t | 2][q];
            else r[t][q] = 0;
          });
        } else {
          if constexpr (!(t & 1)) dev::xor_planes(r[t], r[t | 1]);
          if constexpr (!(t & 2)) dev::xor_planes(r[t], r[t | 2]);
        }
      });
      __syncthreads();
      static_for<4>([&](auto B) {
        constexpr int b = decltype(B)::value;
        if (!((wave >> b) & 1)) {
          const int pw = wave | (1 << b);
          static_for<2>([&](auto U) { lds_get_xor(lds, 2 * pw + decltype(U)::value, lane, r[2 * rho + decltype(U)::value]); });
        }
      });
      __syncthreads();
    });
  }
  // FFT_64 (skew delta DOUT), ending in G0
  x8_layer_t<G4, 5, false, DOUT>(wave, r);
  x8_layer_t<G4, 4, false, DOUT>(wave, r);
  x8_swap<1, 3, 5>(wave, lane, lds, &flags, r);
  x8_layer_t<G3, 3, false, DOUT>(wave, r);
  x8_swap<0, 2, 6>(wave, lane, lds, &flags, r);
  x8_layer_t<G2, 2, false, DOUT>(wave, r);
  x8_swap<1, 1, 7>(wave, lane, lds, &flags, r);
  x8_layer_t<G1, 1, false, DOUT>(wave, r);
  x8_swap<0, 0, 8>(wave, lane, lds, &flags, r);
  const uint32_t mine = static_cast<uint32_t>(out_mask >> (4 * wave)) & 0xF;  // wave-uniform
  if (mine == 0) return;
  x8_layer_t<G0, 0, false, DOUT>(wave, r);
  static_for<4>([&](auto T) {
    constexpr int t = decltype(T)::value;
    const uint32_t j = 4 * wave + t;
    if ((mine >> t) & 1) {
      uint8_t* dst = p.orig + (DOUT + j - opos) * p.orig_shard_stride;
      if constexpr (PASS == 2) {
        // + pass 1's partial, in planes (the youngest memory operation when waited on, as in
        // decode_h8)
        uint32_t o[16];
        static_for<4>([&](auto Q) {
          constexpr int q = decltype(Q)::value;
          const uint4 x = ld_piece(dst + io_o.off[q]);
          o[4 * q] = x.x;
          o[4 * q + 1] = x.y;
          o[4 * q + 2] = x.z;
          o[4 * q + 3] = x.w;
        });
        swap_halves(o);
        dev::planes_from_raw(o);
        dev::xor_planes(r[t], o);
      }
      // the output multiply is linear: pass 1 stores its unmultiplied partial, pass 2 has
      // added it in planes and multiplies once
      if constexpr (PASS != 1) dev::mul_rt_poly_u(r[t], coef_out[j]);
      store_shard(dst, io_o, io_o.valid, r[t]);
    }
  });
}

// =====================================================================================
// decode_h8<OUTH>: the W = 64 per-lane window decoder (decode_x16<true, 0>'s algorithm) on
// 32-column tiles with the lane half as a position bit: 8 waves x 4 slots x 2 lane halves,
// 64 KiB of swap buffer, so two workgroups share a CU and one's loads, swaps and barriers
// overlap the other's arithmetic (decode_x16 runs one 1024-thread workgroup per CU).
// Lane l holds column l & 31 of the tile; h = l >> 5 is a position bit.  Layouts (slot bits
// | lane half | wave bits):
//   A  slots p0 p1 | h p2 | waves p3 p4 p5   loads, locator multiplies, IFFT b0; FFT b0, stores
//   B  slots p2 p1 | h p0 | waves p3 p4 p5   IFFT b1 b2 / FFT b1      (A <-> B: v_permlane32_swap)
//   C  slots p2 p3 | h p0 | waves p1 p4 p5   IFFT b3 / FFT b2
//   D  slots p4 p3 | h p0 | waves p1 p2 p5   IFFT b4 / FFT b3
//   E  slots p4 p5 | h p0 | waves p1 p2 p3   IFFT b5, formal derivative, FFT b5 b4
// A layer-b skew constant depends on the position bits above b.  From B on the lane half is
// p0, below every layer's bit; layer 0 in A has a constant per lane half (both halves' XOR
// programs run under the exec mask).  The derivative's p0 term crosses lane halves
// (v_permlane32_swap of the pre-derivative slot).  OUTH = the window half (p5) holding the
// restored originals (1 HighRate chunk 32, 0 the LowRate sub-window, -1 both): after FFT b4
// the waves whose p5 is the other half send their live slots and retire.
// PASS 1 / 2: the W = 128 window as decode_x16's two 64-point passes (loaded half DIN, output
// half DOUT), with the output multiply deferred: pass 1 stores FFT(u_other) unmultiplied,
// pass 2 adds it to FFT(P u_out) in planes and multiplies once (the multiply is linear), so a
// restored original costs one runtime product instead of two.
// Each lane loads its own whole chunk (four 16-byte pieces of one chunk).  A lane-linear
// option (xform_h8's piece order + quad_exchange) measured slower on the follower's batches
// (14.0-14.1 vs 14.4-14.6 M slices/s, profiles/r03_h8_ll_ab.jsonl) and was removed.
// The derivative's regions are handed over by the swaps' epoch flags (no workgroup barriers):
// ready = published, done = this wave's reads finished; a region is rewritten once every
// reader of its last epoch is done.  Epochs: swaps 1-3, derivative rounds 4-5, swaps 6-8.
// TAIL: shards of S = 64 C + T bytes (16 <= T < 64; p.chunks_per_shard = C + 1): the lanes of
// column C move their block's T-byte tail chunk whole (load_tail_chunk / store_tail_chunk:
// 16-byte accesses inside the tail only), so the follower's slices of any even shred size with
// T >= 16 decode in place, with no restride.
template <int OUTH, int PASS, int DIN, int DOUT, bool TAIL = false>
__global__ __launch_bounds__(512, 4) void decode_h8_kernel(const DecodeXParams p) {
  static_assert(PASS != 0 || (DIN == 0 && DOUT == 0), "the one-pass window starts at 0");
  static_assert(PASS != 2 || DIN == DOUT, "pass 2 loads its output half");
  static_assert(!TAIL || PASS == 0, "tail chunks on the one-pass window");
  using LB = X8Lay<2, 1, 3, 4, 5>;
  using LC = X8Lay<2, 3, 1, 4, 5>;
  using LD = X8Lay<4, 3, 1, 2, 5>;
  using LE = X8Lay<4, 5, 1, 2, 3>;
  constexpr int W = 64, kCols = 32;
  __shared__ uint4 lds[16 * 4 * kXfLanes];  // 8 waves x 2 slots x 4 KiB
  __shared__ X8Flags flags;
  __shared__ uint32_t lcoef[kCols * W];     // the constants of the <= 32 blocks of the tile
  const int lane = threadIdx.x & 63;
  const int h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t tile = dev::xcd_tile(blockIdx.x, gridDim.x);
  const uint64_t c0 = static_cast<uint64_t>(tile) * kCols;
  const uint64_t c1 = c0 + kCols - 1 < p.total_columns ? c0 + kCols - 1 : p.total_columns - 1;
  const uint64_t sb0 = c0 / p.chunks_per_shard;
  {
    const uint32_t nbt = static_cast<uint32_t>(c1 / p.chunks_per_shard - sb0 + 1);  // <= 32
    for (uint32_t i = threadIdx.x; i < nbt * W; i += blockDim.x) lcoef[i] = p.rows[(sb0 + i / W) * p.rows_w + DIN + i % W];
  }
  if (threadIdx.x < 16) reinterpret_cast<uint32_t*>(&flags)[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t gc = c0 + (lane & 31);
  const bool ok = gc < p.total_columns;
  const uint32_t cc = static_cast<uint32_t>(c0 - sb0 * p.chunks_per_shard) + (lane & 31);  // 32-bit per lane
  const uint32_t d = ok ? cc / p.chunks_per_shard : 0;
  const uint64_t blk = sb0 + d;
  const uint64_t col = ok ? cc - d * p.chunks_per_shard : 0;
  const bool tail_lane = TAIL && ok && col + 1 == p.chunks_per_shard;
  const uint64_t in_mask = ok ? p.pmask[2 * blk] : 0;
  const uint64_t out_mask = ok ? p.pmask[2 * blk + 1] : 0;
  const uint32_t* coef = lcoef + (blk - sb0) * W;
  const uint64_t off_r = blk * p.rec_block_stride + col * 64;
  const uint64_t off_o = blk * p.orig_block_stride + col * 64;
  const uint32_t opos = p.low_rate ? 0 : p.chunk, rpos = p.low_rate ? p.chunk : 0;
  // layout A position of slot t in this lane
  auto posA = [&](int t) -> uint32_t {
    return static_cast<uint32_t>((t & 1) | ((t >> 1) << 1) | (h << 2) | (wave << 3));
  };
  Regs4 r;
  static_for<4>([&](auto T) {
    constexpr int t = decltype(T)::value;
    const uint32_t j = posA(t);
    const uint32_t g = DIN + j;  // window position
    const bool is_rec = p.low_rate ? g >= p.chunk : g < p.chunk;
    if ((in_mask >> j) & 1) {
      const uint8_t* src = is_rec ? p.rec + (g - rpos) * p.rec_shard_stride + off_r
                                  : p.orig + (g - opos) * p.orig_shard_stride + off_o;
      if (tail_lane) {
        load_tail_chunk(src, p.tail_bytes, r[t]);
      } else {
        static_for<4>([&](auto Q) {
          constexpr int q = decltype(Q)::value;
          const uint4 x = ld_piece(src + 16 * q);
          r[t][4 * q] = x.x;
          r[t][4 * q + 1] = x.y;
          r[t][4 * q + 2] = x.z;
          r[t][4 * q + 3] = x.w;
        });
      }
    } else {
      static_for<16>([&](auto P) { r[t][decltype(P)::value] = 0; });
    }
  });
  static_for<4>([&](auto T) {
    constexpr int t = decltype(T)::value;
    const uint32_t j = posA(t);
    if ((in_mask >> j) & 1) {
      dev::planes_from_raw(r[t]);
      dev::mul_rt_poly(r[t], coef[j]);
    }
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
  // formal derivative in E (slot t: p4 = t & 1, p5 = t >> 1; lane half p0; waves p1 p2 p3);
  // PASS 2: P = the derivative without its self term; PASS 1: none.  Each wave publishes its
  // two pre-derivative slots of round rho in its own region (its swap inbox); the waves with
  // a wave bit b clear add the region of their partner w | 2^b.
  constexpr int D = PASS != 1 ? 2 : 0;  // FFT swap epochs 4 + D ..
  // the readers of region x in a derivative round: x with one of its set wave bits cleared
  auto wait_readers = [&](int x, uint32_t e) __attribute__((always_inline)) {
    static_for<3>([&](auto Bb) {
      constexpr int b = decltype(Bb)::value;
      if ((x >> b) & 1) x8_wait_ge(&flags.done[x & ~(1 << b)], e);
    });
  };
  if constexpr (PASS != 1) {
    static_for<2>([&](auto Rho) {
      constexpr int rho = decltype(Rho)::value;
      constexpr uint32_t e = 4 + rho;
      if constexpr (rho == 1) wait_readers(wave, e - 1);  // round 0's readers of this region
      static_for<2>([&](auto U) { lds_put(lds, 2 * wave + decltype(U)::value, lane, r[2 * rho + decltype(U)::value]); });
      x8_signal(&flags.ready[wave], e, lane);
      static_for<2>([&](auto U) {
        constexpr int t = 2 * rho + decltype(U)::value;
        // p0 term: the lower half (p0 clear) adds the upper half's pre-derivative value
        uint32_t hi[16];
        static_for<16>([&](auto P) {
          constexpr int q = decltype(P)::value;
          hi[q] = __builtin_amdgcn_permlane32_swap(r[t][q], 0u, false, false)[1];
        });
        // slot bits, ascending t: partners t | 1, t | 2 > t still hold pre-derivative values
        if constexpr (PASS == 2) {
          static_for<16>([&](auto P) {
            constexpr int q = decltype(P)::value;
            uint32_t v = hi[q];
            if constexpr (!(t & 1)) v ^= r[t | 1][q];
            if constexpr (!(t & 2)) v ^= r[t | 2][q];
            r[t][q] = v;
          });
        } else {
          if constexpr (!(t & 1)) dev::xor_planes(r[t], r[t | 1]);
          if constexpr (!(t & 2)) dev::xor_planes(r[t], r[t | 2]);
          dev::xor_planes(r[t], hi);
        }
      });
      static_for<3>([&](auto Bb) {
        constexpr int b = decltype(Bb)::value;
        if (!((wave >> b) & 1)) {
          const int pw = wave | (1 << b);
          x8_wait_ge(&flags.ready[pw], e);
          static_for<2>([&](auto U) { lds_get_xor(lds, 2 * pw + decltype(U)::value, lane, r[2 * rho + decltype(U)::value]); });
        }
      });
      x8_signal(&flags.done[wave], e, lane);
    });
  }
  // FFT_64 (skew delta DOUT), ending in A.  The first swap writes the partner's region: its
  // last derivative round's readers must be done with it.
  x8_layer_t<LE, 5, false, DOUT>(wave, r);
  x8_layer_t<LE, 4, false, DOUT>(wave, r);
  if constexpr (D != 0) wait_readers(wave ^ 4, 5);
  if constexpr (OUTH < 0) {
    x8_swap<1, 2, 4 + D>(wave, lane, lds, &flags, r);
  } else {
    // E -> D: slot bit 1 (p5) <-> wave bit 2 (p3).  After it a wave's slots all have p5 =
    // its wave bit 2; the other half's waves only send the slots the live partner needs.
    const int partner = wave ^ 4;
    if (((wave >> 2) & 1) != OUTH) {
      x8_wait_ge(&flags.done[partner], 3 + D);
      static_for<4>([&](auto T) {
        constexpr int t = decltype(T)::value;
        if constexpr (((t >> 1) & 1) == (OUTH > 0 ? 1 : 0)) {
          lds_put(lds, 2 * partner + (t & 1), lane, r[t]);
          __asm__ volatile("; h8 put %0" ::"n"(t));
        }
      });
      x8_signal(&flags.ready[wave], 4 + D, lane);
      return;
    }
    x8_wait_ge(&flags.ready[partner], 4 + D);
    static_for<4>([&](auto T) {
      constexpr int t = decltype(T)::value;
      if constexpr (((t >> 1) & 1) != (OUTH > 0 ? 1 : 0)) {
        lds_get(lds, 2 * wave + (t & 1), lane, r[t]);
        __asm__ volatile("; h8 get %0" ::"n"(t));
      }
    });
    x8_signal(&flags.done[wave], 4 + D, lane);
  }
  x8_layer_t<LD, 3, false, DOUT>(wave, r);
  x8_swap<0, 1, 5 + D>(wave, lane, lds, &flags, r);
  x8_layer_t<LC, 2, false, DOUT>(wave, r);
  x8_swap<1, 0, 6 + D>(wave, lane, lds, &flags, r);
  x8_layer_t<LB, 1, false, DOUT>(wave, r);
  // the store predicates, packed before the first load or store of the store phase (bit t:
  // slot t restores its position in this lane's block)
  uint32_t qall = 0;
  static_for<4>([&](auto T) { qall |= static_cast<uint32_t>((out_mask >> posA(decltype(T)::value)) & 1) << decltype(T)::value; });
  if (__builtin_amdgcn_ballot_w64(qall != 0) == 0) return;  // nothing to restore in this wave
  h8_relayout(r);
  h8_layer0<false, DOUT>(wave, h, r);
  static_for<4>([&](auto T) {
    constexpr int t = decltype(T)::value;
    const uint32_t j = posA(t);
    if ((qall >> t) & 1) {
      uint8_t* dst = p.orig + (DOUT + j - opos) * p.orig_shard_stride + off_o;
      if constexpr (PASS == 0 && OUTH < 0) {
        // fused coding restore (p.fuse, HighRate): an absent recovery position's value is the
        // re-encoded coding shard; it goes back to its own slot (the ANY_K patterns of other
        // callers never restore recovery positions)
        if (DOUT + j < p.chunk) dst = const_cast<uint8_t*>(p.rec) + (DOUT + j) * p.rec_shard_stride + off_r;
      }
      if constexpr (PASS == 2) {
        // + pass 1's partial, in planes.  The load is the youngest memory operation when it is
        // waited on (vmcnt(0)): the earlier slots' stores may alias it, so it is not hoisted
        // above them (tools/scan_waitcnt.py)
        uint32_t o[16];
        static_for<4>([&](auto Q) {
          constexpr int q = decltype(Q)::value;
          const uint4 x = ld_piece(dst + 16 * q);
          o[4 * q] = x.x;
          o[4 * q + 1] = x.y;
          o[4 * q + 2] = x.z;
          o[4 * q + 3] = x.w;
        });
        dev::planes_from_raw(o);
        dev::xor_planes(r[t], o);
      }
      if constexpr (PASS != 1) dev::mul_rt_poly(r[t], coef[j]);
      if (tail_lane) {
        uint32_t raw[16];
        static_for<16>([&](auto P) { raw[decltype(P)::value] = r[t][decltype(P)::value]; });
        dev::transpose8(raw);
        dev::transpose8(raw + 8);
        store_tail_chunk(dst, p.tail_bytes, raw);
      } else {
        dev::store_chunk<true>(dst, r[t]);  // PASS 1: the unmultiplied partial
      }
    }
  });
}

__device__ __forceinline__ uint32_t m65535_add(uint32_t a, uint32_t b) {
  const uint32_t s = a + b;
  return s >= 65535u ? s - 65535u : s;
}
__device__ __forceinline__ uint32_t m65535_sub(uint32_t a, uint32_t b) { return a >= b ? a - b : a + 65535u - b; }
__device__ __forceinline__ uint32_t m65535_mul(uint32_t a, uint32_t b) {  // canonical a, b < 65535
  const uint32_t p = a * b;
  uint32_t s = (p & 0xFFFFu) + (p >> 16);  // 2^16 = 1 (mod 65535)
  s = (s & 0xFFFFu) + (s >> 16);
  return s >= 65535u ? s - 65535u : s;
}
// the unnormalised Walsh transform over the 64 lanes (one residue per lane)
__device__ __forceinline__ uint32_t walsh64(uint32_t v, int lane) {
  static_for<6>([&](auto B) {
    constexpr int d = 1 << decltype(B)::value;
    const uint32_t o = static_cast<uint32_t>(__shfl_xor(static_cast<int>(v), d));
    v = (lane & d) ? m65535_sub(o, v) : m65535_add(v, o);
  });
  return v;
}
// 128 points: position lane in v0, lane + 64 in v1
__device__ __forceinline__ void walsh128(uint32_t& v0, uint32_t& v1, int lane) {
  v0 = walsh64(v0, lane);
  v1 = walsh64(v1, lane);
  const uint32_t a = v0;
  v0 = m65535_add(a, v1);
  v1 = m65535_sub(a, v1);
}
__device__ __forceinline__ uint16_t locator_log(uint32_t loc, bool in) {  // exp of +loc (present), -loc (restored)
  return static_cast<uint16_t>(in ? loc : 65535u - loc);
}

// =====================================================================================
// decode_pk<OUTH>: decode_h8's W = 64 window for per-slice patterns on 1 KiB shreds (16 chunks
// per shard: a 32-column tile is two slices) with the locator products packed.  In decode_h8 a
// wave-slot holds four 16-lane groups -- two slices x two positions (lane half) -- and runs the
// per-lane Horner product when ANY group's position is present: with random 32-of-64 arrival
// that is ~94 % of the slots where 50 % carry data, and likewise for the restored outputs.
// Here the products run on packed items instead (item = one slice's 16 columns of one position,
// 1 KiB):
//   1. the workgroup ranks each slice's survivors and restored positions (LDS lists);
//   2. item i of the survivors (i < 64: ANY_K keeps at most 32 per slice) is loaded by row
//      group i & 3 of slot (i >> 2) & 1 of wave i >> 3, bitsliced, multiplied by its locator
//      constant and written to the 64 KiB exchange buffer;
//   3. every lane reads its layout-A slots from there (absent positions are zero) and the
//      transform runs as decode_h8's (swaps, derivative, the half-pruned FFT);
//   4. the live waves write their restored positions' values as packed items, and each item is
//      multiplied, converted to bytes and stored by one row group.
// Survivor and restored counts bound the product work instead of the slot count: per 2-slice
// tile 64 input items on 16 wave-slots (decode_h8: ~30 of 32) and the restored items on the
// live waves' 16 wave-slots.  OUTH: the window half of the restored originals (1 HighRate chunk
// 32, 0 the LowRate sub-window); only those geometries launch it.  Requires any_k (at most k
// survivors per pattern) and 16 chunks per shard.
// =====================================================================================
// The transform's multiplies use the subset-greedy programs (TAB 1, rs_device.hpp mul_acc): with
// the cancellation programs this kernel's allocation spills (14 VGPRs).
// The tile body (decode_pk_kernel, and the per-call server's random-arrival job with one slice):
// `lds` is the 64 KiB exchange buffer (packed items [item][q][16 lanes] or swap regions), `sh`
// the tile's lists.  p.pmask / p.rows may address LDS (the server stages them there).
struct PkShared {
  uint32_t lcoef[2 * 64];         // the two slices' locator constants (polynomial basis)
  uint64_t smask[2][2];           // per slice: positions present (loaded), restored
  uint8_t ilist[2][64], olist[2][64];  // per slice: survivor / restored positions by rank
};
// The per-call server's locator tables (built once per server launch): log x for the window's
// 64 positions, and a^i, a^(256 i) (i < 256) in the polynomial basis, where a constant of the
// decoder is to_poly(exp[l]) = a^l (the basis map sends exp[l] to the l-th power of the
// polynomial generator, a^16 = a^5 + a^3 + a^2 + 1; checked for every l by
// tests/test_oracle.py::test_poly_basis_powers) -- so the server needs no table lookups in HBM.
struct PkLocTables {
  uint16_t log64[64];
  uint16_t apow_lo[256], apow_hi[256];
};
__device__ __forceinline__ uint32_t poly_mul(uint32_t a, uint32_t b) {  // GF(2)[a] / (a^16 + a^5 + a^3 + a^2 + 1)
  uint32_t r = 0;
  for (int i = 0; i < 16; ++i) r ^= ((b >> i) & 1) ? a << i : 0u;
  for (int i = 30; i >= 16; --i) r ^= ((r >> i) & 1) ? (1u << i) ^ (0x2Du << (i - 16)) : 0u;
  return r;
}
__device__ __forceinline__ uint32_t poly_pow_a(const PkLocTables& t, uint32_t l) {  // a^l, l <= 65535
  return poly_mul(t.apow_hi[l >> 8], t.apow_lo[l & 255]);
}

// SRV: the per-call server's one-slice job; the locator constants of slice 0 are computed in
// the list phase by wave 0 (decode_rows' Walsh route over `loc`) instead of read from p.rows.
// TAIL: shreds of S = 960 + T bytes (16 <= T < 64): column 15 of an item is the shred's T-byte
// tail, moved whole by its lanes (load_tail_chunk / store_tail_chunk, as decode_h8's TAIL).
template <int OUTH, bool SRV = false, bool TAIL = false>
__device__ __forceinline__ void decode_pk_tile(const DecodeXParams& p, uint32_t tile, uint4* lds, X8Flags* fl,
                                               PkShared& sh, const PkLocTables* loc = nullptr) {
  static_assert(OUTH >= -1 && OUTH <= 1, "OUTH: the restored positions' window half, -1 both");
  using LB = X8Lay<2, 1, 3, 4, 5>;
  using LC = X8Lay<2, 3, 1, 4, 5>;
  using LD = X8Lay<4, 3, 1, 2, 5>;
  using LE = X8Lay<4, 5, 1, 2, 3>;
  constexpr int W = 64, kSl = 16;           // positions, columns per slice
  constexpr int D = 2;                      // derivative epochs 4, 5; FFT swaps 4 + D ..
  X8Flags& flags = *fl;
  uint32_t* lcoef = sh.lcoef;
  auto& smask = sh.smask;
  auto& ilist = sh.ilist;
  auto& olist = sh.olist;
  const int lane = threadIdx.x & 63;
  const int h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t sb0 = static_cast<uint64_t>(tile) * 2;  // the tile's first slice (block)
  const uint64_t nblk = p.total_columns / kSl;
  const uint32_t opos = p.low_rate ? 0 : p.chunk, rpos = p.low_rate ? p.chunk : 0;
  if (threadIdx.x < 2 * W) {
    const uint32_t sl = threadIdx.x >> 6, j = threadIdx.x & 63;
    uint64_t im = 0, om = 0;
    if (sb0 + sl < nblk) {
      im = p.pmask[2 * (sb0 + sl)];
      om = p.pmask[2 * (sb0 + sl) + 1];
      if constexpr (SRV) {
        // wave 0 (slice 0): loc(x) = sum over erased e != x of log(x ^ e), as H(H(L) H(I)) / 64
        const uint64_t e = ~im;
        const uint32_t hl = m65535_mul(walsh64(j ? loc->log64[j] : 0u, static_cast<int>(j)), 1024u);
        const uint32_t hi = walsh64(static_cast<uint32_t>((e >> j) & 1), static_cast<int>(j));
        const uint32_t acc = walsh64(m65535_mul(hl, hi), static_cast<int>(j));
        lcoef[threadIdx.x] = poly_pow_a(*loc, locator_log(acc, (im >> j) & 1));
      } else if (((im | om) >> j) & 1) {
        lcoef[threadIdx.x] = p.rows[(sb0 + sl) * p.rows_w + j];
      }
    }
    const uint64_t below = (uint64_t{1} << j) - 1;
    if ((im >> j) & 1) ilist[sl][__builtin_popcountll(im & below)] = static_cast<uint8_t>(j);
    if ((om >> j) & 1) olist[sl][__builtin_popcountll(om & below)] = static_cast<uint8_t>(j);
    if (j == 0) {
      smask[sl][0] = im;
      smask[sl][1] = om;
    }
  }
  if (threadIdx.x < 16) reinterpret_cast<uint32_t*>(&flags)[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t imA = smask[0][0], imB = smask[1][0], omA = smask[0][1], omB = smask[1][1];
  const uint32_t nA = static_cast<uint32_t>(__builtin_popcountll(imA));
  const uint32_t nin = nA + static_cast<uint32_t>(__builtin_popcountll(imB));
  const uint32_t noA = static_cast<uint32_t>(__builtin_popcountll(omA));
  const uint32_t nout = noA + static_cast<uint32_t>(__builtin_popcountll(omB));
  if (nout == 0) return;  // nothing restored in either slice (workgroup-uniform)
  const int col = lane & 15, row = lane >> 4;
  const bool tail_lane = TAIL && col == kSl - 1;
  // the byte offset of position g's shard of slice sl, column col (recovery shards below the
  // originals in HighRate)
  auto src_of = [&](uint32_t sl, uint32_t g) -> const uint8_t* {
    const bool is_rec = p.low_rate ? g >= p.chunk : g < p.chunk;
    const uint64_t blk = sb0 + sl;
    return is_rec ? p.rec + (g - rpos) * p.rec_shard_stride + blk * p.rec_block_stride + col * 64
                  : p.orig + (g - opos) * p.orig_shard_stride + blk * p.orig_block_stride + col * 64;
  };
  // 2. packed input products: item i on row group i & 3 of wave (i >> 2) & 7, slot i >> 5 (a
  // one-slice tile's 32 items fill all eight waves' first slot).  Both items' loads are issued
  // before either product (one HBM round trip per wave, not two)
  uint32_t v[2][16];
  static_for<2>([&](auto U) {
    constexpr int u = decltype(U)::value;
    const uint32_t i = u * 32 + wave * 4 + row;
    if (i < nin) {
      const uint32_t sl = i < nA ? 0u : 1u;
      const uint8_t* src = src_of(sl, ilist[sl][i - (sl ? nA : 0u)]);
      if (tail_lane) {
        load_tail_chunk(src, p.tail_bytes, v[u]);
      } else {
        static_for<4>([&](auto Q) {
          constexpr int q = decltype(Q)::value;
          const uint4 x = ld_piece(src + 16 * q);
          v[u][4 * q] = x.x;
          v[u][4 * q + 1] = x.y;
          v[u][4 * q + 2] = x.z;
          v[u][4 * q + 3] = x.w;
        });
      }
    } else {
      static_for<16>([&](auto P) { v[u][decltype(P)::value] = 0; });
    }
  });
  static_for<2>([&](auto U) {
    constexpr int u = decltype(U)::value;
    if (static_cast<uint32_t>(u * 32 + wave * 4) < nin) {  // wave-uniform
      const uint32_t i = u * 32 + wave * 4 + row;
      const bool ok = i < nin;
      const uint32_t sl = i < nA ? 0u : 1u;
      const uint32_t j = ok ? ilist[sl][i - (sl ? nA : 0u)] : 0u;
      dev::planes_from_raw(v[u]);
      dev::mul_rt_poly(v[u], lcoef[sl * W + j]);
      if (ok) {
        static_for<4>([&](auto Q) {
          constexpr int q = decltype(Q)::value;
          lds[(i * 4 + q) * kSl + col] = make_uint4(v[u][4 * q], v[u][4 * q + 1], v[u][4 * q + 2], v[u][4 * q + 3]);
        });
      }
    }
  });
  __syncthreads();
  // 3. layout A from the packed items: lane column c = lane & 31 (slice c >> 4), slot t holds
  // position t | h << 2 | wave << 3
  const uint32_t lsl = static_cast<uint32_t>((lane & 31) >> 4);
  const uint64_t in_mask = lsl ? imB : imA, out_mask = lsl ? omB : omA;
  auto posA = [&](int t) -> uint32_t {
    return static_cast<uint32_t>((t & 1) | ((t >> 1) << 1) | (h << 2) | (wave << 3));
  };
  Regs4 r;
  static_for<4>([&](auto T) {
    constexpr int t = decltype(T)::value;
    const uint32_t j = posA(t);
    if ((in_mask >> j) & 1) {
      const uint32_t i = static_cast<uint32_t>(__builtin_popcountll(in_mask & ((uint64_t{1} << j) - 1))) + (lsl ? nA : 0u);
      static_for<4>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        const uint4 x = lds[(i * 4 + q) * kSl + col];
        r[t][4 * q] = x.x;
        r[t][4 * q + 1] = x.y;
        r[t][4 * q + 2] = x.z;
        r[t][4 * q + 3] = x.w;
      });
    } else {
      static_for<16>([&](auto P) { r[t][decltype(P)::value] = 0; });
    }
  });
  __syncthreads();  // every item read: the buffer becomes the swap regions
  // IFFT_64
  h8_layer0<true, 0, 1>(wave, h, r);
  h8_relayout(r);
  x8_layer_t<LB, 1, true, 0, 1>(wave, r);
  x8_layer_t<LB, 2, true, 0, 1>(wave, r);
  x8_swap<1, 0, 1, 0xF, false>(wave, lane, lds, &flags, r);
  x8_layer_t<LC, 3, true, 0, 1>(wave, r);
  x8_swap<0, 1, 2, 0xF, false>(wave, lane, lds, &flags, r);
  x8_layer_t<LD, 4, true, 0, 1>(wave, r);
  x8_swap<1, 2, 3, 0xF, false>(wave, lane, lds, &flags, r);
  x8_layer_t<LE, 5, true, 0, 1>(wave, r);
  // formal derivative in E (decode_h8's, epochs 4 and 5)
  auto wait_readers = [&](int x, uint32_t e) __attribute__((always_inline)) {
    static_for<3>([&](auto Bb) {
      constexpr int b = decltype(Bb)::value;
      if ((x >> b) & 1) x8_wait_ge(&flags.done[x & ~(1 << b)], e);
    });
  };
  static_for<2>([&](auto Rho) {
    constexpr int rho = decltype(Rho)::value;
    constexpr uint32_t e = 4 + rho;
    if constexpr (rho == 1) wait_readers(wave, e - 1);
    static_for<2>([&](auto U) { lds_put(lds, 2 * wave + decltype(U)::value, lane, r[2 * rho + decltype(U)::value]); });
    x8_signal(&flags.ready[wave], e, lane);
    static_for<2>([&](auto U) {
      constexpr int t = 2 * rho + decltype(U)::value;
      uint32_t hi[16];
      static_for<16>([&](auto P) {
        constexpr int q = decltype(P)::value;
        hi[q] = __builtin_amdgcn_permlane32_swap(r[t][q], 0u, false, false)[1];
      });
      if constexpr (!(t & 1)) dev::xor_planes(r[t], r[t | 1]);
      if constexpr (!(t & 2)) dev::xor_planes(r[t], r[t | 2]);
      dev::xor_planes(r[t], hi);
    });
    static_for<3>([&](auto Bb) {
      constexpr int b = decltype(Bb)::value;
      if (!((wave >> b) & 1)) {
        const int pw = wave | (1 << b);
        x8_wait_ge(&flags.ready[pw], e);
        static_for<2>([&](auto U) { lds_get_xor(lds, 2 * pw + decltype(U)::value, lane, r[2 * rho + decltype(U)::value]); });
      }
    });
    x8_signal(&flags.done[wave], e, lane);
  });
  // FFT_64 down to A; the waves of the other window half hand over their live slots and retire
  x8_layer_t<LE, 5, false, 0, 1>(wave, r);
  x8_layer_t<LE, 4, false, 0, 1>(wave, r);
  wait_readers(wave ^ 4, 5);
  if constexpr (OUTH < 0) {
    // restored positions in both halves (fused coding restore): every wave finishes the FFT
    x8_swap<1, 2, 4 + D, 0xF, false>(wave, lane, lds, &flags, r);
  } else {
    const int partner = wave ^ 4;
    if (((wave >> 2) & 1) != OUTH) {
      x8_wait_ge(&flags.done[partner], 3 + D);
      static_for<4>([&](auto T) {
        constexpr int t = decltype(T)::value;
        if constexpr (((t >> 1) & 1) == OUTH) {
          lds_put(lds, 2 * partner + (t & 1), lane, r[t]);
          __asm__ volatile("; pk put %0" ::"n"(t));
        }
      });
      x8_signal(&flags.ready[wave], 4 + D, lane);
      return;
    }
    x8_wait_ge(&flags.ready[partner], 4 + D);
    static_for<4>([&](auto T) {
      constexpr int t = decltype(T)::value;
      if constexpr (((t >> 1) & 1) != OUTH) {
        lds_get(lds, 2 * wave + (t & 1), lane, r[t]);
        __asm__ volatile("; pk get %0" ::"n"(t));
      }
    });
    x8_signal(&flags.done[wave], 4 + D, lane);
  }
  x8_layer_t<LD, 3, false, 0, 1>(wave, r);
  x8_swap<0, 1, 5 + D, 0xF, false>(wave, lane, lds, &flags, r);
  x8_layer_t<LC, 2, false, 0, 1>(wave, r);
  x8_swap<1, 0, 6 + D, 0xF, false>(wave, lane, lds, &flags, r);
  x8_layer_t<LB, 1, false, 0, 1>(wave, r);
  h8_relayout(r);
  h8_layer0<false, 0, 1>(wave, h, r);
  // 4. packed output products.  Every live wave's last swap read is done before any item
  // overwrites a region; items written, then every live wave's items visible before reads.
  constexpr int kLive = OUTH < 0 ? 8 : 4;     // live waves: all, or wave bit 2 == OUTH
  constexpr int kHi = OUTH < 0 ? 0 : OUTH << 2;
  const int lw = wave & (kLive - 1);
  static_for<kLive>([&](auto Wv) {
    constexpr int w2 = decltype(Wv)::value;
    x8_wait_ge(&flags.done[w2 | kHi], 6 + D);
  });
  static_for<4>([&](auto T) {
    constexpr int t = decltype(T)::value;
    // recomputed here: otherwise layout A's rank masks stay live across the transform and
    // the fused variant (kLive 8) spills them
    uint32_t j = posA(t);
    __asm__ volatile("" : "+v"(j));
    if ((out_mask >> j) & 1) {
      const uint32_t o = static_cast<uint32_t>(__builtin_popcountll(out_mask & ((uint64_t{1} << j) - 1))) + (lsl ? noA : 0u);
      static_for<4>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        lds[(o * 4 + q) * kSl + col] = make_uint4(r[t][4 * q], r[t][4 * q + 1], r[t][4 * q + 2], r[t][4 * q + 3]);
      });
    }
  });
  x8_signal(&flags.ready[wave], 7 + D, lane);
  static_for<kLive>([&](auto Wv) {
    constexpr int w2 = decltype(Wv)::value;
    x8_wait_ge(&flags.ready[w2 | kHi], 7 + D);
  });
  // item o on row group o & 3 of live wave (o >> 2) % kLive, slot o / (4 kLive) (the first
  // 4 kLive items spread over every live wave)
  constexpr int kPer = 64 / kLive;  // items per live wave
  static_for<kPer / 4>([&](auto U) {
    constexpr int u = decltype(U)::value;
    if (static_cast<uint32_t>(u * 4 * kLive + lw * 4) < nout) {  // wave-uniform
      const uint32_t o = u * 4 * kLive + lw * 4 + row;
      if (o < nout) {
        const uint32_t sl = o < noA ? 0u : 1u;
        const uint32_t j = olist[sl][o - (sl ? noA : 0u)];
        uint32_t v[16];
        static_for<4>([&](auto Q) {
          constexpr int q = decltype(Q)::value;
          const uint4 x = lds[(o * 4 + q) * kSl + col];
          v[4 * q] = x.x;
          v[4 * q + 1] = x.y;
          v[4 * q + 2] = x.z;
          v[4 * q + 3] = x.w;
        });
        dev::mul_rt_poly(v, lcoef[sl * W + j]);
        if (tail_lane) {
          dev::transpose8(v);
          dev::transpose8(v + 8);
          store_tail_chunk(const_cast<uint8_t*>(src_of(sl, j)), p.tail_bytes, v);
        } else {
          dev::store_chunk<true>(const_cast<uint8_t*>(src_of(sl, j)), v);
        }
      }
    }
  });
}

template <int OUTH, bool TAIL = false>
__global__ __launch_bounds__(512, 4) void decode_pk_kernel(const DecodeXParams p) {
  __shared__ uint4 lds[16 * 4 * kXfLanes];
  __shared__ X8Flags flags;
  __shared__ PkShared sh;
  decode_pk_tile<OUTH, false, TAIL>(p, dev::xcd_tile(blockIdx.x, gridDim.x), lds, &flags, sh);
}

// Per pattern and window position x: the decoder's locator constant as a bitsliced
// multiply matrix.  loc(x) = sum_{e erased, e != x} log(x ^ e) (mod 65535) -- the crate's
// eval_poly over the window up to one constant factor, which cancels between the input
// multiply (present x: exp(loc)) and the output multiply (restored x: exp(-loc)).
// poly: one word per position instead -- the constant in the polynomial basis (mul_rt_poly).
//
// loc is the XOR convolution of L(z) = log z (L(0) = 0, which drops e = x; log[0] = 65535 is
// the same residue) with the erasure indicator, so it comes out of Walsh-Hadamard transforms
// over Z/65535 (the crate's own error-locator route, on the window instead of the field):
// loc = H(H(L) * H(I)) / N.  The window's L is zero past W, so an N-point transform
// (N = 64, or 128 with two positions per lane) serves every W <= N.  One wave per pattern,
// lane-shuffle stages, no loop over the erased positions; exp depends only on the residue
// (exp[65535] = exp[0]), so the constants are the loop form's bit for bit.

__global__ __launch_bounds__(256) void decode_rows_kernel(const uint64_t* __restrict__ emask,
                                                          const uint64_t* __restrict__ pmask, uint32_t npat,
                                                          uint32_t W, const uint16_t* __restrict__ log_t,
                                                          const uint16_t* __restrict__ exp_t, uint32_t* rows,
                                                          uint32_t poly) {
  const uint64_t pat = static_cast<uint64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (pat >= npat) return;  // wave-uniform
  const int lane = threadIdx.x & 63;
  const uint32_t x = static_cast<uint32_t>(lane);
  const uint64_t e = emask[pat], in = pmask[2 * pat], out = pmask[2 * pat + 1];
  // H(L) / 64 (64^-1 = 1024: 2^16 = 1)
  const uint32_t hl = m65535_mul(walsh64(x && x < W ? log_t[x] : 0u, lane), 1024u);
  const uint32_t hi = walsh64(x < W ? static_cast<uint32_t>((e >> x) & 1) : 0u, lane);
  const uint32_t acc = walsh64(m65535_mul(hl, hi), lane);
  if (x >= W) return;
  const bool is_in = (in >> x) & 1, is_out = (out >> x) & 1;
  if (!is_in && !is_out) return;
  const uint16_t lg = locator_log(acc, is_in);
  if (poly) {
    rows[pat * W + x] = dev::to_poly(exp_t[lg]);  // exp[lg] = the constant
    return;
  }
  uint32_t* dst = rows + (pat * W + x) * 16;
  uint32_t r[16] = {};
  for (int i = 0; i < 16; ++i) {
    const uint16_t prod = dev::gmul(exp_t, log_t, static_cast<uint16_t>(1u << i), lg);
    for (int o = 0; o < 16; ++o) r[o] |= ((prod >> o) & 1u) << i;
  }
  for (int o = 0; o < 16; ++o) dst[o] = r[o];
}

// =====================================================================================
// encode_mc<C>: multi-chunk HighRate encode for small recovery sets (chunk C = next_pow2(m)
// in {1, 2, 4}, k <= kMcMaxK).  One wave per 64-column tile, no LDS: the wave streams the
// k/C original chunks (next chunk's loads issued before this chunk's math), runs each
// chunk's in-lane IFFT_C (skew delta C*(c+1)), XOR-accumulates, and ends with FFT_C (delta
// 0) on the accumulator -- the crate's HighRate encoder.
// =====================================================================================
constexpr int kMcMaxK = 64;

template <int C>
constexpr int ilog2c() { return C <= 1 ? 0 : 1 + ilog2c<C / 2>(); }

template <int C, int DELTA, bool INV>
__device__ __forceinline__ void xform_lane(uint32_t (&r)[C][16]) {
  constexpr int LC = ilog2c<C>();
  static_for<LC>([&](auto Lx) {
    constexpr int L = INV ? decltype(Lx)::value : LC - 1 - decltype(Lx)::value;  // IFFT ascending
    constexpr int d = 1 << L;
    static_for<C / 2>([&](auto I) {
      constexpr int i = decltype(I)::value;
      constexpr int g = (i / d) * 2 * d;
      constexpr int u = g + i % d;
      bfly<g + d + DELTA - 1, INV>(r[u], r[u + d]);
    });
  });
}

template <int C>
__device__ __forceinline__ void mc_load(const XformParams& p, const TileIO& io, uint32_t s0, uint32_t (&raw)[C][16]) {
  static_for<C>([&](auto T) {
    constexpr int t = decltype(T)::value;
    if (s0 + t < p.n_in) {  // wave-uniform
      const uint8_t* base = p.in + (s0 + t) * p.in_shard_stride;
      static_for<4>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        const uint4 x = ld_piece(base + io.off[q]);
        raw[t][4 * q] = x.x;
        raw[t][4 * q + 1] = x.y;
        raw[t][4 * q + 2] = x.z;
        raw[t][4 * q + 3] = x.w;
      });
    } else {
      static_for<16>([&](auto P) { raw[t][decltype(P)::value] = 0; });
    }
  });
}

template <int C>
__global__ __launch_bounds__(256, 2) void encode_mc_kernel(const XformParams p) {
  constexpr int NCMAX = kMcMaxK / C;
  const int lane = threadIdx.x & 63;
  const uint64_t tile = static_cast<uint64_t>(dev::xcd_tile(blockIdx.x, gridDim.x)) * 4 + (threadIdx.x >> 6);
  if (tile * kXfLanes >= p.total_columns) return;  // whole wave
  const TileIO io = tile_io(p, tile, lane, p.in_block_stride);
  const uint32_t nc = (p.n_in + C - 1) / C;
  uint32_t acc[C][16];
  uint32_t raw[2][C][16];
  mc_load<C>(p, io, 0, raw[0]);
  static_for<NCMAX>([&](auto Cc) {
    constexpr int c = decltype(Cc)::value;
    if (c < nc) {
      if (c + 1 < nc) mc_load<C>(p, io, (c + 1) * C, raw[(c + 1) & 1]);
      auto& cur = raw[c & 1];
      static_for<C>([&](auto T) {
        swap_halves(cur[decltype(T)::value]);
        dev::planes_from_raw(cur[decltype(T)::value]);
      });
      xform_lane<C, C * (c + 1), true>(cur);
      static_for<C>([&](auto T) {
        constexpr int t = decltype(T)::value;
        static_for<16>([&](auto P) {
          constexpr int q = decltype(P)::value;
          if constexpr (c == 0) acc[t][q] = cur[t][q]; else acc[t][q] ^= cur[t][q];
        });
      });
    }
  });
  xform_lane<C, 0, false>(acc);
  const TileIO out_io = tile_io(p, tile, lane, p.out_block_stride);
  static_for<C>([&](auto T) {
    constexpr int t = decltype(T)::value;
    if (t < p.n_out) store_shard(p.out + t * p.out_shard_stride, out_io, out_io.valid, acc[t]);
  });
}

// =====================================================================================
// decode_syn<C>: syndrome decoder for small recovery sets (chunk C = next_pow2(m) <= 4,
// k <= kMcMaxK).  One wave per 64-column tile, no LDS.  The wave re-encodes the present
// originals exactly as encode_mc does (erased originals read as zero), adds e received
// recovery shards (syndromes S_b = received_b ^ re-encoded_b = sum over erased a of
// G[b][a] * original_a) and restores original E[a] = sum_b Minv[a][b] S_b with e^2 runtime
// multiplies.  Any correct decoder returns the crate's originals on a valid codeword (MDS).
// =====================================================================================
typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));

// the 16 XOR combinations of planes x[0..3] (entry v = XOR of x[i] for the bits i of v)
__device__ __forceinline__ u32x16 syn_table(const uint32_t* x) {
  const uint32_t a = x[0], b = x[1], c = x[2], d = x[3];
  const uint32_t ab = a ^ b, cd = c ^ d;
  return u32x16{0u, a, b, ab, c, a ^ c, b ^ c, ab ^ c, d, a ^ d, b ^ d, ab ^ d, cd, a ^ cd, b ^ cd, ab ^ cd};
}

// acc ^= M x for a runtime 16x16 GF(2) matrix in (wave-uniform) global memory
__device__ __forceinline__ void mul_rt_acc(uint32_t* acc, const uint32_t* x, const uint32_t* __restrict__ rows) {
  static_for<16>([&](auto O) {
    constexpr int o = decltype(O)::value;
    const uint32_t r = __builtin_amdgcn_readfirstlane(rows[o]);
    uint32_t a = acc[o];
    static_for<16>([&](auto I) {
      constexpr int i = decltype(I)::value;
      const uint32_t msk = static_cast<uint32_t>(static_cast<int32_t>(r << (31 - i)) >> 31);
      a = __builtin_amdgcn_bitop3_b32(a, x[i], msk, 0x78);  // a ^ (x & msk)
    });
    acc[o] = a;
  });
}

template <int C>
__device__ __forceinline__ void syn_load(const DecodeSynParams& p, const TileIO& io, uint64_t dmask, uint32_t s0,
                                         uint32_t (&raw)[C][16]) {
  static_for<C>([&](auto T) {
    constexpr int t = decltype(T)::value;
    const uint32_t s = s0 + t;
    if (s < p.k && ((dmask >> s) & 1)) {  // wave-uniform
      const uint8_t* base = p.orig + s * p.orig_shard_stride;
      static_for<4>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        const uint4 x = ld_piece(base + io.off[q]);
        raw[t][4 * q] = x.x;
        raw[t][4 * q + 1] = x.y;
        raw[t][4 * q + 2] = x.z;
        raw[t][4 * q + 3] = x.w;
      });
    } else {
      static_for<16>([&](auto P) { raw[t][decltype(P)::value] = 0; });
    }
  });
}

template <int C>
__global__ __launch_bounds__(256, 2) void decode_syn_kernel(const DecodeSynParams p) {
  constexpr int NCMAX = kMcMaxK / C;
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint64_t tile = static_cast<uint64_t>(dev::xcd_tile(blockIdx.x, gridDim.x)) * 4 + wave;
  if (tile >= p.ntiles) return;  // whole wave
  uint64_t pat = 0;
  if (p.per_block) {
    const uint64_t bi = tile / p.tiles_per_block;
    const uint64_t blk = p.block_ids ? p.block_ids[bi] : bi;
    tile = blk * p.tiles_per_block + (tile - bi * p.tiles_per_block);
    pat = blk;
  }
  const SynPattern* sp = p.pat + pat;
  const uint64_t dmask = sp->dmask;
  const uint32_t e = sp->e;
  const TileIO io = tile_io_g(p.total_columns, p.chunks_per_shard, tile, lane, p.orig_block_stride);
  const TileIO rio = tile_io_g(p.total_columns, p.chunks_per_shard, tile, lane, p.rec_block_stride);
  const uint32_t nc = (p.k + C - 1) / C;
  // recovery positions used for the syndromes (wave-uniform)
  uint32_t used = 0;
  for (uint32_t b = 0; b < e; ++b) used |= 1u << sp->rec[b];
  // Stage 0 streams the used received recovery shards R (zero elsewhere) and starts the
  // accumulator at IFFT_C,0(R); stages 1..nc stream the present originals' chunks as encode_mc.
  // The final FFT_C,0 then yields re-encoded ^ R = the syndromes at the used positions
  // (linearity), so no dependent recovery load sits between the stream and the correction.
  uint32_t acc[C][16];
  uint32_t raw[2][C][16];
  static_for<C>([&](auto T) {
    constexpr int t = decltype(T)::value;
    if ((used >> t) & 1) {
      const uint8_t* base = p.rec + t * p.rec_shard_stride;
      static_for<4>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        const uint4 x = ld_piece(base + rio.off[q]);
        raw[0][t][4 * q] = x.x;
        raw[0][t][4 * q + 1] = x.y;
        raw[0][t][4 * q + 2] = x.z;
        raw[0][t][4 * q + 3] = x.w;
      });
    } else {
      static_for<16>([&](auto P) { raw[0][t][decltype(P)::value] = 0; });
    }
  });
  static_for<NCMAX + 1>([&](auto Sg) {
    constexpr int sg = decltype(Sg)::value;
    if (sg <= nc) {
      if (sg < nc) syn_load<C>(p, io, dmask, sg * C, raw[(sg + 1) & 1]);
      auto& cur = raw[sg & 1];
      static_for<C>([&](auto T) {
        swap_halves(cur[decltype(T)::value]);
        dev::planes_from_raw(cur[decltype(T)::value]);
      });
      if constexpr (sg == 0) {
        xform_lane<C, 0, true>(cur);
      } else {
        xform_lane<C, C * sg, true>(cur);
      }
      static_for<C>([&](auto T) {
        constexpr int t = decltype(T)::value;
        static_for<16>([&](auto P) {
          constexpr int q = decltype(P)::value;
          if constexpr (sg == 0) acc[t][q] = cur[t][q]; else acc[t][q] ^= cur[t][q];
        });
      });
    }
  });
  xform_lane<C, 0, false>(acc);  // syndromes S_b at positions rec[b]
  // Four Russians in registers (mul_rt4's scheme): per syndrome b, the 16 XOR combinations
  // of each 4-plane group (44 VALU) serve all e outputs; output plane o of Minv[a][b] S_b is
  // the XOR of 4 entries picked by row o's wave-uniform nibbles (one v_movrels each).
  // Syndromes, tables and outputs stay in VGPRs (2 waves per SIMD: 256 available).
  uint32_t out[C][16];
  static_for<C>([&](auto A) { static_for<16>([&](auto P) { out[decltype(A)::value][decltype(P)::value] = 0; }); });
  // one set of 4 tables reused for every syndrome: LLVM promotes these allocas to VGPRs
  // (dynamic picks = v_movrels) within its promote-alloca budget; a set per syndrome
  // overflows the budget and lands in scratch
  uint32_t t0[16], t1[16], t2[16], t3[16];
  static_for<C>([&](auto J) {
    constexpr int j = decltype(J)::value;
    if ((used >> j) & 1) {
      uint32_t b = 0;
      while (b + 1 < e && sp->rec[b] != j) ++b;  // wave-uniform: the syndrome index of position j
      const uint32_t* x = acc[j];
      auto fill = [&](uint32_t* t, const uint32_t* v) {
        const u32x16 c = syn_table(v);
        static_for<16>([&](auto V) { t[decltype(V)::value] = c[decltype(V)::value]; });
      };
      fill(t0, x);
      fill(t1, x + 4);
      fill(t2, x + 8);
      fill(t3, x + 12);
      static_for<C>([&](auto A) {
        constexpr int a = decltype(A)::value;
        if (a < e) {
          const uint32_t* rows = sp->rows[a][b];
          static_for<16>([&](auto O) {
            constexpr int o = decltype(O)::value;
            const uint32_t r = __builtin_amdgcn_readfirstlane(rows[o]);
            out[a][o] = dev::xor3(out[a][o], t0[r & 15], t1[(r >> 4) & 15]) ^
                        dev::xor3(t2[(r >> 8) & 15], t3[(r >> 12) & 15], 0u);
          });
        }
      });
    }
  });
  static_for<C>([&](auto A) {
    constexpr int a = decltype(A)::value;
    if (a < e) store_shard(p.orig + sp->out[a] * p.orig_shard_stride, io, io.valid, out[a]);
  });
}

// =====================================================================================
// Generic kernels: one thread per (block, symbol position); the crate's algorithm with
// log/exp tables, work rows in a global scratch column (stride nsym).
// =====================================================================================

struct SymAddr {
  uint32_t lo, hi;
};
__device__ __forceinline__ SymAddr sym_addr(uint32_t j, uint32_t shard_bytes) {
  const uint32_t c = j >> 5, jj = j & 31, whole = shard_bytes >> 6;
  if (c < whole) return {64 * c + jj, 64 * c + 32 + jj};
  const uint32_t h = (shard_bytes & 63) >> 1;
  return {64 * whole + jj, 64 * whole + h + jj};
}

struct Col {
  uint16_t* w;
  uint64_t st;
  __device__ uint16_t& operator[](uint32_t i) const { return w[i * st]; }
};

__device__ void g_fft(const Col& w, const GfDeviceTables& t, uint32_t pos, uint32_t size, uint32_t trunc,
                      uint32_t delta) {
  for (uint32_t dist = size >> 1; dist >= 1; dist >>= 1) {
    for (uint32_t r = 0; r < trunc; r += 2 * dist) {
      const uint16_t lm = t.skew[r + dist + delta - 1];
      for (uint32_t i = r; i < r + dist; ++i) {
        uint16_t x = w[pos + i], y = w[pos + i + dist];
        if (lm != 65535) x ^= dev::gmul(t.exp, t.log, y, lm);
        y ^= x;
        w[pos + i] = x;
        w[pos + i + dist] = y;
      }
    }
  }
}

__device__ void g_ifft(const Col& w, const GfDeviceTables& t, uint32_t pos, uint32_t size, uint32_t trunc,
                       uint32_t delta) {
  for (uint32_t dist = 1; dist < size; dist <<= 1) {
    for (uint32_t r = 0; r < trunc; r += 2 * dist) {
      const uint16_t lm = t.skew[r + dist + delta - 1];
      for (uint32_t i = r; i < r + dist; ++i) {
        uint16_t x = w[pos + i], y = w[pos + i + dist];
        y ^= x;
        if (lm != 65535) x ^= dev::gmul(t.exp, t.log, y, lm);
        w[pos + i] = x;
        w[pos + i + dist] = y;
      }
    }
  }
}

__global__ __launch_bounds__(256) void generic_encode_kernel(const GenericEncodeParams p) {
  const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (tid >= p.nblocks * p.nsym) return;
  const uint64_t b = tid / p.nsym;
  const uint32_t j = static_cast<uint32_t>(tid - b * p.nsym);
  const SymAddr a = sym_addr(j, p.shard_bytes);
  const Col w{p.scratch + b * p.rows * p.nsym + j, p.nsym};
  const uint8_t* ob = p.orig + b * p.orig_block_stride;
  for (uint32_t i = 0; i < p.rows; ++i) {
    uint16_t v = 0;
    if (i < p.k) {
      const uint8_t* s = ob + i * p.orig_shard_stride;
      v = static_cast<uint16_t>(s[a.lo] | (s[a.hi] << 8));
    }
    w[i] = v;
  }
  const uint32_t chunk = p.chunk, k = p.k, m = p.m;
  if (p.high_rate) {
    g_ifft(w, p.t, 0, chunk, k < chunk ? k : chunk, chunk);
    if (k > chunk) {
      uint32_t cs = chunk;
      for (; cs + chunk <= k; cs += chunk) {
        g_ifft(w, p.t, cs, chunk, chunk, cs + chunk);
        for (uint32_t i = 0; i < chunk; ++i) w[i] ^= w[cs + i];
      }
      const uint32_t last = k % chunk;
      if (last) {
        g_ifft(w, p.t, cs, chunk, last, cs + chunk);
        for (uint32_t i = 0; i < chunk; ++i) w[i] ^= w[cs + i];
      }
    }
    g_fft(w, p.t, 0, chunk, m, 0);
  } else {
    g_ifft(w, p.t, 0, chunk, k, 0);
    for (uint32_t cs = chunk; cs < m; cs += chunk)
      for (uint32_t i = 0; i < chunk; ++i) w[cs + i] = w[i];
    uint32_t cs = 0;
    for (; cs + chunk <= m; cs += chunk) g_fft(w, p.t, cs, chunk, chunk, cs + chunk);
    if (m % chunk) g_fft(w, p.t, cs, chunk, m % chunk, cs + chunk);
  }
  uint8_t* rb = p.rec + b * p.rec_block_stride;
  for (uint32_t i = 0; i < m; ++i) {
    uint8_t* s = rb + i * p.rec_shard_stride;
    const uint16_t v = w[i];
    s[a.lo] = static_cast<uint8_t>(v);
    s[a.hi] = static_cast<uint8_t>(v >> 8);
  }
}

__global__ __launch_bounds__(256) void generic_decode_kernel(const GenericDecodeParams p) {
  const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (tid >= p.nblocks * p.nsym) return;
  const uint64_t bi = tid / p.nsym;
  const uint32_t j = static_cast<uint32_t>(tid - bi * p.nsym);
  const uint64_t b = p.block_ids ? p.block_ids[bi] : p.block_base + bi;
  const uint64_t pat = p.pattern_per_block ? b : 0;
  const uint8_t* op = p.orig_present + pat * p.k;
  const uint8_t* rp = p.rec_present + pat * p.m;
  const uint16_t* loc = p.loc + pat * p.W;
  const SymAddr a = sym_addr(j, p.shard_bytes);
  const Col w{p.scratch + bi * p.W * p.nsym + j, p.nsym};
  const uint32_t opos = p.high_rate ? p.chunk : 0, rpos = p.high_rate ? 0 : p.chunk;
  for (uint32_t i = 0; i < p.W; ++i) w[i] = 0;
  uint8_t* ob = p.orig + b * p.orig_block_stride;
  const uint8_t* rbk = p.rec + b * p.rec_block_stride;
  for (uint32_t i = 0; i < p.k; ++i)
    if (op[i]) {
      const uint8_t* s = ob + i * p.orig_shard_stride;
      w[opos + i] = dev::gmul(p.t.exp, p.t.log, static_cast<uint16_t>(s[a.lo] | (s[a.hi] << 8)), loc[opos + i]);
    }
  for (uint32_t i = 0; i < p.m; ++i)
    if (rp[i]) {
      const uint8_t* s = rbk + i * p.rec_shard_stride;
      w[rpos + i] = dev::gmul(p.t.exp, p.t.log, static_cast<uint16_t>(s[a.lo] | (s[a.hi] << 8)), loc[rpos + i]);
    }
  g_ifft(w, p.t, 0, p.W, p.end, 0);
  for (uint32_t i = 1; i < p.W; ++i) {  // formal derivative
    const uint32_t width = i & (~i + 1);
    for (uint32_t q = 0; q < width; ++q) w[i - width + q] ^= w[i + q];
  }
  g_fft(w, p.t, 0, p.W, p.high_rate ? p.end : p.k, 0);
  for (uint32_t i = 0; i < p.k; ++i)
    if (!op[i]) {
      const uint16_t v = dev::gmul(p.t.exp, p.t.log, w[opos + i], static_cast<uint16_t>(65535 - loc[opos + i]));
      uint8_t* s = ob + i * p.orig_shard_stride;
      s[a.lo] = static_cast<uint8_t>(v);
      s[a.hi] = static_cast<uint8_t>(v >> 8);
    }
}

// =====================================================================================
// Erasure locator: the crate's eval_poly (FWHT, pointwise x log_walsh, FWHT), mod 65535,
// one 1024-thread workgroup per pattern with the 65536-entry vector in LDS (128 KiB).
// =====================================================================================
__device__ __forceinline__ void fwht_lds(uint16_t* buf) {
  for (uint32_t dist = 1; dist < 65536; dist <<= 1) {
    for (uint32_t idx = threadIdx.x; idx < 32768; idx += blockDim.x) {
      const uint32_t i = (idx / dist) * 2 * dist + (idx % dist);
      const uint16_t a = buf[i], b = buf[i + dist];
      buf[i] = dev::add_mod(a, b);
      buf[i + dist] = dev::sub_mod(a, b);
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(1024) void locator_kernel(const uint8_t* erased, uint32_t W, uint32_t fill_from,
                                                       const uint16_t* log_walsh, uint16_t* loc) {
  __shared__ uint16_t buf[65536];
  const uint64_t pat = blockIdx.x;
  for (uint32_t x = threadIdx.x; x < 65536; x += blockDim.x)
    buf[x] = x < W ? (erased[pat * W + x] ? 1 : 0) : (x >= fill_from ? 1 : 0);
  __syncthreads();
  fwht_lds(buf);
  for (uint32_t x = threadIdx.x; x < 65536; x += blockDim.x) {
    const uint32_t prod = static_cast<uint32_t>(buf[x]) * log_walsh[x];
    buf[x] = dev::add_mod(prod & 0xFFFF, prod >> 16);
  }
  __syncthreads();
  fwht_lds(buf);
  for (uint32_t x = threadIdx.x; x < W; x += blockDim.x) loc[pat * W + x] = buf[x];
}

// =====================================================================================
// ReedSolomonCoder batch helpers (reed_solomon.rs:88-128 shred padding, :190-203 strip)
// =====================================================================================
// Data region of slice b (32 * S bytes at cw + b * cw_stride) := payload || 0x80 || 0...
// (payload == null: the payload already sits in the data region; only the padding is
// written).  One thread per 16 output bytes.
// One workgroup per slice, its threads striding over the slice's 16-byte pieces: with a
// payload source every piece is copied (the tail piece merged with 0x80 00..); in place
// (payload null) only the pieces from the one holding byte `len` are written -- a maximum
// slice's padding is one piece, where the earlier one-thread-per-piece grid read every
// piece's length word and divided for it (0.3 ms per 65 536 slices for one byte each).
__global__ __launch_bounds__(256) void coder_pad_kernel(const uint8_t* __restrict__ payload, uint64_t payload_stride,
                                                        const uint32_t* __restrict__ lens, uint8_t* cw,
                                                        uint64_t cw_stride, uint32_t data_bytes, uint64_t nslices) {
  // with a payload one workgroup copies one slice; in place (payload null) only the pieces
  // from byte len on change, so a wave serves one slice and a workgroup four (dispatch-bound
  // otherwise: 65 536 one-wave workgroups took 25 us for one piece each)
  const uint64_t b = payload ? blockIdx.x : static_cast<uint64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (b >= nslices) return;
  const uint32_t tid = payload ? threadIdx.x : (threadIdx.x & 63), nt = payload ? blockDim.x : 64;
  const uint32_t per = data_bytes / 16;
  const uint32_t len = lens[b];
  uint8_t* base = cw + b * cw_stride;
  const uint8_t* src = payload ? payload + b * payload_stride : nullptr;
  const bool a16 = src && (reinterpret_cast<uintptr_t>(src) & 15) == 0;
  for (uint32_t piece = (src ? 0u : len / 16) + tid; piece < per; piece += nt) {
    const uint32_t j = piece * 16;
    uint8_t* dst = base + j;
    if (j + 16 <= len) {  // whole payload piece (only with a source)
      if (a16) {
        *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(src + j);
      } else {
        for (int i = 0; i < 16; ++i) dst[i] = src[j + i];
      }
      continue;
    }
    if (j >= len + 1) {  // padding zeros only
      *reinterpret_cast<uint4*>(dst) = make_uint4(0, 0, 0, 0);
      continue;
    }
    uint8_t v[16];
    for (int i = 0; i < 16; ++i) {
      const uint32_t pos = j + i;
      v[i] = pos < len ? (src ? src[pos] : dst[i]) : (pos == len ? 0x80 : 0);
    }
    for (int i = 0; i < 16; ++i) dst[i] = v[i];
  }
}

// Shard restride for shard sizes that are not whole 64-byte chunks (the
// crate stores the last T = S mod 64 bytes as T/2 low bytes then T/2 high bytes of T/2
// symbols).  pack: shard (S bytes, any alignment) -> padded shard of Sp = ceil(S/64)*64
// bytes whose last chunk holds the tail symbols in whole-chunk layout (low bytes at 0..,
// high bytes at 32..) with zero symbols after them; unpack is the inverse and writes only
// the shards selected by the store mask.  A pack mask skips shards (the decoders never read
// an absent shard, so its padded slot may keep stale bytes).  Zero symbols are zero columns of every linear
// transform, so the bitsliced kernels run on the padded shards unchanged.
struct RestrideParams {
  const uint8_t* src;
  uint64_t src_block_stride, src_shard_stride;
  uint8_t* dst;
  uint64_t dst_block_stride, dst_shard_stride;
  uint32_t S, Sp, nshards, unpack;
  uint64_t nblocks;
  const uint64_t* mask;  // unpack: store shard s of block b iff bit s of mask[per_block ? b : 0]
  uint32_t mask_per_block;
};
// padded offset q -> offset in the crate-layout shard, or -1 (a zero symbol's byte)
__device__ __forceinline__ int64_t restride_src(uint32_t q, uint32_t S) {
  const uint32_t whole = S >> 6, h = (S & 63) >> 1;
  if (q < 64 * whole) return q;
  const uint32_t w = q - 64 * whole;
  if (w < 32) return w < h ? static_cast<int64_t>(64 * whole + w) : -1;
  return w - 32 < h ? static_cast<int64_t>(64 * whole + h + (w - 32)) : -1;
}
// 16 bytes at a 2-byte-aligned (or better) address as 4 little-endian dwords
__device__ __forceinline__ uint4 load16_a2(const uint8_t* src) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(src);
  if ((a & 15) == 0) return *reinterpret_cast<const uint4*>(src);
  if ((a & 7) == 0) {
    const uint2 lo = reinterpret_cast<const uint2*>(src)[0], hi = reinterpret_cast<const uint2*>(src)[1];
    return make_uint4(lo.x, lo.y, hi.x, hi.y);
  }
  if ((a & 3) == 0) {
    const uint32_t* d = reinterpret_cast<const uint32_t*>(src);
    return make_uint4(d[0], d[1], d[2], d[3]);
  }
  // a % 4 == 2: the middle three dwords are aligned; the outer half-dwords are read as
  // 16-bit loads so that nothing outside [a, a + 16) is touched
  const uint32_t* d = reinterpret_cast<const uint32_t*>(a + 2);
  const uint32_t d0 = static_cast<uint32_t>(*reinterpret_cast<const uint16_t*>(src)) << 16;
  const uint32_t d1 = d[0], d2 = d[1], d3 = d[2];
  const uint32_t d4 = *reinterpret_cast<const uint16_t*>(src + 14);
  return make_uint4(__builtin_amdgcn_alignbyte(d1, d0, 2), __builtin_amdgcn_alignbyte(d2, d1, 2),
                    __builtin_amdgcn_alignbyte(d3, d2, 2), __builtin_amdgcn_alignbyte(d4, d3, 2));
}
__device__ __forceinline__ void store16_a2(uint8_t* dst, uint4 v) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(dst);
  if ((a & 15) == 0) {
    *reinterpret_cast<uint4*>(dst) = v;
  } else if ((a & 7) == 0) {
    reinterpret_cast<uint2*>(dst)[0] = make_uint2(v.x, v.y);
    reinterpret_cast<uint2*>(dst)[1] = make_uint2(v.z, v.w);
  } else if ((a & 3) == 0) {
    uint32_t* d = reinterpret_cast<uint32_t*>(dst);
    d[0] = v.x;
    d[1] = v.y;
    d[2] = v.z;
    d[3] = v.w;
  } else {  // a % 4 == 2: a half-dword, three dwords, a half-dword
    uint16_t* h = reinterpret_cast<uint16_t*>(dst);
    uint32_t* d = reinterpret_cast<uint32_t*>(dst + 2);
    h[0] = static_cast<uint16_t>(v.x);
    d[0] = __builtin_amdgcn_alignbyte(v.y, v.x, 2);
    d[1] = __builtin_amdgcn_alignbyte(v.z, v.y, 2);
    d[2] = __builtin_amdgcn_alignbyte(v.w, v.z, 2);
    h[7] = static_cast<uint16_t>(v.w >> 16);
  }
}

// One thread per 16 bytes of the padded shard.  Whole chunks move as 16-byte pieces (shard
// sizes are even, so the crate-layout side is at least 2-byte aligned when its strides
// are even); the tail chunk and odd strides go byte by byte.
__global__ __launch_bounds__(256) void restride_kernel(const RestrideParams p) {
  // one thread per 16-byte piece of the padded layout, flattened over (block, shard, piece):
  // small tails (4 pieces per shard) fill whole workgroups
  const uint32_t per_shard = p.Sp / 16, per_block = per_shard * p.nshards;
  const uint64_t gid = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t b = gid / per_block;
  if (b >= p.nblocks) return;
  const uint32_t r = static_cast<uint32_t>(gid - b * per_block);
  const uint32_t sh = r / per_shard, u = r - sh * per_shard;
  const uint32_t q = 16 * u;
  const bool whole = q + 16 <= 64 * (p.S >> 6);
  if (p.mask && !((p.mask[p.mask_per_block ? b : 0] >> sh) & 1)) return;  // shard not selected
  if (!p.unpack) {
    const uint8_t* src = p.src + b * p.src_block_stride + sh * p.src_shard_stride;
    uint4* dst = reinterpret_cast<uint4*>(p.dst + b * p.dst_block_stride + sh * p.dst_shard_stride + q);
    if (whole && (reinterpret_cast<uintptr_t>(src) & 1) == 0) {
      *dst = load16_a2(src + q);
    } else if (!whole && (reinterpret_cast<uintptr_t>(src) & 1) == 0) {
      // a tail piece: L <= 16 contiguous source bytes (low or high half of the tail
      // symbols), read as the aligned dwords holding them (never past a dword with a valid
      // byte, so never across a page), funnel-shifted, bytes past L zeroed
      const uint32_t tb = 64 * (p.S >> 6), h = (p.S & 63) >> 1, w = q - tb;
      const uint32_t off = w & 31, start = tb + (w < 32 ? 0 : h) + off;
      const uint32_t L = off < h ? min(16u, h - off) : 0u;
      uint32_t v[4] = {0, 0, 0, 0};
      if (L) {
        const uintptr_t a = reinterpret_cast<uintptr_t>(src + start);
        const uint32_t* base = reinterpret_cast<const uint32_t*>(a & ~uintptr_t{3});
        const uint32_t sh = static_cast<uint32_t>(a & 3), nd = (sh + L + 3) >> 2;
        uint32_t d[5];
#pragma unroll
        for (uint32_t j = 0; j < 5; ++j) d[j] = base[min(j, nd - 1)];
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
          const uint32_t x = __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh);
          const uint32_t nb = L > 4 * j ? min(4u, L - 4 * j) : 0u;
          v[j] = nb >= 4 ? x : x & ((1u << (8 * nb)) - 1);
        }
      }
      *dst = make_uint4(v[0], v[1], v[2], v[3]);
    } else {
      // 16 independent byte loads (a zero symbol's byte reads the tail's first byte and is
      // masked): a conditional load per byte serialised 16 memory latencies per wave
      const int64_t tb = 64 * (p.S >> 6);
      uint32_t v[4] = {0, 0, 0, 0};
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int64_t o = restride_src(q + i, p.S);
        const uint32_t x = src[o >= 0 ? o : tb];
        v[i >> 2] |= (o >= 0 ? x : 0u) << (8 * (i & 3));
      }
      *dst = make_uint4(v[0], v[1], v[2], v[3]);
    }
  } else {
    const uint4 v = *reinterpret_cast<const uint4*>(p.src + b * p.src_block_stride + sh * p.src_shard_stride + q);
    uint8_t* dst = p.dst + b * p.dst_block_stride + sh * p.dst_shard_stride;
    if (whole && (reinterpret_cast<uintptr_t>(dst) & 1) == 0) {
      store16_a2(dst + q, v);
    } else {
      // a tail piece is one run of L <= 16 contiguous destination bytes (the low or high
      // half of the tail symbols): dword stores when the run is dword-aligned and whole
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
      const uint32_t tb = 64 * (p.S >> 6), h = (p.S & 63) >> 1, wq = q - tb;
      const uint32_t off = wq & 31, start = tb + (wq < 32 ? 0 : h) + off;
      const uint32_t L = whole ? 16u : (off < h ? min(16u, h - off) : 0u);
      if (!whole && ((reinterpret_cast<uintptr_t>(dst + start) | L) & 3) == 0) {
        uint32_t* d4 = reinterpret_cast<uint32_t*>(dst + start);
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
          if (4 * j < L) d4[j] = w[j];
      } else {
        for (int i = 0; i < 16; ++i) {
          const int64_t o = restride_src(q + i, p.S);
          if (o >= 0) dst[o] = static_cast<uint8_t>(w[i >> 2] >> (8 * (i & 3)));
        }
      }
    }
  }
}

// Unpack of tail-only shards (0 < S < 64: one padded chunk per shard) to an even destination.
// The workgroup stages its 64 chunks in LDS; then the four threads of a shard write the S
// destination bytes as aligned dwords, with half-dwords at the two ends.  The per-piece path
// above falls back to byte stores for every run that starts off a dword: 3 of the 4 runs of
// a 62-byte tail.
__global__ __launch_bounds__(256) void unpack_tail_kernel(const RestrideParams p) {
  __shared__ uint4 chunk[256];
  const uint32_t t = threadIdx.x, u = t & 3;
  const uint64_t g = (static_cast<uint64_t>(blockIdx.x) * 256 + t) >> 2;  // (block, shard)
  const uint64_t b = g / p.nshards;
  const uint32_t sh = static_cast<uint32_t>(g - b * p.nshards);
  const bool sel = b < p.nblocks && (!p.mask || ((p.mask[p.mask_per_block ? b : 0] >> sh) & 1));
  if (sel)
    chunk[t] = *reinterpret_cast<const uint4*>(p.src + b * p.src_block_stride + sh * p.src_shard_stride + 16 * u);
  __syncthreads();
  if (!sel) return;
  const uint8_t* c = reinterpret_cast<const uint8_t*>(chunk + (t & ~3u));
  const int32_t T = static_cast<int32_t>(p.S), h = T >> 1;
  uint8_t* a = p.dst + b * p.dst_block_stride + sh * p.dst_shard_stride;
  const int32_t lead = static_cast<int32_t>(reinterpret_cast<uintptr_t>(a) & 3);  // 0 or 2
  uint8_t* a0 = a - lead;
  const int32_t nd = (lead + T + 3) >> 2;
  for (int32_t j = static_cast<int32_t>(u); j < nd; j += 4) {
    const int32_t i0 = 4 * j - lead;  // destination byte of the dword's first byte
    uint32_t x = 0;
#pragma unroll
    for (int32_t s = 0; s < 4; ++s) {
      // destination byte i: the low symbol bytes (padded 0..h-1), then the high (32..)
      const int32_t i = i0 + s;
      if (i >= 0 && i < T) x |= static_cast<uint32_t>(c[i < h ? i : 32 + i - h]) << (8 * s);
    }
    if (i0 >= 0 && i0 + 4 <= T) *reinterpret_cast<uint32_t*>(a0 + 4 * j) = x;
    else if (i0 < 0) *reinterpret_cast<uint16_t*>(a0 + 4 * j + 2) = static_cast<uint16_t>(x >> 16);
    else *reinterpret_cast<uint16_t*>(a0 + 4 * j) = static_cast<uint16_t>(x);
  }
}

// Per slice: payload length after stripping the bit padding (trailing zeros, then a 0x80
// marker), or -1 when the padding is invalid.  One workgroup per slice.
// Padding strip (reed_solomon.rs:191-203): the last non-zero byte of the data region must
// be 0x80.  The padding sits at the end, so the workgroup scans 4 KiB windows backwards
// with 16-byte loads and stops at the first window holding a non-zero byte.
// Padding strip (reed_solomon.rs:189-202): the last nonzero byte of the slice's data region
// must be the 0x80 marker.  One wave per slice scans back from the end in 1 KiB windows (one
// 16-byte piece per lane, a ballot picks the highest lane with a nonzero byte): a maximum
// slice's marker lies in its last shred, so the wave reads 1 KiB and never synchronises.
__global__ __launch_bounds__(256) void coder_strip_kernel(const uint8_t* __restrict__ cw, uint64_t cw_stride,
                                                          uint32_t data_bytes, uint64_t nslices, int64_t* out) {
  const uint64_t b = static_cast<uint64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= nslices) return;  // wave-uniform
  const uint8_t* d = cw + b * cw_stride;
  const bool a16 = ((reinterpret_cast<uintptr_t>(cw) | cw_stride) & 15) == 0;
  int64_t found = -1;
  for (int64_t hi = data_bytes; hi > 0 && found < 0; hi -= 1024) {  // data_bytes % 16 == 0
    const int64_t i0 = hi - 1024 + 16 * static_cast<int64_t>(lane);
    int32_t last = -1;  // highest nonzero byte of this lane's piece
    if (i0 >= 0) {
      uint32_t w[4];
      if (a16) {
        const uint4 x = *reinterpret_cast<const uint4*>(d + i0);
        w[0] = x.x;
        w[1] = x.y;
        w[2] = x.z;
        w[3] = x.w;
      } else {
        for (int q = 0; q < 4; ++q)
          w[q] = d[i0 + 4 * q] | d[i0 + 4 * q + 1] << 8 | d[i0 + 4 * q + 2] << 16 | static_cast<uint32_t>(d[i0 + 4 * q + 3]) << 24;
      }
      for (int q = 0; q < 4; ++q)
        if (w[q]) last = 4 * q + (31 - __builtin_clz(w[q])) / 8;
    }
    const uint64_t any = __builtin_amdgcn_ballot_w64(last >= 0);
    if (any) {
      const int top = 63 - __builtin_clzll(any);
      const int32_t l = __shfl(last, top);
      found = hi - 1024 + 16 * top + l;
    }
  }
  if (lane == 0) out[b] = (found < 0 || d[found] != 0x80) ? -1 : found;
}

// =====================================================================================
// splitmix64 fill (same generator as oracle/rs_oracle.py splitmix64_bytes)
// =====================================================================================
__global__ __launch_bounds__(256) void fill_splitmix_kernel(uint8_t* dst, uint64_t nblocks, uint64_t words_per_block,
                                                            uint64_t dst_block_stride, uint64_t seed_base) {
  const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t pairs = (words_per_block + 1) / 2;
  if (tid >= nblocks * pairs) return;
  const uint64_t b = tid / pairs;
  const uint64_t w0 = (tid - b * pairs) * 2;
  uint64_t out[2];
  for (int q = 0; q < 2; ++q) {
    uint64_t z = seed_base + b + (w0 + q + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    out[q] = z ^ (z >> 31);
  }
  uint64_t* d = reinterpret_cast<uint64_t*>(dst + b * dst_block_stride) + w0;
  d[0] = out[0];
  if (w0 + 1 < words_per_block) d[1] = out[1];
}

}  // namespace

// ---- launchers ----------------------------------------------------------------------
bool xform_supported(unsigned n) { return n == 32 || n == 64; }

hipError_t launch_xform_lowrate(unsigned n, unsigned j, const XformParams& p, hipStream_t stream) {
  if (p.total_columns == 0) return hipSuccess;
  const uint64_t tiles = (p.total_columns + 63) / 64;
  if (tiles > 0x7FFFFFFFull) return hipErrorInvalidValue;
  const dim3 grid(static_cast<unsigned>(tiles));
  if (n == 32) {
    switch (j) {
      case 0: hipLaunchKernelGGL((xform_kernel<4, 0, 32>), grid, dim3(256), 0, stream, p); break;
      case 1: hipLaunchKernelGGL((xform_kernel<4, 0, 64>), grid, dim3(256), 0, stream, p); break;
      case 2: hipLaunchKernelGGL((xform_kernel<4, 0, 96>), grid, dim3(256), 0, stream, p); break;
      case 3: hipLaunchKernelGGL((xform_kernel<4, 0, 128>), grid, dim3(256), 0, stream, p); break;
      default: return hipErrorInvalidValue;
    }
  } else if (n == 64) {
    switch (j) {
      case 0: return launch_xform64(0, 64, p, stream);
      case 1: return launch_xform64(0, 128, p, stream);
      case 2: return launch_xform64(0, 192, p, stream);
      default: return hipErrorInvalidValue;
    }
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_xform_lowrate_decode(unsigned j, const XformParams& p, hipStream_t stream) {
  if (p.total_columns == 0) return hipSuccess;
  const uint64_t tiles = (p.total_columns + 63) / 64;
  if (tiles > 0x7FFFFFFFull) return hipErrorInvalidValue;
  const dim3 grid(static_cast<unsigned>(tiles));
  switch (j) {
    case 0: hipLaunchKernelGGL((xform_kernel<4, 32, 0>), grid, dim3(256), 0, stream, p); break;
    case 1: hipLaunchKernelGGL((xform_kernel<4, 64, 0>), grid, dim3(256), 0, stream, p); break;
    case 2: hipLaunchKernelGGL((xform_kernel<4, 96, 0>), grid, dim3(256), 0, stream, p); break;
    case 3: hipLaunchKernelGGL((xform_kernel<4, 128, 0>), grid, dim3(256), 0, stream, p); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_decode_x(unsigned W, int pass, const DecodeXParams& p, uint64_t ntiles, hipStream_t stream,
                           uint32_t* which) {
  if (ntiles == 0) return hipSuccess;
  auto rec = [&](uint32_t bit) {
    if (which) *which |= bit;
  };
  if (ntiles > 0x7FFFFFFFull) return hipErrorInvalidValue;
  if (p.k + p.chunk > W || p.m > p.chunk || (p.low_rate && (p.k > p.chunk || p.m + p.chunk > W)))
    return hipErrorInvalidValue;
  const dim3 grid(static_cast<unsigned>(ntiles));
  const bool pl = p.per_lane != 0;
  if (W == 32 && pass == 0) {
    if (pl) hipLaunchKernelGGL((decode_x_kernel<4, true>), grid, dim3(256), 0, stream, p);
    else hipLaunchKernelGGL((decode_x_kernel<4>), grid, dim3(256), 0, stream, p);
    return hipGetLastError();
  }
  // per-lane patterns run on decode_h8 (32-column tiles over every column; the caller's
  // ntiles counts 64-column ones), one pattern per tile on decode_x16
  const uint64_t t32 = (p.total_columns + 31) / 32;
  if (t32 > 0x7FFFFFFFull) return hipErrorInvalidValue;
  const dim3 g32(static_cast<unsigned>(t32));
#define AG_H8(O, PS, DI, DO) hipLaunchKernelGGL((decode_h8_kernel<O, PS, DI, DO>), g32, dim3(512), 0, stream, p)
#define AG_H8T(O) hipLaunchKernelGGL((decode_h8_kernel<O, 0, 0, 0, true>), g32, dim3(512), 0, stream, p)
#define AG_X16(PS, DI, DO) hipLaunchKernelGGL((decode_x16_kernel<PS, DI, DO>), grid, dim3(1024), 0, stream, p)
  if (W == 64 && pass == 0) {
    if (p.rows_w != 64) return hipErrorInvalidValue;
    if (p.tail_bytes) {
      // shards with a T-byte tail chunk (per-lane HighRate chunk 32): decode_h8's TAIL variant
      if (!pl || p.low_rate || p.chunk != 32 || p.tail_bytes >= 64 || p.tail_bytes % 2) return hipErrorInvalidValue;
      if (p.any_k && p.chunks_per_shard == 16) {  // S = 960 + T: the packed decoder, tail column 15
        if (p.fuse) hipLaunchKernelGGL((decode_pk_kernel<-1, true>), g32, dim3(512), 0, stream, p);
        else hipLaunchKernelGGL((decode_pk_kernel<1, true>), g32, dim3(512), 0, stream, p);
        rec(p.fuse ? kDxPkFused : kDxPk);
        return hipGetLastError();
      }
      if (p.fuse) AG_H8T(-1);
      else AG_H8T(1);
      rec(p.fuse ? kDxH8Fused : kDxH8);
      return hipGetLastError();
    }
    const bool packed = pl && p.any_k && p.chunks_per_shard == 16 && (p.low_rate || p.chunk == 32);
    // fused coding restore: the caller's patterns restore absent coding positions too and skip
    // those slices in the re-encode, which decode_pk<-1> and the full-FFT decode_h8<-1> honour
    // (per-lane HighRate chunk 32 only)
    if (p.fuse && (p.low_rate || !pl || p.chunk != 32)) return hipErrorInvalidValue;
    if (packed) {
      if (p.low_rate) hipLaunchKernelGGL((decode_pk_kernel<0>), g32, dim3(512), 0, stream, p);
      else if (p.fuse) hipLaunchKernelGGL((decode_pk_kernel<-1>), g32, dim3(512), 0, stream, p);
      else hipLaunchKernelGGL((decode_pk_kernel<1>), g32, dim3(512), 0, stream, p);
      rec(p.fuse ? kDxPkFused : kDxPk);
    } else if (!pl) {
      AG_X16(0, 0, 0);
      rec(kDxX16);
    } else if (p.low_rate) {
      AG_H8(0, 0, 0, 0);
      rec(kDxH8);
    } else if (p.chunk == 32 && !p.fuse) {
      AG_H8(1, 0, 0, 0);
      rec(kDxH8);
    } else {
      AG_H8(-1, 0, 0, 0);  // (fused: restored positions in both window halves)
      rec(p.fuse ? kDxH8Fused : kDxH8);
    }
  } else if (W == 128 && (pass == 1 || pass == 2)) {
    // the originals must lie in one window half: LowRate k <= 64 (half 0); HighRate chunk 64
    // (half 1).  Both passes of a decode come from the same kernel family.
    if (p.rows_w != 128 || (p.low_rate ? p.k > 64 : p.chunk != 64)) return hipErrorInvalidValue;
    if (pl) {
      // LowRate: outputs (originals < 32 when k <= 32) in half 0; HighRate: half 1
      if (p.low_rate && p.k <= 32) {
        if (pass == 1) AG_H8(0, 1, 64, 0);
        else AG_H8(0, 2, 0, 0);
      } else if (p.low_rate) {
        if (pass == 1) AG_H8(-1, 1, 64, 0);
        else AG_H8(-1, 2, 0, 0);
      } else {
        if (pass == 1) AG_H8(-1, 1, 0, 64);
        else AG_H8(-1, 2, 64, 64);
      }
    } else if (p.low_rate) {  // outputs in half 0
      if (pass == 1) AG_X16(1, 64, 0);
      else AG_X16(2, 0, 0);
    } else {                  // outputs in half 1
      if (pass == 1) AG_X16(1, 0, 64);
      else AG_X16(2, 64, 64);
    }
  } else {
    return hipErrorInvalidValue;
  }
#undef AG_H8
#undef AG_H8T
#undef AG_X16
  return hipGetLastError();
}

// W = 128 windows: m6[pat] = {erased lo, hi, present lo, hi, restored lo, hi} (position bits
// 0..63, 64..127); rows [pat][128] polynomial-basis constants (decode_rows poly form).
__global__ __launch_bounds__(256) void decode_rows128_kernel(const uint64_t* __restrict__ m6, uint32_t npat,
                                                            const uint16_t* __restrict__ log_t,
                                                            const uint16_t* __restrict__ exp_t, uint32_t* rows) {
  const uint64_t pat = static_cast<uint64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (pat >= npat) return;  // wave-uniform
  const int lane = threadIdx.x & 63;
  const uint64_t* m = m6 + 6 * pat;
  // decode_rows' Walsh route at N = 128: positions lane (v0) and lane + 64 (v1)
  uint32_t l0 = lane ? log_t[lane] : 0u, l1 = log_t[lane + 64];
  walsh128(l0, l1, lane);
  l0 = m65535_mul(l0, 512u);  // 128^-1 = 512
  l1 = m65535_mul(l1, 512u);
  uint32_t i0 = static_cast<uint32_t>((m[0] >> lane) & 1), i1 = static_cast<uint32_t>((m[1] >> lane) & 1);
  walsh128(i0, i1, lane);
  uint32_t a0 = m65535_mul(l0, i0), a1 = m65535_mul(l1, i1);
  walsh128(a0, a1, lane);
  static_for<2>([&](auto H) {
    constexpr int h = decltype(H)::value;
    const bool is_in = (m[2 + h] >> lane) & 1, is_out = (m[4 + h] >> lane) & 1;
    if (is_in || is_out) rows[pat * 128 + h * 64 + lane] = dev::to_poly(exp_t[locator_log(h ? a1 : a0, is_in)]);
  });
}

hipError_t launch_decode_rows128(const uint64_t* m6, uint32_t npat, const GfDeviceTables& t, uint32_t* rows,
                                 hipStream_t stream) {
  if (npat == 0) return hipSuccess;
  hipLaunchKernelGGL(decode_rows128_kernel, dim3((npat + 3) / 4), dim3(256), 0, stream, m6, npat, t.log, t.exp, rows);
  return hipGetLastError();
}

hipError_t launch_decode_rows(const uint64_t* emask, const uint64_t* pmask, uint32_t npat, uint32_t W,
                              const GfDeviceTables& t, uint32_t* rows, bool poly, hipStream_t stream) {
  if (npat == 0) return hipSuccess;
  if (W > 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(decode_rows_kernel, dim3((npat + 3) / 4), dim3(256), 0, stream, emask, pmask, npat, W, t.log, t.exp,
                     rows, poly ? 1u : 0u);
  return hipGetLastError();
}

hipError_t launch_encode_mc(unsigned chunk, const XformParams& p, hipStream_t stream) {
  if (p.total_columns == 0) return hipSuccess;
  if (p.n_in > static_cast<uint32_t>(kMcMaxK) || p.n_out > chunk) return hipErrorInvalidValue;
  const uint64_t tiles = (p.total_columns + kXfLanes - 1) / kXfLanes;
  const uint64_t groups = (tiles + 3) / 4;
  if (groups > 0x7FFFFFFFull) return hipErrorInvalidValue;
  const dim3 grid(static_cast<unsigned>(groups));
  switch (chunk) {
    case 1: hipLaunchKernelGGL((encode_mc_kernel<1>), grid, dim3(256), 0, stream, p); break;
    case 2: hipLaunchKernelGGL((encode_mc_kernel<2>), grid, dim3(256), 0, stream, p); break;
    case 4: hipLaunchKernelGGL((encode_mc_kernel<4>), grid, dim3(256), 0, stream, p); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_decode_syn(unsigned chunk, const DecodeSynParams& p, hipStream_t stream) {
  if (p.ntiles == 0) return hipSuccess;
  if (p.k > static_cast<uint32_t>(kMcMaxK)) return hipErrorInvalidValue;
  const uint64_t groups = (p.ntiles + 3) / 4;
  if (groups > 0x7FFFFFFFull) return hipErrorInvalidValue;
  const dim3 grid(static_cast<unsigned>(groups));
  switch (chunk) {
    case 1: hipLaunchKernelGGL((decode_syn_kernel<1>), grid, dim3(256), 0, stream, p); break;
    case 2: hipLaunchKernelGGL((decode_syn_kernel<2>), grid, dim3(256), 0, stream, p); break;
    case 4: hipLaunchKernelGGL((decode_syn_kernel<4>), grid, dim3(256), 0, stream, p); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ---- per-call server --------------------------------------------------------------
// One workgroup of xform8's shape, resident between per-slice calls (LatencyMailbox in
// rs_launch.hpp).  Thread 0 polls the doorbell with system-scope loads (vector memory; the
// host memory is fine-grained, so nothing is cached across jobs) and every wave invalidates
// its caches at job start; each wave releases its stores at system scope before thread 0
// publishes done.  Every wave leaves the loop together on kJobQuit or the idle timeout.
__device__ __forceinline__ uint32_t sys_load(const uint32_t* a) {
  return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ __launch_bounds__(512, 1) void latency_server_kernel(LatencyMailbox* mb, uint64_t idle_ticks,
                                                                const uint16_t* log_t) {
  __shared__ uint4 lds[16 * 4 * kXfLanes];
  __shared__ X8Flags flags;
  constexpr unsigned kXw = sizeof(XformParams) / 4, kDw = sizeof(DecodeXParams) / 4;
  __shared__ __attribute__((aligned(16))) uint32_t job[kXw];    // the transform jobs' XformParams
  __shared__ __attribute__((aligned(16))) uint32_t jobd[kDw];   // kJobDecodePk's DecodeXParams
  __shared__ uint64_t mask;
  __shared__ uint32_t cmd, reload;
  __shared__ PkShared pk;                 // kJobDecodePk: the tile's lists
  __shared__ uint64_t pk_mask[4];         // slice 0: present, restored; slice 1: none
  __shared__ PkLocTables loc;             // kJobDecodePk: the locator's tables
  static_assert(sizeof(XformParams) % 4 == 0 && kXw <= 512, "params copy");
  static_assert(sizeof(DecodeXParams) % 4 == 0 && kDw <= 512, "decode params copy");
  // the locator tables, once per launch: log x (x < 64) from the device table, a^i and a^(256 i)
  // by square-and-multiply
  if (threadIdx.x < 64) loc.log64[threadIdx.x] = log_t[threadIdx.x];
  if (threadIdx.x < 256) {
    uint32_t b = 2, bh = 2;  // a^(2^i) and a^(256 * 2^i) at step i
    for (int q = 0; q < 8; ++q) bh = poly_mul(bh, bh);
    uint32_t lo = 1, hi = 1;
    for (int i = 0; i < 8; ++i) {
      if ((threadIdx.x >> i) & 1) {
        lo = poly_mul(lo, b);
        hi = poly_mul(hi, bh);
      }
      b = poly_mul(b, b);
      bh = poly_mul(bh, bh);
    }
    loc.apow_lo[threadIdx.x] = static_cast<uint16_t>(lo);
    loc.apow_hi[threadIdx.x] = static_cast<uint16_t>(hi);
  }
  uint32_t last = 0;
  uint64_t t_job = 0, t_kind = 0, t_par = 0, t_tile = 0;  // thread 0: phase boundaries of the job
  uint32_t have_p = 0, have_dp = 0;  // thread 0: versions of the parameter copies in LDS (0: none)
  if (threadIdx.x == 0) {
    last = sys_load(&mb->done);
    __hip_atomic_store(&mb->alive, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  for (;;) {
    if (threadIdx.x == 0) {
      const uint64_t t0 = wall_clock64();
      uint32_t kind = kJobQuit;
      for (;;) {
        const uint32_t d = __hip_atomic_load(&mb->doorbell, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        if (d != last) {
          t_job = wall_clock64();
          last = d;
          // one round trip: the job's header words are loaded together (no load depends on another)
          kind = sys_load(&mb->kind);
          const uint32_t* m = reinterpret_cast<const uint32_t*>(&mb->mask);
          const uint32_t m0 = sys_load(m), m1 = sys_load(m + 1), ps = sys_load(&mb->p_seq), ds = sys_load(&mb->dp_seq);
          mask = static_cast<uint64_t>(m0) | static_cast<uint64_t>(m1) << 32;
          const uint32_t seq = kind == kJobDecodePk ? ds : ps;
          uint32_t& have = kind == kJobDecodePk ? have_dp : have_p;
          reload = seq != have ? 1u : 0u;
          have = seq;
          t_kind = wall_clock64();
          break;
        }
        if (wall_clock64() - t0 > idle_ticks) break;
        __builtin_amdgcn_s_sleep(2);
      }
      cmd = kind;
    }
    __syncthreads();
    const uint32_t kind = __builtin_amdgcn_readfirstlane(cmd);
    if (kind >= kJobQuit) break;
    if (__builtin_amdgcn_readfirstlane(reload)) {
      if (kind == kJobDecodePk) {
        if (threadIdx.x < kDw) jobd[threadIdx.x] = sys_load(reinterpret_cast<const uint32_t*>(&mb->dp) + threadIdx.x);
      } else if (threadIdx.x < kXw) {
        job[threadIdx.x] = sys_load(reinterpret_cast<const uint32_t*>(&mb->p) + threadIdx.x);
      }
    }
    if (threadIdx.x >= 128 && threadIdx.x < 144) reinterpret_cast<uint32_t*>(&flags)[threadIdx.x - 128] = 0;
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: no stale input bytes in this CU's caches
    if (threadIdx.x == 0) t_par = wall_clock64();
    if (kind == kJobDecodePk) {
      // the tile reads its parameters from the LDS copy: a private copy would be indexed by the
      // rec / orig selects and land in scratch
      DecodeXParams& dp = *reinterpret_cast<DecodeXParams*>(jobd);
      if (threadIdx.x == 0) {
        pk_mask[0] = mask;   // present positions
        pk_mask[1] = ~mask;  // restored: every absent data and coding position
        pk_mask[2] = pk_mask[3] = 0;
        dp.pmask = pk_mask;
      }
      __syncthreads();
      if (dp.tail_bytes) decode_pk_tile<-1, true, true>(dp, 0, lds, &flags, pk, &loc);  // S = 960 + T, T < 64
      else decode_pk_tile<-1, true>(dp, 0, lds, &flags, pk, &loc);
      if (threadIdx.x == 0) t_tile = wall_clock64();
      __threadfence_system();
      __syncthreads();
      if (threadIdx.x == 0) {
        const uint64_t t_end = wall_clock64();
        __hip_atomic_store(&mb->phase_ticks[0], static_cast<uint32_t>(t_kind - t_job), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&mb->phase_ticks[1], static_cast<uint32_t>(t_par - t_kind), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&mb->phase_ticks[2], static_cast<uint32_t>(t_tile - t_par), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&mb->phase_ticks[3], static_cast<uint32_t>(t_end - t_tile), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&mb->job_ticks, t_end - t_job, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&mb->done, last, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      continue;
    }
    XformParams p;
    uint32_t* pw = reinterpret_cast<uint32_t*>(&p);
    for (unsigned i = 0; i < sizeof(XformParams) / 4; ++i) pw[i] = __builtin_amdgcn_readfirstlane(job[i]);
    p.out_mask = kind == kJobEncode32 ? nullptr : &mask;
    p.pattern_per_block = 0;
    if (kind == kJobEncode32)
      xform8_tile<32, 0>(p, 0, lds, &flags);
    else if (kind == kJobDecode32)
      xform8_tile<0, 32>(p, 0, lds, &flags);
    else
      xform8_tile<0, 32, true>(p, 0, lds, &flags);
    if (threadIdx.x == 0) t_tile = wall_clock64();
    __threadfence_system();  // this wave's stores reach the host before done is published
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint64_t t_end = wall_clock64();
      __hip_atomic_store(&mb->phase_ticks[0], static_cast<uint32_t>(t_kind - t_job), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&mb->phase_ticks[1], static_cast<uint32_t>(t_par - t_kind), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&mb->phase_ticks[2], static_cast<uint32_t>(t_tile - t_par), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&mb->phase_ticks[3], static_cast<uint32_t>(t_end - t_tile), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&mb->job_ticks, t_end - t_job, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&mb->done, last, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  if (threadIdx.x == 0) __hip_atomic_store(&mb->alive, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_latency_server(LatencyMailbox* mb_dev, uint64_t idle_ticks, const uint16_t* log_t,
                                 hipStream_t stream) {
  if (!log_t) return hipErrorInvalidValue;
  hipLaunchKernelGGL(latency_server_kernel, dim3(1), dim3(512), 0, stream, mb_dev, idle_ticks, log_t);
  return hipGetLastError();
}

hipError_t launch_xform(XformKind kind, const XformParams& p, hipStream_t stream) {
  if (p.total_columns == 0) return hipSuccess;
  const uint64_t groups = (p.total_columns + kXfLanes - 1) / kXfLanes;
  if (groups > 0x7FFFFFFFull) return hipErrorInvalidValue;
  const dim3 grid(static_cast<unsigned>(groups));
  switch (kind) {
    // 32-point: xform<4> encodes (it runs at its load/store skeleton's speed), xform8
    // reconstructs (half the exposed arithmetic per wave: -8% time), with the pruned FFT when
    // every restored original is < 16.
    case XformKind::kEncode32:
      if (p.tail_bytes) {  // shards ending in a split tail chunk: the TAIL kernels, same dispatch
        if (encode32_kernel(p) == kEkXform8)
          hipLaunchKernelGGL((xform8_kernel<32, 0, false, 1>), grid, dim3(512), 0, stream, p);
        else
          hipLaunchKernelGGL((xform_kernel<4, 32, 0, 1>), grid, dim3(256), 0, stream, p);
        break;
      }
      // batches of fewer tiles than CUs (a single slice per call: one tile) are latency-bound:
      // xform8 spreads a tile's transform over 8 waves of 4 slots, half xform<4>'s instruction
      // stream per wave.  Shards of 8 and 16 KiB (2 or 4 tiles per shard) also take xform8:
      // xform<4> drops to 5.49-5.77 TB/s there while xform8 runs 5.93-6.18, and xform<4> wins
      // by 0.03-0.31 TB/s at every other measured size (profiles/r04_encode_kernel_grid.txt; a
      // copy with either kernel's load/store skeleton shows no such dip, tools/membench/
      // membench7.hip, so it is the kernel's access order against that stride)
      if (encode32_kernel(p) == kEkXform8)
        hipLaunchKernelGGL((xform8_kernel<32, 0>), grid, dim3(512), 0, stream, p);
      else
        hipLaunchKernelGGL((xform_kernel<4, 32, 0>), grid, dim3(256), 0, stream, p);
      break;
    case XformKind::kDecode32:
      // (xform<4> with the same skipped conversions: random-16 reconstruct 5.37 TB/s against
      // xform8's 5.43-5.51, one box)
      if (p.tail_bytes) {
        if (p.out_low_half)
          hipLaunchKernelGGL((xform8_kernel<0, 32, true, 1>), grid, dim3(512), 0, stream, p);
        else
          hipLaunchKernelGGL((xform8_kernel<0, 32, false, 1>), grid, dim3(512), 0, stream, p);
        break;
      }
      if (p.out_low_half)
        hipLaunchKernelGGL((xform8_kernel<0, 32, true>), grid, dim3(512), 0, stream, p);
      else
        hipLaunchKernelGGL((xform8_kernel<0, 32>), grid, dim3(512), 0, stream, p);
      break;
    // 64-point: xform_h8 (32-column tiles, lane-linear I/O, two workgroups per CU)
    case XformKind::kEncode64:
      return launch_xform64(64, 0, p, stream);
    case XformKind::kDecode64:
      return launch_xform64(0, 64, p, stream);
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_generic_encode(const GenericEncodeParams& p, hipStream_t stream) {
  const uint64_t n = p.nblocks * p.nsym;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(generic_encode_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, stream, p);
  return hipGetLastError();
}

hipError_t launch_generic_decode(const GenericDecodeParams& p, hipStream_t stream) {
  const uint64_t n = p.nblocks * p.nsym;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(generic_decode_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, stream, p);
  return hipGetLastError();
}

hipError_t launch_locator(const uint8_t* erased, uint32_t npatterns, uint32_t W, uint32_t fill_from,
                          const uint16_t* log_walsh, uint16_t* loc, hipStream_t stream) {
  if (npatterns == 0) return hipSuccess;
  hipLaunchKernelGGL(locator_kernel, dim3(npatterns), dim3(1024), 0, stream, erased, W, fill_from, log_walsh, loc);
  return hipGetLastError();
}

hipError_t launch_coder_pad(const uint8_t* payload, uint64_t payload_stride, const uint32_t* lens, uint8_t* cw,
                            uint64_t cw_stride, uint32_t data_bytes, uint64_t nslices, hipStream_t stream) {
  if (data_bytes % 16) return hipErrorInvalidValue;
  if (nslices == 0 || data_bytes == 0) return hipSuccess;
  if (nslices > 0x7FFFFFFFull) return hipErrorInvalidValue;
  const uint64_t groups = payload ? nslices : (nslices + 3) / 4;
  hipLaunchKernelGGL(coder_pad_kernel, dim3(static_cast<unsigned>(groups)), dim3(256), 0, stream, payload,
                     payload_stride, lens, cw, cw_stride, data_bytes, nslices);
  return hipGetLastError();
}

hipError_t launch_restride(const uint8_t* src, uint64_t src_block_stride, uint64_t src_shard_stride, uint8_t* dst,
                           uint64_t dst_block_stride, uint64_t dst_shard_stride, uint32_t S, uint32_t nshards,
                           uint64_t nblocks, bool unpack, const uint64_t* mask, bool mask_per_block,
                           hipStream_t stream) {
  RestrideParams p{};
  p.src = src;
  p.src_block_stride = src_block_stride;
  p.src_shard_stride = src_shard_stride;
  p.dst = dst;
  p.dst_block_stride = dst_block_stride;
  p.dst_shard_stride = dst_shard_stride;
  p.S = S;
  p.Sp = (S + 63) / 64 * 64;
  p.nshards = nshards;
  p.unpack = unpack ? 1u : 0u;
  p.nblocks = nblocks;
  p.mask = mask;
  p.mask_per_block = mask_per_block ? 1u : 0u;
  const uint64_t per_block = static_cast<uint64_t>(nshards) * (p.Sp / 16);
  if (per_block == 0 || nblocks == 0) return hipSuccess;
  const uint64_t groups = (per_block * nblocks + 255) / 256;
  if (per_block > 0x7FFFFFFFull || groups > 0x7FFFFFFFull) return hipErrorInvalidValue;
  // tail-only unpack to an even destination (S even: the sizes are whole symbols)
  if (unpack && S > 0 && S < 64 && S % 2 == 0 &&
      ((reinterpret_cast<uintptr_t>(dst) | dst_block_stride | dst_shard_stride) & 1) == 0) {
    hipLaunchKernelGGL(unpack_tail_kernel, dim3(static_cast<unsigned>(groups)), dim3(256), 0, stream, p);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(restride_kernel, dim3(static_cast<unsigned>(groups)), dim3(256), 0, stream, p);
  return hipGetLastError();
}

hipError_t launch_coder_strip(const uint8_t* cw, uint64_t cw_stride, uint32_t data_bytes, uint64_t nslices,
                              int64_t* out, hipStream_t stream) {
  if (nslices == 0) return hipSuccess;
  if (data_bytes % 16) return hipErrorInvalidValue;
  const uint64_t groups = (nslices + 3) / 4;  // one wave per slice
  if (groups > 0x7FFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(coder_strip_kernel, dim3(static_cast<unsigned>(groups)), dim3(256), 0, stream, cw, cw_stride,
                     data_bytes, nslices, out);
  return hipGetLastError();
}

hipError_t launch_fill_splitmix(uint8_t* dst, uint64_t nblocks, uint64_t block_bytes, uint64_t dst_block_stride,
                                uint64_t seed_base, hipStream_t stream) {
  if (block_bytes % 8) return hipErrorInvalidValue;
  const uint64_t words = block_bytes / 8, pairs = (words + 1) / 2;
  if (nblocks == 0 || pairs == 0) return hipSuccess;
  if (pairs > (uint64_t{1} << 30)) return hipErrorInvalidValue;
  // a dispatch's grid is at most 2^32 - 1 work-items (HSA packet): launches of at most 2^30
  // threads' worth of whole blocks (BASELINE configs[4]'s 64 GiB stream at N = 1 is 2^32 pairs)
  const uint64_t per = std::max<uint64_t>(1, (uint64_t{1} << 30) / pairs);
  for (uint64_t b0 = 0; b0 < nblocks; b0 += per) {
    const uint64_t nb = std::min(per, nblocks - b0), n = nb * pairs;
    hipLaunchKernelGGL(fill_splitmix_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, stream,
                       dst + b0 * dst_block_stride, nb, words, dst_block_stride, seed_base + b0);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace ag
