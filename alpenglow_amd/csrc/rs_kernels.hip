// HIP kernels for the Reed-Solomon shredder path (gfx950 / CDNA4).
//
// What they replace: the reed-solomon-simd 3.1.0 calls inside ReedSolomonCoder
// (/root/reference/src/shredder/reed_solomon.rs:96-125 encode, :150-180 decode,
// :211-231 re-encode).  Arithmetic: GF(2^16) Leopard additive FFT.
//
// Kernels
//   xform32_kernel    bitsliced IFFT-32 + FFT-32 over one 32-point block; HighRate encode
//                     (k <= m = 32) and decode-from-a-full-recovery-set.  HBM-bound.
//   generic_*         table-driven crate algorithm for every geometry (correctness path:
//                     multi-chunk HighRate, LowRate, exact decode with any erasures).
//   locator_kernel    erasure-locator logs (crate eval_poly: FWHT over 65536 in LDS).
//   fill_splitmix     synthetic input blocks (bench / tests), generated on the device.
#include <hip/hip_runtime.h>

#include "rs_device.hpp"
#include "rs_launch.hpp"

namespace ag {
namespace {

using dev::static_for;

// =====================================================================================
// xform32: 4 waves x 64 lanes; lane = one 64-byte column (32 symbols) of one block,
// each lane owns 8 of the 32 shards in each of three passes:
//   pass A  (wave w: shards 8w+t)      IFFT layers dist 1, 2, 4      (skew delta DIN)
//   pass B  (wave w: shards w+4t)      IFFT dist 8, 16; FFT dist 16, 8 (DIN / DOUT)
//   pass C  (wave w: shards 8w+t)      FFT layers dist 4, 2, 1       (skew delta DOUT)
// Shards change owner between passes through LDS (2 rounds x 64 KiB per exchange).
// Skew index of a layer of distance d on the group starting at g: g + d + delta - 1.
// =====================================================================================

constexpr int kXfLanes = 64;
constexpr int kXfLdsSlots = 16;  // 16 shards x 16 planes x 64 lanes x 4 B = 64 KiB

using Regs8 = uint32_t[8][16];

// butterfly whose skew index is BASE + 8 * wave (wave-uniform, runtime)
template <int BASE, bool INV>
__device__ __forceinline__ void bfly_w(int wave, uint32_t* x, uint32_t* y) {
#ifdef AG_XF_DIAG_ONE_ROLE
  wave = 0;  // diagnostic build only: every wave runs role 0's code (wrong output)
#endif
  switch (wave) {
    case 0: if constexpr (INV) dev::ifft_bfly<BASE>(x, y); else dev::fft_bfly<BASE>(x, y); break;
    case 1: if constexpr (INV) dev::ifft_bfly<BASE + 8>(x, y); else dev::fft_bfly<BASE + 8>(x, y); break;
    case 2: if constexpr (INV) dev::ifft_bfly<BASE + 16>(x, y); else dev::fft_bfly<BASE + 16>(x, y); break;
    default: if constexpr (INV) dev::ifft_bfly<BASE + 24>(x, y); else dev::fft_bfly<BASE + 24>(x, y); break;
  }
}
template <int DIN>
__device__ __forceinline__ void xf32_pass_a(int wave, Regs8& r) {
  static_for<4>([&](auto I) {  // dist 1
    constexpr int t = 2 * decltype(I)::value;
    bfly_w<t + 1 + DIN - 1, true>(wave, r[t], r[t + 1]);
  });
  static_for<4>([&](auto I) {  // dist 2
    constexpr int g = 4 * (decltype(I)::value >> 1);
    constexpr int u = g + (decltype(I)::value & 1);
    bfly_w<g + 2 + DIN - 1, true>(wave, r[u], r[u + 2]);
  });
  static_for<4>([&](auto I) {  // dist 4
    constexpr int u = decltype(I)::value;
    bfly_w<4 + DIN - 1, true>(wave, r[u], r[u + 4]);
  });
}

// Slot t holds shard w + 4t: bit 2 <- t0, bit 3 <- t1, bit 4 <- t2.  The layers touched
// here have group starts that depend only on bit 4, so the code is wave-independent.
template <int DIN, int DOUT>
__device__ __forceinline__ void xf32_pass_b(Regs8& r) {
  constexpr int kPairs8[4] = {0, 1, 4, 5};
  static_for<4>([&](auto I) {  // IFFT dist 8 (bit 3)
    constexpr int t = kPairs8[decltype(I)::value];
    dev::ifft_bfly<16 * (t >> 2) + 8 + DIN - 1>(r[t], r[t + 2]);
  });
  static_for<4>([&](auto I) {  // IFFT dist 16 (bit 4)
    constexpr int t = decltype(I)::value;
    dev::ifft_bfly<16 + DIN - 1>(r[t], r[t + 4]);
  });
  static_for<4>([&](auto I) {  // FFT dist 16
    constexpr int t = decltype(I)::value;
    dev::fft_bfly<16 + DOUT - 1>(r[t], r[t + 4]);
  });
  static_for<4>([&](auto I) {  // FFT dist 8
    constexpr int t = kPairs8[decltype(I)::value];
    dev::fft_bfly<16 * (t >> 2) + 8 + DOUT - 1>(r[t], r[t + 2]);
  });
}

template <int DOUT>
__device__ __forceinline__ void xf32_pass_c(int wave, Regs8& r) {
  static_for<4>([&](auto I) {  // dist 4
    constexpr int u = decltype(I)::value;
    bfly_w<4 + DOUT - 1, false>(wave, r[u], r[u + 4]);
  });
  static_for<4>([&](auto I) {  // dist 2
    constexpr int g = 4 * (decltype(I)::value >> 1);
    constexpr int u = g + (decltype(I)::value & 1);
    bfly_w<g + 2 + DOUT - 1, false>(wave, r[u], r[u + 2]);
  });
  static_for<4>([&](auto I) {  // dist 1
    constexpr int t = 2 * decltype(I)::value;
    bfly_w<t + 1 + DOUT - 1, false>(wave, r[t], r[t + 1]);
  });
}

__device__ __forceinline__ void lds_put(uint4* lds, int slot, int lane, const uint32_t* v) {
  static_for<4>([&](auto Q) {
    constexpr int q = decltype(Q)::value;
    lds[(slot * 4 + q) * kXfLanes + lane] = make_uint4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
  });
}
__device__ __forceinline__ void lds_get(const uint4* lds, int slot, int lane, uint32_t* v) {
  static_for<4>([&](auto Q) {
    constexpr int q = decltype(Q)::value;
    const uint4 x = lds[(slot * 4 + q) * kXfLanes + lane];
    v[4 * q] = x.x;
    v[4 * q + 1] = x.y;
    v[4 * q + 2] = x.z;
    v[4 * q + 3] = x.w;
  });
}

// ---- tile I/O -------------------------------------------------------------------
// A tile is 64 consecutive 64-byte chunks (global chunk index g = 64 * tile + c; chunk g
// is chunk g % C of block g / C, C = chunks per shard).  Each of a lane's four 16-byte
// loads per shard is one slice of a lane-linear 1 KiB wave access: instruction q covers
// chunks 16q .. 16q+15 of the tile; lane l < 32 takes low-byte quarter (l & 1) of chunk
// 16q + (l >> 1), lane l + 32 the matching high-byte quarter.  One v_permlane32_swap per
// register pair then gives every lane the low AND high bytes of 32 symbols (2 chunks x 16
// symbols): lane l < 32 keeps chunks q = 0, 1, lane l + 32 chunks q = 2, 3.
struct TileIO {
  uint64_t off[4];  // byte offset of this lane's 16-byte piece of shard 0, per instruction q
  uint64_t blk[4];  // block of chunk q (for the per-block store mask)
  uint32_t valid;   // bit q: chunk q exists (idle pieces re-read the last chunk, never store)
};
__device__ __forceinline__ TileIO tile_io(const XformParams& p, uint64_t tile, int lane, uint64_t block_stride) {
  TileIO io;
  io.valid = 0;
  const uint32_t quarter = ((lane >> 5) << 1) | (lane & 1);
  static_for<4>([&](auto Q) {
    constexpr int q = decltype(Q)::value;
    const uint64_t g = tile * kXfLanes + 16 * q + ((lane & 31) >> 1);
    const bool ok = g < p.total_columns;
    const uint64_t gc = ok ? g : p.total_columns - 1;
    const uint64_t blk = gc / p.chunks_per_shard;
    io.blk[q] = blk;
    io.off[q] = blk * block_stride + (gc - blk * p.chunks_per_shard) * 64 + 16 * quarter;
    io.valid |= ok ? (1u << q) : 0u;
  });
  return io;
}

// lanes l and l + 32 exchange register halves (see TileIO); an involution
__device__ __forceinline__ void swap_halves(uint32_t* v) {
  static_for<8>([&](auto K) {
    constexpr int k = decltype(K)::value;
    const auto r = __builtin_amdgcn_permlane32_swap(v[k], v[k + 8], false, false);
    v[k] = r[0];
    v[k + 8] = r[1];
  });
}

// Raw 16-byte pieces of this wave's pass-A shards 8*wave + t (before swap / transpose).
__device__ __forceinline__ void xf32_load_raw(const XformParams& p, const TileIO& io, int wave, Regs8& raw) {
  static_for<8>([&](auto T) {
    constexpr int t = decltype(T)::value;
    const uint32_t s = 8 * wave + t;  // wave-uniform condition
    if (s < p.n_in) {
      const uint8_t* base = p.in + s * p.in_shard_stride;
      static_for<4>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        const uint4 x = *reinterpret_cast<const uint4*>(base + io.off[q]);
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

// Planes -> bytes -> lane-linear pieces, stored where the input pieces were read.
__device__ __forceinline__ void store_shard(uint8_t* __restrict__ base, const TileIO& io, uint32_t qmask,
                                            const uint32_t* planes) {
  uint32_t v[16];
  static_for<16>([&](auto P) {
    constexpr int i = decltype(P)::value;
    v[i] = planes[i];
  });
  dev::transpose8(v);
  dev::transpose8(v + 8);
  swap_halves(v);
  static_for<4>([&](auto Q) {
    constexpr int q = decltype(Q)::value;
    if (qmask & (1u << q))
      *reinterpret_cast<uint4*>(base + io.off[q]) = make_uint4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
  });
}

// LDS exchange between passes.  Pass A/C slot t of wave w holds shard 8w+t; pass B slot
// t' of wave w' holds shard w'+4t' (so A-slot t of wave w <-> B-slot 2w+(t>>2) of wave t&3).
// ROUNDS = 2: each round moves 4 slots per wave through 64 KiB.  (ROUNDS = 4, 32 KiB per
// round with wave-dependent slot pairing, is kept for experiments: it spills, because the
// slot indices then depend on the runtime wave id.)
template <int ROUNDS>
__device__ __forceinline__ void xf32_exchange_ab(int wave, int lane, uint4* lds, Regs8& ra, Regs8& rb) {
  if constexpr (ROUNDS == 2) {
    static_for<2>([&](auto Rho) {
      constexpr int rho = decltype(Rho)::value;
      static_for<4>([&](auto U) {
        constexpr int u = decltype(U)::value;
        lds_put(lds, 4 * wave + u, lane, ra[4 * rho + u]);
      });
      __syncthreads();
      static_for<4>([&](auto W2) {
        constexpr int w2 = decltype(W2)::value;
        lds_get(lds, 4 * w2 + wave, lane, rb[2 * w2 + rho]);
      });
      __syncthreads();
    });
  } else {
    static_for<4>([&](auto Rho) {
      constexpr int rho = decltype(Rho)::value;
      // writer w sends A-slots t0, t0+4 with t0 = (w+rho)&3 to wave t0
      static_for<4>([&](auto Wc) {
        constexpr int w = decltype(Wc)::value;
        if (wave == w) {
          constexpr int t0 = (w + rho) & 3;
          lds_put(lds, 2 * w + 0, lane, ra[t0]);
          lds_put(lds, 2 * w + 1, lane, ra[t0 + 4]);
        }
      });
      __syncthreads();
      // reader w' receives from writer w = (w'-rho)&3 into B-slots 2w, 2w+1
      static_for<4>([&](auto Wc) {
        constexpr int wr = decltype(Wc)::value;
        if (wave == wr) {
          constexpr int w = (wr - rho) & 3;
          lds_get(lds, 2 * w + 0, lane, rb[2 * w + 0]);
          lds_get(lds, 2 * w + 1, lane, rb[2 * w + 1]);
        }
      });
      __syncthreads();
    });
  }
}

template <int ROUNDS>
__device__ __forceinline__ void xf32_exchange_bc(int wave, int lane, uint4* lds, Regs8& rb, Regs8& ra) {
  if constexpr (ROUNDS == 2) {
    static_for<2>([&](auto Rho) {
      constexpr int rho = decltype(Rho)::value;
      static_for<4>([&](auto W2) {
        constexpr int w2 = decltype(W2)::value;
        lds_put(lds, 4 * w2 + wave, lane, rb[2 * w2 + rho]);
      });
      __syncthreads();
      static_for<4>([&](auto U) {
        constexpr int u = decltype(U)::value;
        lds_get(lds, 4 * wave + u, lane, ra[4 * rho + u]);
      });
      __syncthreads();
    });
  } else {
    static_for<4>([&](auto Rho) {
      constexpr int rho = decltype(Rho)::value;
      // writer w' sends B-slots 2w, 2w+1 to pass-C wave w = (w'-rho)&3
      static_for<4>([&](auto Wc) {
        constexpr int wp = decltype(Wc)::value;
        if (wave == wp) {
          constexpr int w = (wp - rho) & 3;
          lds_put(lds, 2 * wp + 0, lane, rb[2 * w + 0]);
          lds_put(lds, 2 * wp + 1, lane, rb[2 * w + 1]);
        }
      });
      __syncthreads();
      // reader w receives from w' = (w+rho)&3 into C-slots w', w'+4
      static_for<4>([&](auto Wc) {
        constexpr int w = decltype(Wc)::value;
        if (wave == w) {
          constexpr int wp = (w + rho) & 3;
          lds_get(lds, 2 * wp + 0, lane, ra[wp]);
          lds_get(lds, 2 * wp + 1, lane, ra[wp + 4]);
        }
      });
      __syncthreads();
    });
  }
}

// Store predicate of this wave's shard s for the four chunk slices of the tile: chunk
// exists and, with a mask, bit s of its block's pattern word is set.
__device__ __forceinline__ uint32_t store_qmask(const TileIO& io, const uint64_t* mask, uint32_t s) {
  uint32_t qm = io.valid;
  static_for<4>([&](auto Q) {
    constexpr int q = decltype(Q)::value;
    if (!((mask[q] >> s) & 1)) qm &= ~(1u << q);
  });
  return qm;
}

// One 64-chunk tile per workgroup: 64 KiB LDS (ROUNDS = 2), two workgroups per CU.
template <int DIN, int DOUT, int ROUNDS, int LB>
__global__ __launch_bounds__(256, LB) void xform32_kernel(const XformParams p) {
  __shared__ uint4 lds[(ROUNDS == 2 ? 16 : 8) * 4 * kXfLanes];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  Regs8 ra;
  xf32_load_raw(p, tile_io(p, blockIdx.x, lane, p.in_block_stride), wave, ra);
  // Store-mask words, fetched now so their latency hides under the data loads.  With
  // one pattern for the batch the word is wave-uniform (scalar load).
  uint64_t mask[4] = {~0ull, ~0ull, ~0ull, ~0ull};
  if (p.out_mask) {
    if (!p.pattern_per_block) {
      const uint64_t m = p.out_mask[0];
      mask[0] = mask[1] = mask[2] = mask[3] = m;
    } else {
      const TileIO io = tile_io(p, blockIdx.x, lane, p.out_block_stride);
      static_for<4>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        mask[q] = p.out_mask[io.blk[q]];
      });
    }
  }

  static_for<8>([&](auto T) {
    swap_halves(ra[decltype(T)::value]);
    dev::planes_from_raw(ra[decltype(T)::value]);
  });
  xf32_pass_a<DIN>(wave, ra);
  Regs8 rb;
  xf32_exchange_ab<ROUNDS>(wave, lane, lds, ra, rb);
  xf32_pass_b<DIN, DOUT>(rb);
  xf32_exchange_bc<ROUNDS>(wave, lane, lds, rb, ra);

  // pass C only where some lane of the wave stores one of its 8 shards (a decode restores
  // only the erased originals)
  const TileIO out_io = tile_io(p, blockIdx.x, lane, p.out_block_stride);
  uint32_t need = 0;
  static_for<8>([&](auto T) {
    constexpr int t = decltype(T)::value;
    const uint32_t s = 8 * wave + t;
    if (s < p.n_out && store_qmask(out_io, mask, s)) need = 1;
  });
  if (__builtin_amdgcn_ballot_w64(need != 0) == 0) return;
  xf32_pass_c<DOUT>(wave, ra);
  static_for<8>([&](auto T) {
    constexpr int t = decltype(T)::value;
    const uint32_t s = 8 * wave + t;  // wave-uniform
    if (s < p.n_out) store_shard(p.out + s * p.out_shard_stride, out_io, store_qmask(out_io, mask, s), ra[t]);
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
bool xform_supported(unsigned n) { return n == 32; }

hipError_t launch_xform(XformKind kind, const XformParams& p, hipStream_t stream) {
  if (p.total_columns == 0) return hipSuccess;
  const uint64_t groups = (p.total_columns + kXfLanes - 1) / kXfLanes;
  if (groups > 0x7FFFFFFFull) return hipErrorInvalidValue;
  const dim3 block(256);
  const dim3 grid(static_cast<unsigned>(groups));
  switch (kind) {
    case XformKind::kEncode32:
      hipLaunchKernelGGL((xform32_kernel<32, 0, 2, 2>), grid, block, 0, stream, p);
      break;
    case XformKind::kDecode32:
      hipLaunchKernelGGL((xform32_kernel<0, 32, 2, 2>), grid, block, 0, stream, p);
      break;
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

hipError_t launch_fill_splitmix(uint8_t* dst, uint64_t nblocks, uint64_t block_bytes, uint64_t dst_block_stride,
                                uint64_t seed_base, hipStream_t stream) {
  if (block_bytes % 8) return hipErrorInvalidValue;
  const uint64_t words = block_bytes / 8, pairs = (words + 1) / 2, n = nblocks * pairs;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(fill_splitmix_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, stream, dst,
                     nblocks, words, dst_block_stride, seed_base);
  return hipGetLastError();
}

}  // namespace ag
