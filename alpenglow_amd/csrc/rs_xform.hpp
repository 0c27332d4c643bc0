// Device building blocks of the bitsliced transform kernels, shared by rs_kernels.hip
// (xform / xform8 / decode_x) and rs_decode_c.hip (the correction decoder): tile I/O, the
// pass A / B / C butterfly layers of xform<NW>, LDS exchanges, and the xform8 layouts and
// pairwise slot swaps.  gfx950 / CDNA4 only.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "rs_device.hpp"
#include "rs_launch.hpp"
#include "unaligned.hpp"

namespace ag {
namespace {

using dev::static_for;

// =====================================================================================
// xform<NW>: N = 8 * NW point transform (NW = 4 -> 32, NW = 8 -> 64); NW waves x 64
// lanes; lane = one 64-byte column (32 symbols) of one block, each lane owns 8 of the N
// shards in each of three passes:
//   pass A  (wave w: shards 8w+t)       IFFT layers dist 1, 2, 4        (skew delta DIN)
//   pass B  (wave w: shards w+NW*t)     IFFT dist 8 .. N/2; FFT N/2 .. 8 (DIN / DOUT)
//   pass C  (wave w: shards 8w+t)       FFT layers dist 4, 2, 1         (skew delta DOUT)
// Shards change owner between passes through LDS (2 rounds per exchange: 64 KiB per
// round for N = 32, 128 KiB for N = 64).
// Skew index of a layer of distance d on the group starting at g: g + d + delta - 1.
// In pass B the group start depends only on shard bits >= 4, i.e. on the slot index, so
// that code is wave-independent; passes A and C branch once per butterfly on the
// (scalar) wave id.
// =====================================================================================

constexpr int kXfLanes = 64;

using Regs8 = uint32_t[8][16];

// butterfly whose skew index is BASE + 8 * wave (wave-uniform, runtime)
template <int S, bool INV>
__device__ __forceinline__ void bfly(uint32_t* x, uint32_t* y) {
  if constexpr (INV) dev::ifft_bfly<S>(x, y); else dev::fft_bfly<S>(x, y);
}
template <int BASE, bool INV, int NW>
__device__ __forceinline__ void bfly_w(int wave, uint32_t* x, uint32_t* y) {
  if constexpr (NW == 4) {
    switch (wave) {
      case 0: bfly<BASE, INV>(x, y); break;
      case 1: bfly<BASE + 8, INV>(x, y); break;
      case 2: bfly<BASE + 16, INV>(x, y); break;
      default: bfly<BASE + 24, INV>(x, y); break;
    }
  } else {
    switch (wave) {
      case 0: bfly<BASE, INV>(x, y); break;
      case 1: bfly<BASE + 8, INV>(x, y); break;
      case 2: bfly<BASE + 16, INV>(x, y); break;
      case 3: bfly<BASE + 24, INV>(x, y); break;
      case 4: bfly<BASE + 32, INV>(x, y); break;
      case 5: bfly<BASE + 40, INV>(x, y); break;
      case 6: bfly<BASE + 48, INV>(x, y); break;
      default: bfly<BASE + 56, INV>(x, y); break;
    }
  }
}
template <int NW, int DIN>
__device__ __forceinline__ void xf_pass_a(int wave, Regs8& r) {
  static_for<4>([&](auto I) {  // dist 1
    constexpr int t = 2 * decltype(I)::value;
    bfly_w<t + 1 + DIN - 1, true, NW>(wave, r[t], r[t + 1]);
  });
  static_for<4>([&](auto I) {  // dist 2
    constexpr int g = 4 * (decltype(I)::value >> 1);
    constexpr int u = g + (decltype(I)::value & 1);
    bfly_w<g + 2 + DIN - 1, true, NW>(wave, r[u], r[u + 2]);
  });
  static_for<4>([&](auto I) {  // dist 4
    constexpr int u = decltype(I)::value;
    bfly_w<4 + DIN - 1, true, NW>(wave, r[u], r[u + 4]);
  });
}

// Pass B: slot t holds shard w + NW*t.  Layer on shard bit sb (dist 2^sb, sb >= 3) pairs
// slots t, t + 2^tb with tb = sb - log2(NW); group start (NW*t) & ~(2d - 1).
template <int NW>
struct PassB {
  static constexpr int kLogNw = NW == 4 ? 2 : 3;
  static constexpr int kLayers = NW == 4 ? 2 : 3;  // shard bits 3 .. 3 + kLayers - 1
  template <int L, int I>
  struct Pair {
    static constexpr int sb = 3 + L, tb = sb - kLogNw, d = 1 << sb;
    static constexpr int t = ((I >> tb) << (tb + 1)) | (I & ((1 << tb) - 1));
    static constexpr int u = t + (1 << tb);
    static constexpr int g = (NW * t) & ~(2 * d - 1);
  };
};
template <int NW, int DIN>
__device__ __forceinline__ void xf_pass_b_ifft(Regs8& r) {
  constexpr int NL = PassB<NW>::kLayers;
  static_for<NL>([&](auto L) {  // ascending distance
    static_for<4>([&](auto I) {
      using P = typename PassB<NW>::template Pair<decltype(L)::value, decltype(I)::value>;
      dev::ifft_bfly<P::g + P::d + DIN - 1>(r[P::t], r[P::u]);
    });
  });
}
template <int NW, int DOUT>
__device__ __forceinline__ void xf_pass_b_fft(Regs8& r) {
  constexpr int NL = PassB<NW>::kLayers;
  static_for<NL>([&](auto L) {  // descending distance
    static_for<4>([&](auto I) {
      using P = typename PassB<NW>::template Pair<NL - 1 - decltype(L)::value, decltype(I)::value>;
      dev::fft_bfly<P::g + P::d + DOUT - 1>(r[P::t], r[P::u]);
    });
  });
}
template <int NW, int DIN, int DOUT>
__device__ __forceinline__ void xf_pass_b(Regs8& r) {
  xf_pass_b_ifft<NW, DIN>(r);
  xf_pass_b_fft<NW, DOUT>(r);
}

template <int NW, int DOUT>
__device__ __forceinline__ void xf_pass_c(int wave, Regs8& r) {
  static_for<4>([&](auto I) {  // dist 4
    constexpr int u = decltype(I)::value;
    bfly_w<4 + DOUT - 1, false, NW>(wave, r[u], r[u + 4]);
  });
  static_for<4>([&](auto I) {  // dist 2
    constexpr int g = 4 * (decltype(I)::value >> 1);
    constexpr int u = g + (decltype(I)::value & 1);
    bfly_w<g + 2 + DOUT - 1, false, NW>(wave, r[u], r[u + 2]);
  });
  static_for<4>([&](auto I) {  // dist 1
    constexpr int t = 2 * decltype(I)::value;
    bfly_w<t + 1 + DOUT - 1, false, NW>(wave, r[t], r[t + 1]);
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
// Streamed shard pieces: read once, written once, so the transform kernels load and store
// them non-temporally (nt).  Measured on the headline (profiles/r03_nt_ab.txt, two
// interleaved rounds): encode 5.67 -> 5.81-5.85 TB/s, reconstruct 5.44-5.47 -> 5.89-5.93 TB/s
// with both; loads alone +1-2 %, stores alone +2-5 %.
__device__ __forceinline__ uint4 ld_piece(const uint8_t* p) {
  const dev::u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const dev::u32x4*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_piece(uint8_t* p, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  const dev::u32x4 v = {a, b, c, d};
  __builtin_nontemporal_store(v, reinterpret_cast<dev::u32x4*>(p));
}
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
  uint32_t tailq;   // bit q: chunk q is its shard's tail chunk (TAIL kernels)
  uint32_t tlen;    // bytes of this lane's run in a tail chunk (0..16)
  uint32_t tsh;     // its run's start within the lane's 16-byte tail window (off[q] = the window)
  uint32_t tlen_h;  // h = T / 2 (uniform)
};
// Tail chunks (shard bytes S with T = S mod 64 != 0): the crate stores the last T bytes as T/2
// low bytes then T/2 high bytes, i.e. a 64-byte chunk whose symbols h..31
// (h = T/2) are zero.  The four quarter lanes of a chunk (low bytes of symbols 0-15 / 16-31,
// high bytes of 0-15 / 16-31) own the runs [0, 16) [16, h) [h, h + 16) [h + 16, T) of the
// tail (for h >= 16; for 8 <= h < 16: [0, h) and [h, T), quarters 1 and 3 empty).  Each lane
// moves one whole 16-byte window of the tail that contains its run -- [0, 16), [h - 16, h),
// [h, h + 16), [T - 16, T); for h < 16: [0, 16) and [T - 16, T) -- so tail pieces load and
// store with the same instructions as every other piece (T >= 16: every window lies inside the
// tail).  A loaded window is shifted down to its run (tail_fix_all); a stored window is
// completed with the neighbouring run's bytes from the partner lane (tail_window), so the
// bytes two lanes both write are equal.
__device__ __forceinline__ TileIO tile_io_g(uint64_t total_columns, uint32_t chunks_per_shard, uint64_t tile, int lane,
                                           uint64_t block_stride, uint32_t tail = 0) {
  TileIO io;
  io.valid = 0;
  io.tailq = 0;
  const uint32_t quarter = ((lane >> 5) << 1) | (lane & 1);
  const uint32_t h = tail / 2;
  io.tlen_h = h;
  uint32_t win;  // window start in the tail
  if (h >= 16) {
    win = quarter == 0 ? 0 : quarter == 1 ? h - 16 : quarter == 2 ? h : tail - 16;
    io.tsh = (quarter & 1) ? 32 - h : 0;
    io.tlen = (quarter & 1) ? h - 16 : 16;
  } else {
    win = quarter < 2 ? 0 : tail - 16;
    io.tsh = quarter == 2 ? 16 - h : 0;
    io.tlen = (quarter & 1) ? 0 : h;
  }  // the tile's first chunk once per wave (scalar division); lanes add < 64 chunks to its
  // in-block index, so a lane crosses at most one block boundary when C >= 64 (the 64-bit
  // division per lane and piece cost ~10 % of a reconstruct's VALU)
  const uint32_t C = chunks_per_shard;
  const uint64_t g0 = tile * kXfLanes;
  const uint64_t b0 = g0 / C;
  const uint32_t r0 = static_cast<uint32_t>(g0 - b0 * C);
  const uint64_t base = b0 * block_stride;
  const uint32_t lc = (lane & 31) >> 1;
  // Tail kernels with 16 or 32 chunks per shard and T % 8 == 0 (a tile is 64 / C whole shard
  // rows): instruction q takes chunks [q C/4, (q + 1) C/4) of each row -- runs of C/4 chunks
  // instead of one 16-chunk run -- so every tail chunk falls in instruction 3 and the window
  // fix-ups run for one of the four pieces of each slot.  Measured against the 16-chunk runs
  // (profiles/r05_ab_tail_runs.jsonl, one box): S = 1000 3.90 -> 4.37 / 4.37 -> 4.65 TB/s
  // encode / reconstruct, S = 2000 4.31 -> 4.68 / 4.77 -> 4.95; but S = 1022 (2-byte aligned
  // shards) 3.85 -> 3.57 encode and C = 8 (128-byte runs) 3.51 -> 2.77: those keep 16-chunk runs
  const uint32_t R = (tail != 0 && tail % 8 == 0 && (C == 16 || C == 32)) ? C / 4 : 16;
  static_for<4>([&](auto Q) {
    constexpr int q = decltype(Q)::value;
    const uint32_t cl = R == 16 ? 16 * q + lc : (lc / R) * C + q * R + lc % R;
    const bool ok = g0 + cl < total_columns;
    const uint32_t c = ok ? r0 + cl : r0;  // idle pieces re-read the tile's first chunk, never store
    uint32_t d, rem;
    if (C >= kXfLanes) {
      d = c >= C ? 1u : 0u;
      rem = d ? c - C : c;
    } else {
      d = c / C;
      rem = c - d * C;
    }
    io.blk[q] = b0 + d;
    const bool tq = tail != 0 && rem == C - 1;
    io.off[q] = base + d * block_stride + static_cast<uint64_t>(rem) * 64 + (tq ? win : 16 * quarter);
    io.valid |= ok ? (1u << q) : 0u;
    io.tailq |= tq ? (1u << q) : 0u;
  });
  return io;
}
template <int TAIL = 0>
__device__ __forceinline__ TileIO tile_io(const XformParams& p, uint64_t tile, int lane, uint64_t block_stride) {
  return tile_io_g(p.total_columns, p.chunks_per_shard, tile, lane, block_stride, TAIL ? p.tail_bytes : 0u);
}

// Byte funnels on 16-byte windows with a wave-uniform byte count j (0..16): out = bytes
// [j, j + 16) of the 32-byte little-endian value lo ++ hi.  One scalar branch on j / 4 picks
// the word offset, then four v_alignbyte_b32 (the 64-bit shift pairs and their selects of a
// per-lane form cost ~2x the VALU and a branch per shift).
template <int W>
__device__ __forceinline__ void funnel_w(const uint32_t* lo, const uint32_t* hi, uint32_t b, uint32_t* out) {
  const uint32_t c[9] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3], 0u};
  static_for<4>([&](auto I) {
    constexpr int i = decltype(I)::value;
    out[i] = __builtin_amdgcn_alignbyte(c[i + W + 1], c[i + W], b);
  });
}
__device__ __forceinline__ void funnel16(const uint32_t* lo, const uint32_t* hi, uint32_t j, uint32_t* out) {
  j = __builtin_amdgcn_readfirstlane(j);
  const uint32_t b = j & 3;
  switch (j >> 2) {
    case 0: funnel_w<0>(lo, hi, b, out); break;
    case 1: funnel_w<1>(lo, hi, b, out); break;
    case 2: funnel_w<2>(lo, hi, b, out); break;
    case 3: funnel_w<3>(lo, hi, b, out); break;
    default: funnel_w<4>(lo, hi, b, out); break;
  }
}
// keep the low `len` bytes (0..16, uniform): word masks from scalar arithmetic
__device__ __forceinline__ void keep16(uint32_t* v, uint32_t len) {
  len = __builtin_amdgcn_readfirstlane(len);
  static_for<4>([&](auto K) {
    constexpr int k = decltype(K)::value;
    const int keep = static_cast<int>(len) - 4 * k;
    const uint32_t m = keep >= 4 ? ~0u : keep <= 0 ? 0u : (1u << (8 * keep)) - 1;
    v[k] &= m;
  });
}
// A short tail (T < 16 bytes, even, uniform) as one 16-byte value, zeros from T on: its 8-, 4-
// and 2-byte parts where present (accesses inside [0, T) only)
__device__ __forceinline__ void load_short_tail(const uint8_t* src, uint32_t T, uint32_t* b) {
  b[0] = b[1] = b[2] = b[3] = 0u;
  if (T & 8) {
    const uint2 x = ld8u(src);
    b[0] = x.x;
    b[1] = x.y;
  }
  if (T & 4) {
    const uint32_t x = ld4u(src + (T & 8));
    if (T & 8) b[2] = x;
    else b[0] = x;
  }
  if (T & 2) {
    const uint32_t x = ld2u(src + (T & 12));  // word (T & 12) / 4, low half
    const uint32_t w = (T & 12) >> 2;
    if (w == 0) b[0] |= x;
    else if (w == 1) b[1] |= x;
    else if (w == 2) b[2] |= x;
    else b[3] |= x;
  }
}
__device__ __forceinline__ void store_short_tail(uint8_t* dst, uint32_t T, const uint32_t* b) {
  if (T & 8) st8u(dst, make_uint2(b[0], b[1]));
  if (T & 4) st4u(dst + (T & 8), (T & 8) ? b[2] : b[0]);
  if (T & 2) {
    const uint32_t w = (T & 12) >> 2;
    st2u(dst + (T & 12), w == 0 ? b[0] : w == 1 ? b[1] : w == 2 ? b[2] : b[3]);
  }
}
// One lane's whole tail chunk (T = S mod 64 bytes, 2 <= T < 64, even, uniform; h = T / 2
// symbols): the crate keeps the h low bytes then the h high bytes, i.e. the
// 64-byte chunk (low bytes [0, 32), high bytes [32, 64)) with symbols h..31 zero.  Moved with
// accesses inside [0, T) only, so no byte of the next shard is touched: for T >= 16, 16-byte
// windows, a run that would cross T coming from (going to) the window [T - 16, T) through one
// uniform funnel; a shorter tail as its 8-, 4- and 2-byte parts.  Raw chunk words in v[16]
// (before planes_from_raw / after the inverse transpose).
__device__ __forceinline__ void load_tail_chunk(const uint8_t* src, uint32_t T, uint32_t* v) {
  T = __builtin_amdgcn_readfirstlane(T);
  const uint32_t h = T / 2;
  const uint32_t z[4] = {0u, 0u, 0u, 0u};
  if (T < 16) {  // low [0, h) and high [0, h) of the one short value
    load_short_tail(src, T, v);
    funnel16(v, z, h, v + 8);
    keep16(v, h);
    keep16(v + 8, h);
    static_for<4>([&](auto W) {
      v[4 + decltype(W)::value] = 0u;
      v[12 + decltype(W)::value] = 0u;
    });
    return;
  }
  auto ld = [&](uint32_t off, uint32_t* out) __attribute__((always_inline)) {
    const uint4 x = ld16u(src + off);
    out[0] = x.x; out[1] = x.y; out[2] = x.z; out[3] = x.w;
  };
  uint32_t w[4];
  ld(T - 16, w);  // tail bytes [T - 16, T)
  if (h >= 16) {  // low [0, 16) [16, h), high [h, h + 16) and [h + 16, T) from the last window
    ld(0, v);
    ld(16, v + 4);
    keep16(v + 4, h - 16);
    ld(h, v + 8);
    funnel16(w, z, 32 - h, v + 12);  // high byte 16 sits at 32 - h of the window
    keep16(v + 12, h - 16);
  } else {        // T < 32: low [0, h) from the first 16 bytes, high [0, h) from the last window
    ld(0, v);
    keep16(v, h);
    funnel16(w, z, 16 - h, v + 8);
    keep16(v + 8, h);
    static_for<4>([&](auto W) {
      v[4 + decltype(W)::value] = 0u;
      v[12 + decltype(W)::value] = 0u;
    });
  }
}
// The inverse: the T bytes of a restored tail chunk (raw words v[16], symbols h..31 zero).
// Stores go low run first, then high run, so a window's bytes past the low run are rewritten
// by the high run's stores in program order; overlapping windows carry equal bytes.
__device__ __forceinline__ void store_tail_chunk(uint8_t* dst, uint32_t T, const uint32_t* v) {
  T = __builtin_amdgcn_readfirstlane(T);
  const uint32_t h = T / 2;
  const uint32_t z[4] = {0u, 0u, 0u, 0u};
  if (T < 16) {  // low [0, h) | high [0, h) << h as one short value
    uint32_t lo[4] = {v[0], v[1], v[2], v[3]}, hs[4];
    keep16(lo, h);
    funnel16(z, v + 8, 16 - h, hs);
    static_for<4>([&](auto W) { lo[decltype(W)::value] |= hs[decltype(W)::value]; });
    store_short_tail(dst, T, lo);
    return;
  }
  auto st = [&](uint32_t off, const uint32_t* x) __attribute__((always_inline)) {
    st16u(dst + off, make_uint4(x[0], x[1], x[2], x[3]));
  };
  if (h >= 16) {
    st(0, v);      // low [0, 16)
    st(16, v + 4); // low [16, h) (bytes [h, 32) are rewritten below)
    st(h, v + 8);  // high [0, 16) at [h, h + 16)
    uint32_t w[4];
    funnel16(v + 8, v + 12, h - 16, w);  // high [h - 16, h) at [T - 16, T)
    st(T - 16, w);
  } else {
    st(0, v);      // low [0, h) (bytes [h, 16) are rewritten below)
    // the window [T - 16, T) = low [T - 16, h) ++ high [0, h): the 32 bytes low | high << h
    uint32_t lo[4] = {v[0], v[1], v[2], v[3]}, a[4], b[4], w[4];
    keep16(lo, h);
    funnel16(z, v + 8, 16 - h, a);  // high [0, 16 - h) at byte h
    static_for<4>([&](auto W) { a[decltype(W)::value] |= lo[decltype(W)::value]; });
    funnel16(v + 8, z, 16 - h, b);  // high [16 - h, h) at byte 16
    funnel16(a, b, T - 16, w);
    st(T - 16, w);
  }
}

// piece q of shard `base` (a tail piece is its lane's whole window: tail_fix_all after the
// tile's loads, so no load waits on the others)
template <int TAIL>
__device__ __forceinline__ uint4 ld_piece_io(const uint8_t* base, const TileIO& io, int q) {
  return ld_piece(base + io.off[q]);
}
// the loaded tail windows of one slot (registers 4 q .. 4 q + 3 = piece q) -> their runs at
// byte 0, zeros above (the transform then sees symbols h..31 as zero).  Shift and length
// depend only on h (uniform) and the lane's quarter.
template <int TAIL>
__device__ __forceinline__ void tail_fix_all(const TileIO& io, uint32_t* v) {
  if constexpr (TAIL == 1) {
    const int lane = threadIdx.x & 63;
    const uint32_t h = __builtin_amdgcn_readfirstlane(io.tlen_h);
    const uint32_t zero[4] = {0u, 0u, 0u, 0u};
    static_for<4>([&](auto Q) {
      constexpr int q = decltype(Q)::value;
      if (__builtin_amdgcn_ballot_w64((io.tailq >> q) & 1) != 0) {  // wave-uniform
        uint32_t* x = v + 4 * q;
        const bool tl = (io.tailq >> q) & 1;
        uint32_t t[4];
        if (h >= 16) {  // quarters 1 / 3: window [h - 16, h) / [T - 16, T), run at 32 - h
          funnel16(x, zero, 32 - h, t);
          keep16(t, h - 16);
          if (tl && (lane & 1)) static_for<4>([&](auto K) { x[decltype(K)::value] = t[decltype(K)::value]; });
        } else {  // quarter 0: run [0, h) at 0; quarter 2: window [T - 16, T), run at 16 - h; 1 / 3 empty
          funnel16(x, zero, 16 - h, t);
          if (tl) {
            static_for<4>([&](auto K) {
              constexpr int k = decltype(K)::value;
              x[k] = (lane & 1) ? 0u : lane >= 32 ? t[k] : x[k];
            });
            keep16(x, h);
          }
        }
      }
    });
  }
}
// The window a tail lane stores, from its run (bytes 0..tlen-1 of v, zeros above) and the
// partner run's bytes: quarters 1 / 3 take quarter 0 / 2 (the lane below, quad permute);
// with h < 16 quarters 0 / 2 take each other (lanes l, l + 32).  Wave-wide: every lane runs
// the exchanges; the caller stores the result on tail lanes only.  h is uniform.
__device__ __forceinline__ void tail_window(uint32_t* v, int lane, uint32_t h) {
  h = __builtin_amdgcn_readfirstlane(h);
  const uint32_t zero[4] = {0u, 0u, 0u, 0u};
  if (h >= 16) {
    uint32_t lo[4];  // the lane below's run (quarter 0 / 2 of the chunk)
    static_for<4>([&](auto K) {
      constexpr int k = decltype(K)::value;
      lo[k] = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v[k]), 0xA0 /* quad_perm 0,0,2,2 */, 0xF,
                                                             0xF, false));
    });
    // window [h - 16, h) = lo[h - 16, 16) ++ own[0, h - 16): bytes h - 16 .. h + 15 of lo ++ own
    uint32_t w[4];
    funnel16(lo, v, h - 16, w);
    if (lane & 1) static_for<4>([&](auto K) { v[decltype(K)::value] = w[decltype(K)::value]; });
  } else {
    uint32_t pr[4];  // the partner half's run: quarter 0 <-> 2
    static_for<4>([&](auto K) {
      constexpr int k = decltype(K)::value;
      pr[k] = __builtin_amdgcn_permlane32_swap(v[k], v[k], false, false)[0];
    });
    // quarter 2: window [T - 16, T) = q0[2h - 16, h) ++ own[0, h) (pr is zero from byte h on);
    // quarter 0: window [0, 16) = own[0, h) ++ q2[0, 16 - h)
    uint32_t a[4], b[4];
    funnel16(pr, zero, 2 * h - 16, a);  // q0's bytes from 2h - 16 down to 0
    funnel16(zero, v, h, b);            // own run moved up by 16 - h
    uint32_t c[4];
    funnel16(zero, pr, 16 - h, c);      // q2's run moved up by h
    static_for<4>([&](auto K) {
      constexpr int k = decltype(K)::value;
      v[k] = lane >= 32 ? (a[k] | b[k]) : (v[k] | c[k]);
    });
  }
}
template <int TAIL>
__device__ __forceinline__ void st_piece_io(uint8_t* base, const TileIO& io, int q, uint32_t a, uint32_t b, uint32_t c,
                                            uint32_t d) {
  st_piece(base + io.off[q], a, b, c, d);
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
template <int TAIL = 0>
__device__ __forceinline__ void xf_load_raw(const XformParams& p, const TileIO& io, int wave, Regs8& raw) {
  static_for<8>([&](auto T) {
    constexpr int t = decltype(T)::value;
    const uint32_t s = 8 * wave + t;  // wave-uniform condition
    if (s < p.n_in) {
      const uint8_t* base = p.in + s * p.in_shard_stride;
      static_for<4>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        const uint4 x = ld_piece_io<TAIL>(base, io, q);
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

// Planes -> bytes -> lane-linear pieces, stored where the input pieces were read.  ACC: XOR
// into the bytes already there (a partial result stored by an earlier pass).
template <bool ACC = false, int TAIL = 0>
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
  if constexpr (TAIL == 1) {
    // tail pieces: the run (symbols >= h are zero: the inputs there were zero) completed to
    // the lane's window; lanes with an empty run (tlen 0) store nothing
    const int lane = threadIdx.x & 63;
    static_for<4>([&](auto Q) {
      constexpr int q = decltype(Q)::value;
      if (__builtin_amdgcn_ballot_w64((io.tailq >> q) & 1) != 0) {  // wave-uniform
        // (bytes past the run are zero: outputs at symbols >= h come from zero inputs)
        uint32_t w[4] = {v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
        tail_window(w, lane, io.tlen_h);
        if ((io.tailq >> q) & 1) {
          static_for<4>([&](auto K) { v[4 * q + decltype(K)::value] = w[decltype(K)::value]; });
          if (io.tlen == 0) qmask &= ~(1u << q);
        }
      }
    });
  }
  static_for<4>([&](auto Q) {
    constexpr int q = decltype(Q)::value;
    if (qmask & (1u << q)) {
      if constexpr (ACC) {
        static_assert(TAIL != 1, "accumulating stores of tail windows are not supported");
        const uint4 x = ld_piece_io<TAIL>(base, io, q);
        uint32_t o[4] = {x.x, x.y, x.z, x.w};
        st_piece_io<TAIL>(base, io, q, v[4 * q] ^ o[0], v[4 * q + 1] ^ o[1], v[4 * q + 2] ^ o[2], v[4 * q + 3] ^ o[3]);
      } else {
        st_piece_io<TAIL>(base, io, q, v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
      }
    }
  });
}

// LDS exchange between passes (2 rounds, 4 A-slots per wave per round).
//   NW = 4: A-slot t of wave w (shard 8w+t) <-> B-slot 2w+(t>>2) of wave t&3
//   NW = 8: A-slot t of wave w (shard 8w+t) <-> B-slot w of wave t
template <int NW>
__device__ __forceinline__ void xf_exchange_ab(int wave, int lane, uint4* lds, Regs8& ra, Regs8& rb) {
  static_for<2>([&](auto Rho) {
    constexpr int rho = decltype(Rho)::value;
    static_for<4>([&](auto U) {
      constexpr int u = decltype(U)::value;
      lds_put(lds, 4 * wave + u, lane, ra[4 * rho + u]);
    });
    __syncthreads();
    if constexpr (NW == 4) {
      static_for<4>([&](auto W2) {
        constexpr int w2 = decltype(W2)::value;
        lds_get(lds, 4 * w2 + wave, lane, rb[2 * w2 + rho]);
      });
    } else {
      if ((wave >> 2) == rho) {
        static_for<8>([&](auto W2) {
          constexpr int w2 = decltype(W2)::value;
          lds_get(lds, 4 * w2 + (wave & 3), lane, rb[w2]);
        });
      }
    }
    __syncthreads();
  });
}

template <int NW>
__device__ __forceinline__ void xf_exchange_bc(int wave, int lane, uint4* lds, Regs8& rb, Regs8& ra) {
  static_for<2>([&](auto Rho) {
    constexpr int rho = decltype(Rho)::value;
    if constexpr (NW == 4) {
      static_for<4>([&](auto W2) {
        constexpr int w2 = decltype(W2)::value;
        lds_put(lds, 4 * w2 + wave, lane, rb[2 * w2 + rho]);
      });
    } else {
      if ((wave >> 2) == rho) {
        static_for<8>([&](auto W2) {
          constexpr int w2 = decltype(W2)::value;
          lds_put(lds, 4 * w2 + (wave & 3), lane, rb[w2]);
        });
      }
    }
    __syncthreads();
    static_for<4>([&](auto U) {
      constexpr int u = decltype(U)::value;
      lds_get(lds, 4 * wave + u, lane, ra[4 * rho + u]);
    });
    __syncthreads();
  });
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

// The store predicates of NS consecutive shards s0 .. s0 + NS - 1 (wave-uniform s0), packed
// before the first store: bits 4 i + q = store piece q of shard s0 + i.  Store loops read these
// bits instead of re-deriving them from the mask words between stores: xform_h8 did that and
// intermittently skipped whole lane classes' stores (per-block masks re-read with the slot
// before's stores in flight; tools/stress_xform64.py).  NS <= 8.
template <int NS>
__device__ __forceinline__ uint32_t qmask_all(const TileIO& io, const uint64_t* mask, uint32_t s0, uint32_t n_out) {
  uint32_t q = 0;
  static_for<NS>([&](auto I) {
    constexpr int i = decltype(I)::value;
    if (s0 + i < n_out) q |= store_qmask(io, mask, s0 + i) << (4 * i);
  });
  return q;
}

// =====================================================================================
// xform8: the 32-point transform with 8 waves per workgroup and 4 shard slots per lane.
// Half the per-lane state of xform<4> (16 loads per lane in flight instead of 32, ~half
// the VGPRs), so two 8-wave workgroups share a CU and each wave has half the arithmetic
// between its loads and its stores (tools/membench/membench4.hip: 64-column tile copies
// 5.57 -> 5.74 TB/s at 8 waves; xform<4> runs at its own load/store skeleton's speed).
// Every position bit is a slot bit (2) or a wave bit (3), so a layer's skew constant
// depends only on slot bits (compile time) and wave bits (a scalar switch over the wave
// bits above the layer).  A layer needs its bit in a slot; between layers one slot bit
// trades places with one wave bit (x8_swap: partner waves swap half their slots through
// 64 KiB of LDS; the other half stay in place):
//   L0 slots p0 p1 | waves p2 p3 p4   IFFT b0 b1            (loads, FFT b0, stores)
//   L1 slots p2 p1 | waves p0 p3 p4   IFFT b2               (FFT b1)
//   L2 slots p2 p3 | waves p0 p1 p4   IFFT b3               (FFT b2)
//   L3 slots p4 p3 | waves p0 p1 p2   IFFT b4, FFT b4 b3
// =====================================================================================
using Regs4 = uint32_t[4][16];

// Position bits held by slot bits (S0, S1) and wave bits (W0, W1, W2[, W3]).  W3 < 0: three
// wave bits (xform8, 32 points); W3 >= 0: sixteen waves (decode_x16, 64 points).
template <int S0, int S1, int W0, int W1, int W2, int W3 = -1>
struct X8Lay {
  static constexpr int sb[2] = {S0, S1};
  static constexpr int wb[4] = {W0, W1, W2, W3};
  static constexpr int pos(int w, int t) {
    return (((t >> 0) & 1) << sb[0]) | (((t >> 1) & 1) << sb[1]) | (((w >> 0) & 1) << wb[0]) |
           (((w >> 1) & 1) << wb[1]) | (((w >> 2) & 1) << wb[2]) | (W3 >= 0 ? ((w >> 3) & 1) << (W3 & 31) : 0);
  }
  static constexpr int slot_of(int b) { return sb[0] == b ? 0 : sb[1] == b ? 1 : -1; }
  // wave bits whose position bit exceeds b (the ones a layer-b constant depends on)
  static constexpr int rel(int b) {
    return (wb[0] > b ? 1 : 0) | (wb[1] > b ? 2 : 0) | (wb[2] > b ? 4 : 0) | (W3 >= 0 && wb[3] > b ? 8 : 0);
  }
};
template <int L>
struct X8LayoutSel;
template <>
struct X8LayoutSel<0> { using T = X8Lay<0, 1, 2, 3, 4>; };
template <>
struct X8LayoutSel<1> { using T = X8Lay<2, 1, 0, 3, 4>; };
template <>
struct X8LayoutSel<2> { using T = X8Lay<2, 3, 0, 1, 4>; };
template <>
struct X8LayoutSel<3> { using T = X8Lay<4, 3, 0, 1, 2>; };
template <int L>
using X8Layout = typename X8LayoutSel<L>::T;

constexpr int x8_popc(int m) { return (m & 1) + ((m >> 1) & 1) + ((m >> 2) & 1) + ((m >> 3) & 1); }
// wave bits selected by REL packed into the low bits, and back
template <int REL>
__device__ __forceinline__ int x8_compress(int w) {
  if constexpr (REL == 0) return 0;
  if constexpr (REL == 15) return w;
  int v = 0, k = 0;
  if constexpr (REL & 1) v |= (w & 1) << k++;
  if constexpr (REL & 2) v |= ((w >> 1) & 1) << k++;
  if constexpr (REL & 4) v |= ((w >> 2) & 1) << k++;
  if constexpr (REL & 8) v |= ((w >> 3) & 1) << k++;
  return v;
}
constexpr int x8_expand(int v, int rel) {
  int w = 0, k = 0;
  for (int j = 0; j < 4; ++j)
    if ((rel >> j) & 1) w |= ((v >> k++) & 1) << j;
  return w;
}

// The butterfly on slots (T, T | 2^i) of layer bit B in layout Lay for the wave bits V.
// FFT butterflies with upd_y false skip y ^= x (y's new value is never used).
template <typename Lay, int B, bool INV, int DELTA, int T, int V, int TAB = 0>
__device__ __forceinline__ void x8_bfly(uint32_t* x, uint32_t* y, bool upd_y) {
  constexpr int w = x8_expand(V, Lay::rel(B));
  constexpr int S = (Lay::pos(w, T) & ~((2 << B) - 1)) + (1 << B) + DELTA - 1;
  if constexpr (INV) {
    dev::ifft_bfly<S, TAB>(x, y);
  } else {
    if constexpr (kSkewLog[S] != 65535) dev::mul_acc<S, TAB>(x, y);
    if (upd_y) dev::xor_planes(y, x);
  }
}
template <typename Lay, int B, bool INV, int DELTA, int T, int TAB = 0>
__device__ __forceinline__ void x8_bfly_w(int v, uint32_t* x, uint32_t* y, bool upd_y = true) {
  constexpr int n = 1 << x8_popc(Lay::rel(B));
  if constexpr (n == 1) {
    x8_bfly<Lay, B, INV, DELTA, T, 0, TAB>(x, y, upd_y);
  } else if constexpr (n == 2) {
    if (v == 0) x8_bfly<Lay, B, INV, DELTA, T, 0, TAB>(x, y, upd_y); else x8_bfly<Lay, B, INV, DELTA, T, 1, TAB>(x, y, upd_y);
  } else if constexpr (n == 4) {
    switch (v) {
      case 0: x8_bfly<Lay, B, INV, DELTA, T, 0, TAB>(x, y, upd_y); break;
      case 1: x8_bfly<Lay, B, INV, DELTA, T, 1, TAB>(x, y, upd_y); break;
      case 2: x8_bfly<Lay, B, INV, DELTA, T, 2, TAB>(x, y, upd_y); break;
      default: x8_bfly<Lay, B, INV, DELTA, T, 3, TAB>(x, y, upd_y); break;
    }
  } else if constexpr (n == 8) {
    switch (v) {
      case 0: x8_bfly<Lay, B, INV, DELTA, T, 0, TAB>(x, y, upd_y); break;
      case 1: x8_bfly<Lay, B, INV, DELTA, T, 1, TAB>(x, y, upd_y); break;
      case 2: x8_bfly<Lay, B, INV, DELTA, T, 2, TAB>(x, y, upd_y); break;
      case 3: x8_bfly<Lay, B, INV, DELTA, T, 3, TAB>(x, y, upd_y); break;
      case 4: x8_bfly<Lay, B, INV, DELTA, T, 4, TAB>(x, y, upd_y); break;
      case 5: x8_bfly<Lay, B, INV, DELTA, T, 5, TAB>(x, y, upd_y); break;
      case 6: x8_bfly<Lay, B, INV, DELTA, T, 6, TAB>(x, y, upd_y); break;
      default: x8_bfly<Lay, B, INV, DELTA, T, 7, TAB>(x, y, upd_y); break;
    }
  } else {
    switch (v) {
      case 0: x8_bfly<Lay, B, INV, DELTA, T, 0, TAB>(x, y, upd_y); break;
      case 1: x8_bfly<Lay, B, INV, DELTA, T, 1, TAB>(x, y, upd_y); break;
      case 2: x8_bfly<Lay, B, INV, DELTA, T, 2, TAB>(x, y, upd_y); break;
      case 3: x8_bfly<Lay, B, INV, DELTA, T, 3, TAB>(x, y, upd_y); break;
      case 4: x8_bfly<Lay, B, INV, DELTA, T, 4, TAB>(x, y, upd_y); break;
      case 5: x8_bfly<Lay, B, INV, DELTA, T, 5, TAB>(x, y, upd_y); break;
      case 6: x8_bfly<Lay, B, INV, DELTA, T, 6, TAB>(x, y, upd_y); break;
      case 7: x8_bfly<Lay, B, INV, DELTA, T, 7, TAB>(x, y, upd_y); break;
      case 8: x8_bfly<Lay, B, INV, DELTA, T, 8, TAB>(x, y, upd_y); break;
      case 9: x8_bfly<Lay, B, INV, DELTA, T, 9, TAB>(x, y, upd_y); break;
      case 10: x8_bfly<Lay, B, INV, DELTA, T, 10, TAB>(x, y, upd_y); break;
      case 11: x8_bfly<Lay, B, INV, DELTA, T, 11, TAB>(x, y, upd_y); break;
      case 12: x8_bfly<Lay, B, INV, DELTA, T, 12, TAB>(x, y, upd_y); break;
      case 13: x8_bfly<Lay, B, INV, DELTA, T, 13, TAB>(x, y, upd_y); break;
      case 14: x8_bfly<Lay, B, INV, DELTA, T, 14, TAB>(x, y, upd_y); break;
      default: x8_bfly<Lay, B, INV, DELTA, T, 15, TAB>(x, y, upd_y); break;
    }
  }
}
// One butterfly layer on position bit B in layout L (skew delta DELTA).  LIVE: the slots
// that still carry needed values (half-pruned FFT); UPD_Y false: FFT x updates only.
template <int L, int B, bool INV, int DELTA, int LIVE = 0xF, bool UPD_Y = true, int TAB = 0>
__device__ __forceinline__ void x8_layer(int wave, Regs4& r) {
  using Lay = X8Layout<L>;
  constexpr int i = Lay::slot_of(B);
  static_assert(i >= 0, "layer bit must be a slot bit");
  const int v = x8_compress<Lay::rel(B)>(wave);
  constexpr int t0 = 0, t1 = i == 0 ? 2 : 1;  // the slots with bit i clear
  if constexpr ((LIVE >> t0) & 1) x8_bfly_w<Lay, B, INV, DELTA, t0, TAB>(v, r[t0], r[t0 | (1 << i)], UPD_Y);
  if constexpr ((LIVE >> t1) & 1) x8_bfly_w<Lay, B, INV, DELTA, t1, TAB>(v, r[t1], r[t1 | (1 << i)], UPD_Y);
}
// the same on an explicit layout type (xform8's pruned FFT layouts, decode_x16's layouts)
template <typename Lay, int B, bool INV, int DELTA, int TAB = 0>
__device__ __forceinline__ void x8_layer_t(int wave, Regs4& r) {
  constexpr int i = Lay::slot_of(B);
  static_assert(i >= 0, "layer bit must be a slot bit");
  const int v = x8_compress<Lay::rel(B)>(wave);
  constexpr int t0 = 0, t1 = i == 0 ? 2 : 1;
  x8_bfly_w<Lay, B, INV, DELTA, t0, TAB>(v, r[t0], r[t0 | (1 << i)]);
  x8_bfly_w<Lay, B, INV, DELTA, t1, TAB>(v, r[t1], r[t1 | (1 << i)]);
}
template <typename Lay, int B, int DELTA, int LIVE, int TAB = 0>
__device__ __forceinline__ void x8_layer_lay(int wave, Regs4& r) {
  constexpr int i = Lay::slot_of(B);
  static_assert(i >= 0, "layer bit must be a slot bit");
  const int v = x8_compress<Lay::rel(B)>(wave);
  constexpr int t0 = 0, t1 = i == 0 ? 2 : 1;
  if constexpr ((LIVE >> t0) & 1) x8_bfly_w<Lay, B, false, DELTA, t0, TAB>(v, r[t0], r[t0 | (1 << i)]);
  if constexpr ((LIVE >> t1) & 1) x8_bfly_w<Lay, B, false, DELTA, t1, TAB>(v, r[t1], r[t1 | (1 << i)]);
}

// Slot bit I <-> wave bit J.  Slot t of wave w moves iff t_I != w_J: to slot t ^ 2^I of
// wave w ^ 2^J, whose outgoing slots are exactly the incoming ones' registers.
// The branches for t and t ^ 2^I have complementary conditions; the asm markers keep
// LLVM from merging them into one access through a phi of register-array pointers
// (which would send the whole slot array to scratch).
// Partner waves synchronise through LDS epoch flags instead of workgroup barriers (ready[w] =
// last swap whose data w has written, done[w] = last swap w has read).
template <int NWAVES>
struct XFlags {
  uint32_t ready[NWAVES];
  uint32_t done[NWAVES];
};
using X8Flags = XFlags<8>;
__device__ __forceinline__ void x8_wait_ge(const uint32_t* f, uint32_t e) {
  while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < e) __builtin_amdgcn_s_sleep(1);
}
__device__ __forceinline__ void x8_signal(uint32_t* f, uint32_t e, int lane) {
  if (lane == 0) __hip_atomic_store(f, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// SPLIT (default): each branch reads its slot behind an opaque zero offset, so LLVM cannot
// hoist the two branches' identical reads into one read ahead of the branch (which left a
// 16-32 VGPR copy after it: -96 VALU per xform8 wave).  decode_c and decode_pk keep the
// hoisted form: at their register pressure the split reads spill (35 and 4-6 VGPRs).
template <int I, int J, int EP, int LIVE = 0xF, bool SPLIT = true, typename Flags>
__device__ __forceinline__ void x8_swap(int wave, int lane, uint4* lds, Flags* fl, Regs4& r) {
  const int wj = (wave >> J) & 1;
  const int partner = wave ^ (1 << J);
  // region `partner` was last read by the partner in swap EP - 1
  if constexpr (EP > 1) x8_wait_ge(&fl->done[partner], EP - 1);
  static_for<4>([&](auto T) {
    constexpr int t = decltype(T)::value;
    constexpr int k = (t >> (1 - I)) & 1;  // the other slot bit: index within the pair
    if (((LIVE >> t) & 1) && ((t >> I) & 1) != wj) {
      lds_put(lds, 2 * partner + k, lane, r[t]);
      __asm__ volatile("; x8_swap put %0" ::"n"(t));
    }
  });
  x8_signal(&fl->ready[wave], EP, lane);
  x8_wait_ge(&fl->ready[partner], EP);
  static_for<4>([&](auto T) {
    constexpr int t = decltype(T)::value;
    constexpr int k = (t >> (1 - I)) & 1;
    if (((LIVE >> t) & 1) && ((t >> I) & 1) != wj) {
      int z = 0;
      if constexpr (SPLIT) __asm__ volatile("s_mov_b32 %0, 0 ; x8_swap slot %1" : "=s"(z) : "n"(t));
      lds_get(lds, 2 * wave + k + z, lane, r[t]);
      __asm__ volatile("; x8_swap get %0" ::"n"(t));
    }
  });
  x8_signal(&fl->done[wave], EP, lane);
}

// ---- 32-column tiles with the lane half as a position bit (decode_h8, xform_h8) --------
// Lane l holds column l & 31 of the tile; h = l >> 5 is position bit 2 in layout A (slots p0
// p1 | h p2 | waves p3 p4 p5).  A <-> B (h8_relayout) trades slot bit 0 and the lane half.
// The layer-0 butterfly of layout A; HPOS = the lane half's position bit (4 or 0).
template <typename Lay, int B, bool INV, int DELTA, int T, int V, int HPOS, int TAB = 0>
__device__ __forceinline__ void h8_bfly(uint32_t* x, uint32_t* y) {
  constexpr int w = x8_expand(V, Lay::rel(B));
  constexpr int S = ((Lay::pos(w, T) | HPOS) & ~((2 << B) - 1)) + (1 << B) + DELTA - 1;
  if constexpr (kSkewLog[S] != 65535) dev::mul_acc<S, TAB>(x, y);
}
// layer 0 in layout A: butterflies on slots (0, 1) and (2, 3); the lane half is p2
template <bool INV, int DELTA, int TAB = 0>
__device__ __forceinline__ void h8_layer0(int wave, int h, Regs4& r) {
  using LA = X8Lay<0, 1, 3, 4, 5>;
  static_for<2>([&](auto TT) {
    constexpr int t = 2 * decltype(TT)::value;
    if constexpr (INV) dev::xor_planes(r[t + 1], r[t]);
    auto mul = [&](auto Vc) {
      constexpr int v = decltype(Vc)::value;
      if (h) h8_bfly<LA, 0, INV, DELTA, t, v, 4, TAB>(r[t], r[t + 1]);
      else h8_bfly<LA, 0, INV, DELTA, t, v, 0, TAB>(r[t], r[t + 1]);
    };
    switch (wave) {  // every wave bit lies above bit 0
      case 0: mul(std::integral_constant<int, 0>{}); break;
      case 1: mul(std::integral_constant<int, 1>{}); break;
      case 2: mul(std::integral_constant<int, 2>{}); break;
      case 3: mul(std::integral_constant<int, 3>{}); break;
      case 4: mul(std::integral_constant<int, 4>{}); break;
      case 5: mul(std::integral_constant<int, 5>{}); break;
      case 6: mul(std::integral_constant<int, 6>{}); break;
      default: mul(std::integral_constant<int, 7>{}); break;
    }
    if constexpr (!INV) dev::xor_planes(r[t + 1], r[t]);
  });
}
// A <-> B: slot bit 0 and the lane half trade places (an involution)
__device__ __forceinline__ void h8_relayout(Regs4& r) {
  static_for<2>([&](auto TT) {
    constexpr int t = 2 * decltype(TT)::value;
    static_for<16>([&](auto P) {
      constexpr int q = decltype(P)::value;
      const auto s = __builtin_amdgcn_permlane32_swap(r[t][q], r[t + 1][q], false, false);
      r[t][q] = s[0];
      r[t + 1][q] = s[1];
    });
  });
}

// Lane-linear I/O for 32-column tiles (xform_h8): in each half (lanes 0..31, 32..63: two
// positions) lane i reads quarter i & 3 of chunk (i >> 2) + 8 q with instruction q, so every
// instruction streams 512 contiguous bytes per half (when 8 | chunks per shard).  Quarters 0 /
// 1 are the low bytes of symbols 0-15 / 16-31, quarters 2 / 3 the high bytes of the same
// symbols: quad_exchange (lanes i <-> i ^ 2, one DPP quad permute per dword) leaves each lane
// the low and high bytes of 16 symbols of two chunks -- registers 0..7 low bytes, 8..15 high
// bytes, planes_from_raw's input -- and, being an involution, turns computed bytes back into
// the pieces each lane stores.
__device__ __forceinline__ TileIO tile_io_l32(uint64_t total_columns, uint32_t chunks_per_shard, uint64_t tile, int lane,
                                              uint64_t block_stride) {
  TileIO io;
  io.valid = 0;
  const uint32_t i = lane & 31;
  // as tile_io_g: one scalar division per wave, lanes add < 32 chunks
  const uint32_t C = chunks_per_shard;
  const uint64_t g0 = tile * 32;
  const uint64_t b0 = g0 / C;
  const uint32_t r0 = static_cast<uint32_t>(g0 - b0 * C);
  const uint64_t base = b0 * block_stride;
  static_for<4>([&](auto Q) {
    constexpr int q = decltype(Q)::value;
    const uint32_t lc = (i >> 2) + 8 * q;
    const bool ok = g0 + lc < total_columns;
    const uint32_t c = ok ? r0 + lc : r0;  // idle pieces re-read the tile's first chunk, never store
    uint32_t d, rem;
    if (C >= 32) {
      d = c >= C ? 1u : 0u;
      rem = d ? c - C : c;
    } else {
      d = c / C;
      rem = c - d * C;
    }
    io.blk[q] = b0 + d;
    io.off[q] = base + d * block_stride + static_cast<uint64_t>(rem) * 64 + 16 * (i & 3);
    io.valid |= ok ? (1u << q) : 0u;
  });
  return io;
}
__device__ __forceinline__ void quad_exchange(uint32_t* v, int lane) {
  const bool lo = (lane & 2) == 0;  // quarters 0, 1 keep registers 0..7
  static_for<8>([&](auto D) {
    constexpr int d = decltype(D)::value;
    const uint32_t a = v[d], b = v[8 + d];  // selects, not a pointer choice (keeps v in VGPRs)
    const uint32_t recv = static_cast<uint32_t>(
        __builtin_amdgcn_mov_dpp(static_cast<int>(lo ? b : a), 0x4E /* quad_perm 2,3,0,1 */, 0xF, 0xF, false));
    v[d] = lo ? a : recv;
    v[8 + d] = lo ? recv : b;
  });
}

}  // namespace
}  // namespace ag
