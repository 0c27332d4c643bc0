// Device-side building blocks shared by the HIP kernels (gfx950 / CDNA4 only).
//
// Bitsliced GF(2^16): a 64-byte chunk of a shard holds 32 symbols (crate layout:
// byte j = low byte, byte 32 + j = high byte of symbol j).  One lane
// transposes its chunk into 16 bit-planes (uint32 word p holds bit p of all 32 symbols);
// an FFT butterfly's constant multiply then becomes a 16x16 GF(2) XOR network over
// planes, evaluated with v_bitop3_b32 (3-input XOR), ~2 VALU ops per symbol-multiply.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>

#include "rs_consts.inc"

namespace ag {
namespace dev {

// ---- compile-time loops ----------------------------------------------------------
template <typename F, int... Is>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// acc ^ XOR_{i in MASK} y[i], pairing terms into 3-input XORs.
template <unsigned MASK>
__device__ __forceinline__ uint32_t xsum(uint32_t acc, const uint32_t* y) {
  if constexpr (MASK == 0) {
    return acc;
  } else {
    constexpr int i = __builtin_ctz(MASK);
    constexpr unsigned rest = MASK & (MASK - 1);
    if constexpr (rest == 0) {
      return acc ^ y[i];
    } else {
      constexpr int j = __builtin_ctz(rest);
      return xsum<rest & (rest - 1)>(xor3(acc, y[i], y[j]), y);
    }
  }
}

// acc ^ XOR_{i in MASK} s[i] over a 64-bit signal mask, 3-input XORs.
template <uint64_t MASK>
__device__ __forceinline__ uint32_t xsum64(uint32_t acc, const uint32_t* s) {
  if constexpr (MASK == 0) {
    return acc;
  } else {
    constexpr int i = __builtin_ctzll(MASK);
    constexpr uint64_t rest = MASK & (MASK - 1);
    if constexpr (rest == 0) {
      return acc ^ s[i];
    } else {
      constexpr int j = __builtin_ctzll(rest);
      return xsum64<rest & (rest - 1)>(xor3(acc, s[i], s[j]), s);
    }
  }
}

// x ^= y * skew[S]   (bitsliced; S is a compile-time skew index).  Shared sub-sums of the
// 16x16 network (kCse*, gen_consts.cpp) are computed once: ~36 VALU ops on average.
// TAB 0: the cheapest programs (subset and cancellation greedies, ~32.8 VALU); TAB 1: the
// subset greedy's (~35.2), for decode_c and decode_pk, whose register allocation spills with
// TAB 0.
template <int S, int TAB = 0>
__device__ __forceinline__ void mul_acc(uint32_t* x, const uint32_t* y) {
  static_assert(S >= 0 && S < kSkewConstCount, "skew index outside generated table");
  constexpr int NT = TAB ? kCseSubNTemps[S] : kCseNTemps[S];
  uint32_t sig[16 + (kCseMaxTemps > kCseSubMaxTemps ? kCseMaxTemps : kCseSubMaxTemps)];
  static_for<16>([&](auto I) { sig[decltype(I)::value] = y[decltype(I)::value]; });
  static_for<NT>([&](auto J) {
    constexpr int j = decltype(J)::value;
    constexpr int a = TAB ? kCseSubTemp[S][j][0] : kCseTemp[S][j][0];
    constexpr int b = TAB ? kCseSubTemp[S][j][1] : kCseTemp[S][j][1];
    constexpr int c = TAB ? kCseSubTemp[S][j][2] : kCseTemp[S][j][2];
    if constexpr (c == 255) sig[16 + j] = sig[a] ^ sig[b]; else sig[16 + j] = xor3(sig[a], sig[b], sig[c]);
  });
  static_for<16>([&](auto O) {
    constexpr int o = decltype(O)::value;
    x[o] = xsum64<TAB ? kCseSubRow[S][o] : kCseRow[S][o]>(x[o], sig);
  });
}

// out = B x for the basis changes of rs_consts.inc (B = 0: Cantor -> polynomial basis,
// 1: back), out of place, as a CSE'd XOR network.
template <int B>
__device__ __forceinline__ void basis_apply(const uint32_t* x, uint32_t* out) {
  constexpr int NT = kBasisNTemps[B];
  uint32_t sig[16 + kBasisMaxTemps];
  static_for<16>([&](auto I) { sig[decltype(I)::value] = x[decltype(I)::value]; });
  static_for<NT>([&](auto J) {
    constexpr int j = decltype(J)::value;
    constexpr int a = kBasisTemp[B][j][0], b = kBasisTemp[B][j][1], c = kBasisTemp[B][j][2];
    if constexpr (c == 255) sig[16 + j] = sig[a] ^ sig[b]; else sig[16 + j] = xor3(sig[a], sig[b], sig[c]);
  });
  static_for<16>([&](auto O) {
    constexpr int o = decltype(O)::value;
    constexpr uint64_t row = kBasisRow[B][o];
    constexpr int first = __builtin_ctzll(row);
    out[o] = xsum64<row & (row - 1)>(sig[first], sig);
  });
}

// x <- c x for a runtime constant c that differs per lane (per-lane erasure patterns).
// `coef` holds c in the polynomial basis (bit i: coefficient of a^i).  Horner over the 16
// coefficients in the polynomial basis, where a multiply by a is a plane shift plus 3
// XORs (a^16 = a^5 + a^3 + a^2 + 1): 16 x 16 masked XORs, 45 XORs, 16 masks and the two
// basis changes (~70 XORs), against 256 masks + 256 masked XORs for a row matrix.
__device__ __forceinline__ void mul_rt_poly(uint32_t* x, uint32_t coef) {
  uint32_t X[16], acc[16];
  basis_apply<0>(x, X);
  {
    const uint32_t m = static_cast<uint32_t>(__builtin_amdgcn_sbfe(static_cast<int>(coef), 15, 1));
    static_for<16>([&](auto P) { acc[decltype(P)::value] = X[decltype(P)::value] & m; });
  }
  static_for<15>([&](auto I) {
    constexpr int i = 14 - decltype(I)::value;
    const uint32_t top = acc[15];
    static_for<15>([&](auto P) {
      constexpr int q = 15 - decltype(P)::value;  // 15 .. 1
      acc[q] = acc[q - 1];
    });
    acc[0] = top;
    acc[2] ^= top;
    acc[3] ^= top;
    acc[5] ^= top;
    const uint32_t m = static_cast<uint32_t>(__builtin_amdgcn_sbfe(static_cast<int>(coef), i, 1));
    static_for<16>([&](auto P) {
      constexpr int q = decltype(P)::value;
      acc[q] = __builtin_amdgcn_bitop3_b32(acc[q], X[q], m, 0x78);  // acc ^ (X & m)
    });
  });
  basis_apply<1>(acc, x);
}

// x <- c x for a wave-uniform runtime constant c (polynomial basis, as mul_rt_poly): the same
// Horner scheme with the coefficient bits tested on the scalar unit, so a clear bit costs no
// vector work (~45 XORs of doublings + 16 per set bit + the two basis changes, against
// mul_rt_poly's 16 masked XORs per bit).
__device__ __forceinline__ void mul_rt_poly_u(uint32_t* x, uint32_t coef) {
  const uint32_t c = __builtin_amdgcn_readfirstlane(coef);
  uint32_t X[16], acc[16];
  basis_apply<0>(x, X);
  static_for<16>([&](auto P) { acc[decltype(P)::value] = ((c >> 15) & 1) ? X[decltype(P)::value] : 0u; });
  static_for<15>([&](auto I) {  // unrolled: every index static (a runtime loop sent x to scratch)
    constexpr int i = 14 - decltype(I)::value;
    const uint32_t t = acc[15];
    static_for<15>([&](auto P) {
      constexpr int q = 15 - decltype(P)::value;  // 15 .. 1
      acc[q] = acc[q - 1];
    });
    acc[0] = t;
    acc[2] ^= t;
    acc[3] ^= t;
    acc[5] ^= t;
    if ((c >> i) & 1) static_for<16>([&](auto P) { acc[decltype(P)::value] ^= X[decltype(P)::value]; });
  });
  basis_apply<1>(acc, x);
}

// the polynomial-basis form of a Cantor-coordinate element (host or device)
__host__ __device__ constexpr uint32_t to_poly(uint32_t c) {
  uint32_t r = 0;
  for (int o = 0; o < 16; ++o) r |= static_cast<uint32_t>(__builtin_popcount(kBasisMat[0][o] & c) & 1) << o;
  return r;
}

__device__ __forceinline__ void xor_planes(uint32_t* y, const uint32_t* x) {
  static_for<16>([&](auto P) {
    constexpr int p = decltype(P)::value;
    y[p] ^= x[p];
  });
}

// FFT butterfly (crate fft_butterfly_two): x ^= y * skew; y ^= x.
template <int S, int TAB = 0>
__device__ __forceinline__ void fft_bfly(uint32_t* x, uint32_t* y) {
  if constexpr (kSkewLog[S] != 65535) mul_acc<S, TAB>(x, y);
  xor_planes(y, x);
}
// IFFT butterfly (crate ifft_butterfly_two): y ^= x; x ^= y * skew.
template <int S, int TAB = 0>
__device__ __forceinline__ void ifft_bfly(uint32_t* x, uint32_t* y) {
  xor_planes(y, x);
  if constexpr (kSkewLog[S] != 65535) mul_acc<S, TAB>(x, y);
}

// ---- XCD-aware tile order ----------------------------------------------------------
// Workgroups are dispatched round-robin over the 8 XCDs (XCD = b % 8).  xcd_tile gives
// each XCD one contiguous range of tiles, so the tiles in flight on one XCD are HBM
// neighbours (tools/membench/membench4.hip: 32-shard tile copies 5.18 -> 5.49 TB/s at 64
// chunks per tile, 5.76 -> 6.20 TB/s at 16).  A bijection on [0, g) for any g.
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t g) {
  const uint32_t x = b & 7, q = g >> 3, r = g & 7;
  return x * q + (x < r ? x : r) + (b >> 3);
}

// ---- 8x32 bit transpose (3 delta swaps; an involution) ------------------------------
// In: x[r] byte y = byte (4r + y) of a 32-byte plane group.  Out: x[b] bit (8y + r) =
// bit b of that byte.  Any fixed bijection of symbol positions is fine because all
// arithmetic is per symbol position; the inverse is the same network.
// bfi(m, x, y) = (m & x) | (~m & y) as one v_bitop3_b32 (truth table 0xCA).
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t x, uint32_t y) {
  return __builtin_amdgcn_bitop3_b32(m, x, y, 0xCA);
}
__device__ __forceinline__ void swap_bits(uint32_t& a, uint32_t& b, int sh, uint32_t m) {
  const uint32_t na = bfi(m, a, b << sh);
  const uint32_t nb = bfi(m, a >> sh, b);
  a = na;
  b = nb;
}
__device__ __forceinline__ void transpose8(uint32_t* x) {
  swap_bits(x[0], x[4], 4, 0x0F0F0F0Fu);
  swap_bits(x[1], x[5], 4, 0x0F0F0F0Fu);
  swap_bits(x[2], x[6], 4, 0x0F0F0F0Fu);
  swap_bits(x[3], x[7], 4, 0x0F0F0F0Fu);
  swap_bits(x[0], x[2], 2, 0x33333333u);
  swap_bits(x[1], x[3], 2, 0x33333333u);
  swap_bits(x[4], x[6], 2, 0x33333333u);
  swap_bits(x[5], x[7], 2, 0x33333333u);
  swap_bits(x[0], x[1], 1, 0x55555555u);
  swap_bits(x[2], x[3], 1, 0x55555555u);
  swap_bits(x[4], x[5], 1, 0x55555555u);
  swap_bits(x[6], x[7], 1, 0x55555555u);
}

// 64-byte chunk <-> 16 planes (planes 0..7 = low-byte bits, 8..15 = high-byte bits).
__device__ __forceinline__ void load_chunk(const uint8_t* __restrict__ src, uint32_t* v) {
  const uint4* s = reinterpret_cast<const uint4*>(src);
  const uint4 a = s[0], b = s[1], c = s[2], d = s[3];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  v[8] = c.x; v[9] = c.y; v[10] = c.z; v[11] = c.w;
  v[12] = d.x; v[13] = d.y; v[14] = d.z; v[15] = d.w;
}
__device__ __forceinline__ void planes_from_raw(uint32_t* v) {
  transpose8(v);
  transpose8(v + 8);
}
using u32x4 = uint32_t __attribute__((ext_vector_type(4)));

// NT: non-temporal stores (streamed once; keeps L2 for the loads).  ACC: XOR into the bytes
// already at dst (a partial result stored by an earlier pass).
template <bool NT = false, bool ACC = false>
__device__ __forceinline__ void store_chunk(uint8_t* __restrict__ dst, const uint32_t* planes) {
  uint32_t v[16];
  static_for<16>([&](auto P) {
    constexpr int p = decltype(P)::value;
    v[p] = planes[p];
  });
  transpose8(v);
  transpose8(v + 8);
  u32x4* d = reinterpret_cast<u32x4*>(dst);
  static_for<4>([&](auto Q) {
    constexpr int q = decltype(Q)::value;
    u32x4 x = {v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
    if constexpr (ACC) x ^= d[q];
    if constexpr (NT) {
      __builtin_nontemporal_store(x, d + q);
    } else {
      d[q] = x;
    }
  });
}

// ---- table arithmetic for the generic (any-geometry) kernels ------------------------
__device__ __forceinline__ uint16_t add_mod(uint32_t x, uint32_t y) {
  const uint32_t s = x + y;
  return static_cast<uint16_t>(s + (s >> 16));
}
__device__ __forceinline__ uint16_t sub_mod(uint32_t x, uint32_t y) {
  const uint32_t d = x - y;
  return static_cast<uint16_t>(d + (d >> 16));
}
__device__ __forceinline__ uint16_t gmul(const uint16_t* __restrict__ exp_t,
                                         const uint16_t* __restrict__ log_t, uint16_t x,
                                         uint16_t log_m) {
  return x == 0 ? uint16_t(0) : exp_t[add_mod(log_t[x], log_m)];
}

}  // namespace dev
}  // namespace ag
