// Ed25519 arithmetic shared by the kernels (ed25519.hip) -- header-only, __host__ __device__
// so the same code is also compiled into a host check binary (tests/ed_host_check.cpp: test
// infrastructure; the library's entry points only launch the kernels).
//
// What the reference computes (crypto/signature.rs:60-104 over ed25519-zebra 4.2.0 /
// curve25519-dalek 4.1.3, neither vendored): RFC 8032 keygen / sign and ZIP-215 verify
// (canonical s, non-canonical A / R accepted, cofactored equation).  Restated here from the
// published algorithms:
//
//   field  GF(2^255 - 19), ten signed limbs of 26/25 bits (radix 2^25.5), int64 products
//          (v_mad_i64_i32); carries round to nearest so a reduced limb is |x| <= 2^25 / 2^24.
//          Bound rule: fe_mul(f, g) takes g at most 3x a reduced element (19*g fits int32)
//          and f * g at most ~60x; every formula below stays inside that (noted per step).
//   group  twisted Edwards a = -1, extended coordinates (Hisil-Wong-Carter-Dawson 2008):
//          P2 (X:Y:Z), P3 (X:Y:Z:T), P1 "completed" ((X:Z), (Y:T)), Cached (Y+X, Y-X, Z, 2dT),
//          Precomp affine (y+x, y-x, 2dxy).
//   scalar mod l = 2^252 + 27742317777372353535851937790883648493: bit-serial reduction
//          (one 512-bit digest per signature -- a few % of the scalar multiplication).
//   SHA-512 FIPS 180-4 (k = H(R || A || M), RFC 8032 nonce / key expansion).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace ag {
namespace ed {

#define ED_INL __host__ __device__ inline __attribute__((always_inline))

struct Fe {
  int32_t v[10];
};

// 256-bit little-endian constants as eight 32-bit words
struct W8 {
  uint32_t w[8];
};

constexpr int kOff[10] = {0, 26, 51, 77, 102, 128, 153, 179, 204, 230};
constexpr int kBits[10] = {26, 25, 26, 25, 26, 25, 26, 25, 26, 25};

// 255 low bits of a little-endian 256-bit value -> limbs (value may be >= p: arithmetic is
// mod p regardless; this is how dalek reads a non-canonical y).
ED_INL constexpr Fe fe_from_words(const W8& x) {
  Fe f{};
  for (int i = 0; i < 10; ++i) {
    const int o = kOff[i], wi = o >> 5, sh = o & 31;
    uint64_t v = x.w[wi];
    if (wi < 7) v |= static_cast<uint64_t>(x.w[wi + 1]) << 32;
    v >>= sh;
    f.v[i] = static_cast<int32_t>(v & ((1u << kBits[i]) - 1));
  }
  return f;
}

constexpr W8 kD{{0x135978a3, 0x75eb4dca, 0x4141d8ab, 0x00700a4d, 0x7779e898, 0x8cc74079, 0x2b6ffe73, 0x52036cee}};
constexpr W8 kD2{{0x26b2f159, 0xebd69b94, 0x8283b156, 0x00e0149a, 0xeef3d130, 0x198e80f2, 0x56dffce7, 0x2406d9dc}};
constexpr W8 kSqrtM1{{0x4a0ea0b0, 0xc4ee1b27, 0xad2fe478, 0x2f431806, 0x3dfbd7a7, 0x2b4d0099, 0x4fc1df0b, 0x2b832480}};
constexpr W8 kBx{{0x8f25d51a, 0xc9562d60, 0x9525a7b2, 0x692cc760, 0xfdd6dc5c, 0xc0a4e231, 0xcd6e53fe, 0x216936d3}};
constexpr W8 kBy{{0x66666658, 0x66666666, 0x66666666, 0x66666666, 0x66666666, 0x66666666, 0x66666666, 0x66666666}};
constexpr W8 kL{{0x5cf5d3ed, 0x5812631a, 0xa2f79cd6, 0x14def9de, 0x00000000, 0x00000000, 0x00000000, 0x10000000}};

// ---- field -------------------------------------------------------------------------------

ED_INL void fe_carry(int64_t h[10], Fe& o) {
  int64_t c;
  c = (h[0] + (int64_t{1} << 25)) >> 26; h[1] += c; h[0] -= c * (int64_t{1} << 26);
  c = (h[4] + (int64_t{1} << 25)) >> 26; h[5] += c; h[4] -= c * (int64_t{1} << 26);
  c = (h[1] + (int64_t{1} << 24)) >> 25; h[2] += c; h[1] -= c * (int64_t{1} << 25);
  c = (h[5] + (int64_t{1} << 24)) >> 25; h[6] += c; h[5] -= c * (int64_t{1} << 25);
  c = (h[2] + (int64_t{1} << 25)) >> 26; h[3] += c; h[2] -= c * (int64_t{1} << 26);
  c = (h[6] + (int64_t{1} << 25)) >> 26; h[7] += c; h[6] -= c * (int64_t{1} << 26);
  c = (h[3] + (int64_t{1} << 24)) >> 25; h[4] += c; h[3] -= c * (int64_t{1} << 25);
  c = (h[7] + (int64_t{1} << 24)) >> 25; h[8] += c; h[7] -= c * (int64_t{1} << 25);
  c = (h[4] + (int64_t{1} << 25)) >> 26; h[5] += c; h[4] -= c * (int64_t{1} << 26);
  c = (h[8] + (int64_t{1} << 25)) >> 26; h[9] += c; h[8] -= c * (int64_t{1} << 26);
  c = (h[9] + (int64_t{1} << 24)) >> 25; h[0] += c * 19; h[9] -= c * (int64_t{1} << 25);
  c = (h[0] + (int64_t{1} << 25)) >> 26; h[1] += c; h[0] -= c * (int64_t{1} << 26);
#pragma unroll
  for (int i = 0; i < 10; ++i) o.v[i] = static_cast<int32_t>(h[i]);
}

ED_INL void fe_norm(Fe& f) {
  int64_t h[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) h[i] = f.v[i];
  fe_carry(h, f);
}

ED_INL void fe_add(Fe& o, const Fe& a, const Fe& b) {
#pragma unroll
  for (int i = 0; i < 10; ++i) o.v[i] = a.v[i] + b.v[i];
}
ED_INL void fe_sub(Fe& o, const Fe& a, const Fe& b) {
#pragma unroll
  for (int i = 0; i < 10; ++i) o.v[i] = a.v[i] - b.v[i];
}
ED_INL void fe_neg(Fe& o, const Fe& a) {
#pragma unroll
  for (int i = 0; i < 10; ++i) o.v[i] = -a.v[i];
}
ED_INL Fe fe_zero() { return Fe{}; }
ED_INL Fe fe_one() {
  Fe f{};
  f.v[0] = 1;
  return f;
}
// o = c ? b : a (no branch)
ED_INL void fe_select(Fe& o, const Fe& a, const Fe& b, bool c) {
#pragma unroll
  for (int i = 0; i < 10; ++i) o.v[i] = c ? b.v[i] : a.v[i];
}

ED_INL void fe_mul(Fe& o, const Fe& f, const Fe& g) {
  int32_t g19[10], f2[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    g19[i] = 19 * g.v[i];
    f2[i] = (i & 1) ? 2 * f.v[i] : f.v[i];
  }
  int64_t h[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 10; ++i) {
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      const int32_t a = ((i & 1) && (j & 1)) ? f2[i] : f.v[i];
      const int32_t b = (i + j >= 10) ? g19[j] : g.v[j];
      h[(i + j) % 10] += static_cast<int64_t>(a) * b;
    }
  }
  fe_carry(h, o);
}

// o = f^2 (times 2 if dbl): 55 products
ED_INL void fe_sq_impl(Fe& o, const Fe& f, bool dbl) {
  int32_t f19[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) f19[i] = 19 * f.v[i];
  int64_t h[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 10; ++i) {
#pragma unroll
    for (int j = i; j < 10; ++j) {
      const int sc = ((i != j) ? 2 : 1) * (((i & 1) && (j & 1)) ? 2 : 1);
      const int32_t a = sc * f.v[i];
      const int32_t b = (i + j >= 10) ? f19[j] : f.v[j];
      h[(i + j) % 10] += static_cast<int64_t>(a) * b;
    }
  }
  if (dbl) {
#pragma unroll
    for (int i = 0; i < 10; ++i) h[i] *= 2;
  }
  fe_carry(h, o);
}
ED_INL void fe_sq(Fe& o, const Fe& f) { fe_sq_impl(o, f, false); }
ED_INL void fe_sq2(Fe& o, const Fe& f) { fe_sq_impl(o, f, true); }
ED_INL void fe_sqn(Fe& o, const Fe& f, int n) {
  fe_sq(o, f);
  for (int i = 1; i < n; ++i) fe_sq(o, o);
}

// canonical value in [0, p) as eight little-endian words
ED_INL void fe_to_words(const Fe& f, uint32_t out[8]) {
  int64_t h[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) h[i] = f.v[i];
#pragma unroll
  for (int pass = 0; pass < 3; ++pass) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      const int64_t c = h[i] >> kBits[i];
      h[i] -= c * (int64_t{1} << kBits[i]);
      if (i < 9) h[i + 1] += c;
      else h[0] += 19 * c;
    }
  }
  // value v in [0, 2^255): v >= p iff v + 19 >= 2^255
  int64_t t[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) t[i] = h[i];
  t[0] += 19;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int64_t c = t[i] >> kBits[i];
    t[i] -= c * (int64_t{1} << kBits[i]);
    t[i + 1] += c;
  }
  const int64_t top = t[9] >> 25;
  t[9] -= top * (int64_t{1} << 25);
#pragma unroll
  for (int i = 0; i < 10; ++i) h[i] = top ? t[i] : h[i];
  uint64_t acc = 0;
  int nb = 0, wi = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    acc |= static_cast<uint64_t>(h[i]) << nb;
    nb += kBits[i];
    if (nb >= 32) {
      out[wi++] = static_cast<uint32_t>(acc);
      acc >>= 32;
      nb -= 32;
    }
  }
  out[7] = static_cast<uint32_t>(acc);
}

ED_INL bool fe_is_zero(const Fe& f) {
  uint32_t w[8];
  fe_to_words(f, w);
  uint32_t a = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) a |= w[i];
  return a == 0;
}
ED_INL bool fe_is_odd(const Fe& f) {
  uint32_t w[8];
  fe_to_words(f, w);
  return w[0] & 1;
}

// z^(2^250 - 1) and z^11 (shared prefix of inversion and the square-root power)
ED_INL void fe_pow_chain(const Fe& z, Fe& z2_250_0, Fe& z11) {
  Fe z2, z9, t, z2_5_0, z2_10_0, z2_20_0, z2_50_0, z2_100_0;
  fe_sq(z2, z);                // 2
  fe_sqn(t, z2, 2);            // 8
  fe_mul(z9, t, z);            // 9
  fe_mul(z11, z9, z2);         // 11
  fe_sq(t, z11);               // 22
  fe_mul(z2_5_0, t, z9);       // 2^5 - 1
  fe_sqn(t, z2_5_0, 5);
  fe_mul(z2_10_0, t, z2_5_0);  // 2^10 - 1
  fe_sqn(t, z2_10_0, 10);
  fe_mul(z2_20_0, t, z2_10_0);
  fe_sqn(t, z2_20_0, 20);
  fe_mul(t, t, z2_20_0);       // 2^40 - 1
  fe_sqn(t, t, 10);
  fe_mul(z2_50_0, t, z2_10_0);
  fe_sqn(t, z2_50_0, 50);
  fe_mul(z2_100_0, t, z2_50_0);
  fe_sqn(t, z2_100_0, 100);
  fe_mul(t, t, z2_100_0);      // 2^200 - 1
  fe_sqn(t, t, 50);
  fe_mul(z2_250_0, t, z2_50_0);
}
ED_INL void fe_invert(Fe& o, const Fe& z) {  // z^(p-2) = z^(2^255 - 21)
  Fe a, z11;
  fe_pow_chain(z, a, z11);
  fe_sqn(a, a, 5);
  fe_mul(o, a, z11);
}
ED_INL void fe_pow22523(Fe& o, const Fe& z) {  // z^((p-5)/8) = z^(2^252 - 3)
  Fe a, z11;
  fe_pow_chain(z, a, z11);
  fe_sqn(a, a, 2);
  fe_mul(o, a, z);
}

// ---- group -------------------------------------------------------------------------------

struct P2 {
  Fe X, Y, Z;
};
struct P3 {
  Fe X, Y, Z, T;
};
struct P1 {
  Fe X, Y, Z, T;
};
struct Cached {
  Fe YpX, YmX, Z, T2d;
};
struct Precomp {
  Fe ypx, ymx, xy2d;
};

ED_INL void p1_to_p2(P2& r, const P1& p) {
  fe_mul(r.X, p.T, p.X);  // f = T (3x), g = X (3x)
  fe_mul(r.Y, p.Z, p.Y);
  fe_mul(r.Z, p.T, p.Z);
}
ED_INL void p1_to_p3(P3& r, const P1& p) {
  fe_mul(r.X, p.T, p.X);
  fe_mul(r.Y, p.Z, p.Y);
  fe_mul(r.Z, p.T, p.Z);
  fe_mul(r.T, p.X, p.Y);
}
ED_INL void p3_to_p2(P2& r, const P3& p) {
  r.X = p.X;
  r.Y = p.Y;
  r.Z = p.Z;
}
ED_INL P3 p3_identity() {
  P3 r;
  r.X = fe_zero();
  r.Y = fe_one();
  r.Z = fe_one();
  r.T = fe_zero();
  return r;
}
ED_INL Cached cached_identity() {
  Cached c;
  c.YpX = fe_one();
  c.YmX = fe_one();
  c.Z = fe_one();
  c.T2d = fe_zero();
  return c;
}
ED_INL void p3_to_cached(Cached& c, const P3& p) {
  constexpr Fe d2 = fe_from_words(kD2);
  fe_add(c.YpX, p.Y, p.X);
  fe_sub(c.YmX, p.Y, p.X);
  fe_norm(c.YpX);
  fe_norm(c.YmX);
  c.Z = p.Z;
  fe_mul(c.T2d, p.T, d2);
}

// dbl-2008-hwcd: r = 2p (completed)
ED_INL void p2_dbl(P1& r, const P2& p) {
  Fe t0;
  fe_sq(r.X, p.X);
  fe_sq(r.Z, p.Y);
  fe_sq2(r.T, p.Z);
  fe_add(r.Y, p.X, p.Y);   // 2x
  fe_sq(t0, r.Y);
  fe_add(r.Y, r.Z, r.X);   // 2x
  fe_sub(r.Z, r.Z, r.X);   // 2x
  fe_sub(r.X, t0, r.Y);    // 3x
  fe_sub(r.T, r.T, r.Z);   // 3x
}

// add-2008-hwcd-3: r = p + q, q cached; neg: r = p - q
ED_INL void p3_add(P1& r, const P3& p, const Cached& q) {
  Fe t0;
  fe_add(r.X, p.Y, p.X);
  fe_sub(r.Y, p.Y, p.X);
  fe_mul(r.Z, r.X, q.YpX);  // 2x * 1x
  fe_mul(r.Y, r.Y, q.YmX);
  fe_mul(r.T, q.T2d, p.T);
  fe_mul(r.X, p.Z, q.Z);
  fe_add(t0, r.X, r.X);     // 2x
  fe_sub(r.X, r.Z, r.Y);    // 2x
  fe_add(r.Y, r.Z, r.Y);    // 2x
  fe_add(r.Z, t0, r.T);     // 3x
  fe_sub(r.T, t0, r.T);     // 3x
}
// mixed add with an affine precomputed point
ED_INL void p3_madd(P1& r, const P3& p, const Precomp& q) {
  Fe t0;
  fe_add(r.X, p.Y, p.X);
  fe_sub(r.Y, p.Y, p.X);
  fe_mul(r.Z, r.X, q.ypx);
  fe_mul(r.Y, r.Y, q.ymx);
  fe_mul(r.T, q.xy2d, p.T);
  fe_add(t0, p.Z, p.Z);
  fe_sub(r.X, r.Z, r.Y);
  fe_add(r.Y, r.Z, r.Y);
  fe_add(r.Z, t0, r.T);
  fe_sub(r.T, t0, r.T);
}
// negation of a cached / precomputed point: swap Y+X and Y-X, negate the T term
ED_INL void cached_cneg(Cached& c, bool neg) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const int32_t a = c.YpX.v[i], b = c.YmX.v[i];
    c.YpX.v[i] = neg ? b : a;
    c.YmX.v[i] = neg ? a : b;
    c.T2d.v[i] = neg ? -c.T2d.v[i] : c.T2d.v[i];
  }
}
ED_INL void precomp_cneg(Precomp& c, bool neg) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const int32_t a = c.ypx.v[i], b = c.ymx.v[i];
    c.ypx.v[i] = neg ? b : a;
    c.ymx.v[i] = neg ? a : b;
    c.xy2d.v[i] = neg ? -c.xy2d.v[i] : c.xy2d.v[i];
  }
}

ED_INL void p3_dbl(P3& r, const P3& p) {
  P2 q;
  P1 t;
  p3_to_p2(q, p);
  p2_dbl(t, q);
  p1_to_p3(r, t);
}

// compressed encoding: y with x's parity in bit 255
ED_INL void p3_compress(uint32_t out[8], const P3& p) {
  Fe zi, x, y;
  fe_invert(zi, p.Z);
  fe_mul(x, p.X, zi);
  fe_mul(y, p.Y, zi);
  fe_to_words(y, out);
  out[7] |= static_cast<uint32_t>(fe_is_odd(x)) << 31;
}

ED_INL void p3_to_precomp(Precomp& c, const P3& p) {
  constexpr Fe d2 = fe_from_words(kD2);
  Fe zi, x, y, xy;
  fe_invert(zi, p.Z);
  fe_mul(x, p.X, zi);
  fe_mul(y, p.Y, zi);
  fe_add(c.ypx, y, x);
  fe_sub(c.ymx, y, x);
  fe_norm(c.ypx);
  fe_norm(c.ymx);
  fe_mul(xy, x, y);
  fe_mul(c.xy2d, xy, d2);
}

// CompressedEdwardsY::decompress (curve25519-dalek 4.1): y = low 255 bits (reduced mod p,
// non-canonical accepted), x = sqrt((y^2 - 1) / (d y^2 + 1)) (nonnegative root), then x's
// sign from bit 255 -- with no rejection of sign = 1 at x = 0 (ZIP-215).  False when
// (y^2 - 1) / (d y^2 + 1) is not a square.
ED_INL bool p3_decompress(P3& r, const uint32_t in[8]) {
  constexpr Fe d = fe_from_words(kD);
  constexpr Fe sqrtm1 = fe_from_words(kSqrtM1);
  W8 w{};
#pragma unroll
  for (int i = 0; i < 8; ++i) w.w[i] = in[i];
  const bool sign = in[7] >> 31;
  r.Y = fe_from_words(w);
  r.Z = fe_one();
  Fe u, v, v3, vxx, check, x;
  fe_sq(u, r.Y);
  fe_mul(v, u, d);
  u.v[0] -= 1;      // u = y^2 - 1
  v.v[0] += 1;      // v = d y^2 + 1
  fe_sq(v3, v);
  fe_mul(v3, v3, v);  // v^3
  fe_sq(x, v3);
  fe_mul(x, x, v);
  fe_mul(x, x, u);    // u v^7
  fe_pow22523(x, x);  // (u v^7)^((p-5)/8)
  fe_mul(x, x, v3);
  fe_mul(x, x, u);    // u v^3 (u v^7)^((p-5)/8)
  fe_sq(vxx, x);
  fe_mul(vxx, vxx, v);
  fe_sub(check, vxx, u);
  const bool direct = fe_is_zero(check);
  fe_add(check, vxx, u);
  const bool flipped = fe_is_zero(check);
  if (!direct && !flipped) return false;
  if (!direct) fe_mul(x, x, sqrtm1);
  const bool odd = fe_is_odd(x);
  if (odd != sign) fe_neg(x, x);  // |x| then the sign bit: x -> -x exactly when parity != sign
  fe_norm(x);
  r.X = x;
  fe_mul(r.T, r.X, r.Y);
  return true;
}

// ---- scalars -------------------------------------------------------------------------------

// r = (sum of nbits bits of x, most significant first) mod l; x little-endian 32-bit words.
ED_INL void sc_reduce_words(const uint32_t* x, int nwords, uint32_t r[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = 0;
  for (int wi = nwords - 1; wi >= 0; --wi) {
    const uint32_t word = x[wi];
    for (int b = 31; b >= 0; --b) {
      // r = 2r + bit  (r < l < 2^253: no overflow)
      uint32_t carry = (word >> b) & 1;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint32_t nc = r[i] >> 31;
        r[i] = (r[i] << 1) | carry;
        carry = nc;
      }
      // r -= l if r >= l
      uint32_t t[8];
      uint64_t borrow = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint64_t d = static_cast<uint64_t>(r[i]) - kL.w[i] - borrow;
        t[i] = static_cast<uint32_t>(d);
        borrow = (d >> 32) & 1;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) r[i] = borrow ? r[i] : t[i];
    }
  }
}

ED_INL bool sc_is_canonical(const uint32_t s[8]) {  // s < l
  uint64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t d = static_cast<uint64_t>(s[i]) - kL.w[i] - borrow;
    borrow = (d >> 32) & 1;
  }
  return borrow != 0;
}

// signed radix-16 digits of s < 2^253: digit i = nibble_i(s + 0x88..8) - 8 in [-8, 7],
// kept as the 256-bit value s + 0x88..8 (digit extraction is a shift and a subtract).
ED_INL void sc_recode(const uint32_t s[8], uint32_t out[8]) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t t = static_cast<uint64_t>(s[i]) + 0x88888888u + c;
    out[i] = static_cast<uint32_t>(t);
    c = t >> 32;
  }
}
ED_INL int sc_digit(uint32_t word, int j) { return static_cast<int>((word >> (4 * j)) & 15) - 8; }

// ---- SHA-512 -------------------------------------------------------------------------------

namespace sha512 {
constexpr uint64_t kK[80] = {
    0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull, 0x3956c25bf348b538ull,
    0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull, 0xd807aa98a3030242ull, 0x12835b0145706fbeull,
    0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull, 0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull,
    0xc19bf174cf692694ull, 0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
    0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull, 0x983e5152ee66dfabull,
    0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull, 0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull,
    0x06ca6351e003826full, 0x142929670a0e6e70ull, 0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull,
    0x53380d139d95b3dfull, 0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
    0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull, 0xd192e819d6ef5218ull,
    0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull, 0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull,
    0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull, 0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull,
    0x682e6ff3d6b2b8a3ull, 0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
    0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull, 0xca273eceea26619cull,
    0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull, 0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull,
    0x113f9804bef90daeull, 0x1b710b35131c471bull, 0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull,
    0x431d67c49c100d4cull, 0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull};
constexpr uint64_t kIv[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull,
                                                 0xa54ff53a5f1d36f1ull, 0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
                                                 0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};

ED_INL uint64_t rotr(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

ED_INL void compress(uint64_t st[8], uint64_t w[16]) {
  uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  for (int r = 0; r < 80; ++r) {
    uint64_t wr;
    if (r < 16) {
      wr = w[r];
    } else {
      const uint64_t w15 = w[(r + 1) & 15], w2 = w[(r + 14) & 15];
      const uint64_t s0 = rotr(w15, 1) ^ rotr(w15, 8) ^ (w15 >> 7);
      const uint64_t s1 = rotr(w2, 19) ^ rotr(w2, 61) ^ (w2 >> 6);
      wr = w[r & 15] = w[r & 15] + s0 + w[(r + 9) & 15] + s1;
    }
    const uint64_t S1 = rotr(e, 14) ^ rotr(e, 18) ^ rotr(e, 41);
    const uint64_t ch = (e & f) ^ (~e & g);
    const uint64_t t1 = h + S1 + ch + kK[r] + wr;
    const uint64_t S0 = rotr(a, 28) ^ rotr(a, 34) ^ rotr(a, 39);
    const uint64_t mj = (a & b) ^ (a & c) ^ (b & c);
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + S0 + mj;
  }
  st[0] += a;
  st[1] += b;
  st[2] += c;
  st[3] += d;
  st[4] += e;
  st[5] += f;
  st[6] += g;
  st[7] += h;
}

// SHA-512 of the T-byte message whose byte i is byte(i); digest as the integer's eight
// little-endian 64-bit words split into 16 little-endian 32-bit words (the digest bytes read
// as a 512-bit little-endian number, which is how RFC 8032 uses it).
template <typename Byte>
ED_INL void digest_le_words(uint32_t T, Byte&& byte, uint32_t out[16]) {
  uint64_t st[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) st[i] = kIv[i];
  const uint32_t nblk = (T + 17 + 127) / 128;
  for (uint32_t b = 0; b < nblk; ++b) {
    uint64_t w[16];
    for (int j = 0; j < 16; ++j) {
      const uint32_t o = 128 * b + 8 * j;
      uint64_t v = 0;
      if (b == nblk - 1 && j == 15) {
        v = static_cast<uint64_t>(T) * 8;
      } else if (b == nblk - 1 && j == 14) {
        v = 0;
      } else if (o + 8 <= T) {
        for (int k = 0; k < 8; ++k) v = (v << 8) | byte(o + k);
      } else {
        for (int k = 0; k < 8; ++k) {
          const uint32_t ob = o + k;
          const uint32_t bv = ob < T ? byte(ob) : (ob == T ? 0x80u : 0u);
          v = (v << 8) | bv;
        }
      }
      w[j] = v;
    }
    compress(st, w);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    // digest bytes are st[i] big-endian: as a little-endian integer, word i = bswap64(st[i])
    const uint64_t x = st[i];
    uint64_t y = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) y |= ((x >> (8 * k)) & 0xFF) << (8 * (7 - k));
    out[2 * i] = static_cast<uint32_t>(y);
    out[2 * i + 1] = static_cast<uint32_t>(y >> 32);
  }
}
}  // namespace sha512

// 32 bytes (little-endian) -> 8 words
ED_INL void load_words(const uint8_t* p, uint32_t w[8]) {
  for (int i = 0; i < 8; ++i)
    w[i] = uint32_t(p[4 * i]) | (uint32_t(p[4 * i + 1]) << 8) | (uint32_t(p[4 * i + 2]) << 16) |
           (uint32_t(p[4 * i + 3]) << 24);
}
ED_INL void store_words(uint8_t* p, const uint32_t w[8]) {
  for (int i = 0; i < 8; ++i) {
    p[4 * i] = static_cast<uint8_t>(w[i]);
    p[4 * i + 1] = static_cast<uint8_t>(w[i] >> 8);
    p[4 * i + 2] = static_cast<uint8_t>(w[i] >> 16);
    p[4 * i + 3] = static_cast<uint8_t>(w[i] >> 24);
  }
}
ED_INL uint8_t word_byte(const uint32_t w[8], uint32_t i) { return static_cast<uint8_t>(w[i >> 2] >> (8 * (i & 3))); }

// ---- the operations ---------------------------------------------------------------------------

// table: [64][8] Precomp entries (j+1) * 16^i * B as 30 int32 each
ED_INL void load_precomp(Precomp& c, const int32_t* table, int row, int col) {
  const int32_t* e = table + (static_cast<size_t>(row) * 8 + col) * 30;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    c.ypx.v[i] = e[i];
    c.ymx.v[i] = e[10 + i];
    c.xy2d.v[i] = e[20 + i];
  }
}
// digit e in [-8, 8] -> Precomp (identity for 0)
ED_INL void select_precomp(Precomp& c, const int32_t* table, int row, int e) {
  const int a = e < 0 ? -e : e;
  load_precomp(c, table, row, a > 0 ? a - 1 : 0);
  if (a == 0) {
    c.ypx = fe_one();
    c.ymx = fe_one();
    c.xy2d = fe_zero();
  }
  precomp_cneg(c, e < 0);
}

// [s]B for s < 2^253 with the 64-row fixed-base table: 64 mixed additions, no doublings.
ED_INL void scalarmult_base(P3& r, const uint32_t s[8], const int32_t* table) {
  uint32_t rec[8];
  sc_recode(s, rec);
  r = p3_identity();
  for (int i = 0; i < 64; ++i) {
    Precomp q;
    select_precomp(q, table, i, sc_digit(rec[i >> 3], i & 7));
    P1 t;
    p3_madd(t, r, q);
    p1_to_p3(r, t);
  }
}

// RFC 8032 §5.1.5: a = clamp(SHA-512(seed)[0..32)), prefix = [32..64)
ED_INL void expand_seed(const uint8_t* seed, uint32_t a[8], uint32_t prefix[8]) {
  uint32_t h[16];
  sha512::digest_le_words(32, [&](uint32_t i) -> uint32_t { return seed[i]; }, h);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = h[i];
    prefix[i] = h[8 + i];
  }
  a[0] &= ~7u;
  a[7] &= 0x7FFFFFFFu;
  a[7] |= 0x40000000u;
}

ED_INL void public_key(const uint8_t* seed, uint8_t* pk_out, const int32_t* table) {
  uint32_t a[8], prefix[8], am[8], pk[8];
  expand_seed(seed, a, prefix);
  sc_reduce_words(a, 8, am);  // [a]B = [a mod l]B
  P3 A;
  scalarmult_base(A, am, table);
  p3_compress(pk, A);
  store_words(pk_out, pk);
}

// RFC 8032 §5.1.6 (ed25519-zebra SigningKey::sign)
template <typename MsgByte>
ED_INL void sign(const uint8_t* seed, const uint8_t* pk_bytes, uint32_t mlen, MsgByte&& msg, uint8_t* sig_out,
                 const int32_t* table) {
  uint32_t a[8], prefix[8], h[16], r[8], Rw[8], pkw[8], k[8];
  expand_seed(seed, a, prefix);
  load_words(pk_bytes, pkw);
  sha512::digest_le_words(
      32 + mlen, [&](uint32_t i) -> uint32_t { return i < 32 ? word_byte(prefix, i) : msg(i - 32); }, h);
  sc_reduce_words(h, 16, r);
  P3 R;
  scalarmult_base(R, r, table);
  p3_compress(Rw, R);
  sha512::digest_le_words(
      64 + mlen,
      [&](uint32_t i) -> uint32_t { return i < 32 ? word_byte(Rw, i) : (i < 64 ? word_byte(pkw, i - 32) : msg(i - 64)); },
      h);
  sc_reduce_words(h, 16, k);
  // S = (r + k * a) mod l
  uint32_t prod[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) prod[i] = 0;
  for (int i = 0; i < 8; ++i) {
    uint64_t carry = 0;
    for (int j = 0; j < 8; ++j) {
      const uint64_t t = static_cast<uint64_t>(k[i]) * a[j] + prod[i + j] + carry;
      prod[i + j] = static_cast<uint32_t>(t);
      carry = t >> 32;
    }
    prod[i + 8] = static_cast<uint32_t>(carry);
  }
  uint64_t c = 0;
  for (int i = 0; i < 16; ++i) {
    const uint64_t t = static_cast<uint64_t>(prod[i]) + (i < 8 ? r[i] : 0u) + c;
    prod[i] = static_cast<uint32_t>(t);
    c = t >> 32;
  }
  uint32_t S[8];
  sc_reduce_words(prod, 16, S);
  store_words(sig_out, Rw);
  store_words(sig_out + 32, S);
}

// ed25519-zebra VerificationKey::verify (ZIP-215).  tab: scratch for 9 Cached entries.
template <typename MsgByte>
ED_INL bool verify(const uint8_t* pk_bytes, const uint8_t* sig, uint32_t mlen, MsgByte&& msg, const int32_t* table,
                   Cached* tab) {
  uint32_t pkw[8], Rw[8], s[8];
  load_words(pk_bytes, pkw);
  load_words(sig, Rw);
  load_words(sig + 32, s);
  if (!sc_is_canonical(s)) return false;
  P3 A, R;
  if (!p3_decompress(A, pkw)) return false;
  if (!p3_decompress(R, Rw)) return false;
  uint32_t h[16], k[8];
  sha512::digest_le_words(
      64 + mlen,
      [&](uint32_t i) -> uint32_t { return i < 32 ? word_byte(Rw, i) : (i < 64 ? word_byte(pkw, i - 32) : msg(i - 64)); },
      h);
  sc_reduce_words(h, 16, k);
  // table of j * (-A), j = 0..8
  P3 nA = A;
  fe_neg(nA.X, A.X);
  fe_neg(nA.T, A.T);
  tab[0] = cached_identity();
  p3_to_cached(tab[1], nA);
  {
    P3 acc = nA;
    for (int j = 2; j <= 8; ++j) {
      P1 t;
      p3_add(t, acc, tab[1]);
      p1_to_p3(acc, t);
      p3_to_cached(tab[j], acc);
    }
  }
  uint32_t rk[8], rs[8];
  sc_recode(k, rk);
  sc_recode(s, rs);
  // R' = [k](-A) + [s]B, joint signed radix-16 (Straus), 4 doublings per digit
  P3 acc = p3_identity();
  for (int i = 63; i >= 0; --i) {
    P1 t;
    P2 q;
    if (i != 63) {
      p3_to_p2(q, acc);
      p2_dbl(t, q);
      p1_to_p2(q, t);
      p2_dbl(t, q);
      p1_to_p2(q, t);
      p2_dbl(t, q);
      p1_to_p2(q, t);
      p2_dbl(t, q);
      p1_to_p3(acc, t);
    }
    const int ek = sc_digit(rk[i >> 3], i & 7);
    const int es = sc_digit(rs[i >> 3], i & 7);
    Cached ca = tab[ek < 0 ? -ek : ek];
    cached_cneg(ca, ek < 0);
    p3_add(t, acc, ca);
    p1_to_p3(acc, t);
    Precomp pb;
    select_precomp(pb, table, 0, es);
    p3_madd(t, acc, pb);
    p1_to_p3(acc, t);
  }
  // [8](R - R') == identity
  Cached cr;
  p3_to_cached(cr, acc);
  cached_cneg(cr, true);
  P1 t;
  P2 q;
  p3_add(t, R, cr);
  p1_to_p2(q, t);
  for (int j = 0; j < 3; ++j) {
    p2_dbl(t, q);
    p1_to_p2(q, t);
  }
  Fe d;
  fe_sub(d, q.Y, q.Z);
  return fe_is_zero(q.X) && fe_is_zero(d);
}

// base table entries (j + 1) * 16^row * B, j = 0..7 (one row per call)
ED_INL void base_table_row(int row, int32_t* table) {
  P3 Q;
  Q.X = fe_from_words(kBx);
  Q.Y = fe_from_words(kBy);
  Q.Z = fe_one();
  fe_mul(Q.T, Q.X, Q.Y);
  for (int i = 0; i < 4 * row; ++i) p3_dbl(Q, Q);
  Cached cq;
  p3_to_cached(cq, Q);
  P3 acc = Q;
  for (int j = 0; j < 8; ++j) {
    if (j > 0) {
      P1 t;
      p3_add(t, acc, cq);
      p1_to_p3(acc, t);
    }
    Precomp c;
    p3_to_precomp(c, acc);
    int32_t* e = table + (static_cast<size_t>(row) * 8 + j) * 30;
    for (int i = 0; i < 10; ++i) {
      e[i] = c.ypx.v[i];
      e[10 + i] = c.ymx.v[i];
      e[20 + i] = c.xy2d.v[i];
    }
  }
}

#undef ED_INL

}  // namespace ed
}  // namespace ag
