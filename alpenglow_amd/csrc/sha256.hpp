// SHA-256 (FIPS 180-4) shared by the host and the kernels: the hash the reference uses
// everywhere (crypto/hash.rs:64-79, the sha2 crate) -- Merkle trees (merkle.hip) and the
// all-or-nothing key masking (cipher.hip).  Header-only; the device compiles the 64 rounds
// fully unrolled (v_alignbit rotations, v_bitop3 XORs / ch / maj, v_add3).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace ag {
namespace sha {

constexpr uint32_t kK[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
constexpr uint32_t kIv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                                 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

// The 32-byte labels of merkle.rs:42-44 as big-endian message words.
struct Label {
  uint32_t w[8];
};
__host__ __device__ constexpr Label make_label(const char (&s)[33]) {
  Label l{};
  for (int i = 0; i < 8; ++i)
    l.w[i] = (uint32_t(uint8_t(s[4 * i])) << 24) | (uint32_t(uint8_t(s[4 * i + 1])) << 16) |
             (uint32_t(uint8_t(s[4 * i + 2])) << 8) | uint32_t(uint8_t(s[4 * i + 3]));
  return l;
}
constexpr Label kLeafLabel = make_label("ALPENGLOW-MERKLE-TREE  LEAF-NODE");
constexpr Label kLeftLabel = make_label("ALPENGLOW-MERKLE-TREE  LEFT-NODE");
constexpr Label kRightLabel = make_label("ALPENGLOW-MERKLE-TREE RIGHT-NODE");

__host__ __device__ inline __attribute__((always_inline)) uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
// 3-input XOR: one v_bitop3_b32 on the device (LLVM leaves the sigma XORs as two ops)
__host__ __device__ inline __attribute__((always_inline)) uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#ifdef __HIP_DEVICE_COMPILE__
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}
__host__ __device__ inline __attribute__((always_inline)) uint32_t bswap(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xFF00u) | ((x << 8) & 0xFF0000u) | (x << 24);
}

// One SHA-256 compression of the 16 big-endian words w (consumed as the schedule).
__host__ __device__ inline __attribute__((always_inline)) void compress(uint32_t st[8], uint32_t w[16]) {
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int r = 0; r < 64; ++r) {
    uint32_t wr;
    if (r < 16) {
      wr = w[r];
    } else {
      const uint32_t w15 = w[(r + 1) & 15], w2 = w[(r + 14) & 15];
      const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
      const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
      wr = w[r & 15] = w[r & 15] + s0 + w[(r + 9) & 15] + s1;
    }
    const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
    const uint32_t ch = (e & f) ^ (~e & g);
    const uint32_t t1 = h + S1 + ch + kK[r] + wr;
    const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
    const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    const uint32_t t2 = S0 + mj;
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
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

// hash_pair: SHA-256(LEFT_LABEL || l || RIGHT_LABEL || r), 128 bytes = 2 blocks + padding.
__host__ __device__ inline __attribute__((always_inline)) void hash_pair(const uint32_t l[8], const uint32_t r[8], uint32_t out[8]) {
  uint32_t st[8], w[16];
  for (int i = 0; i < 8; ++i) st[i] = kIv[i];
  for (int i = 0; i < 8; ++i) {
    w[i] = kLeftLabel.w[i];
    w[8 + i] = l[i];
  }
  compress(st, w);
  for (int i = 0; i < 8; ++i) {
    w[i] = kRightLabel.w[i];
    w[8 + i] = r[i];
  }
  compress(st, w);
  w[0] = 0x80000000u;
  for (int i = 1; i < 15; ++i) w[i] = 0;
  w[15] = 128 * 8;
  compress(st, w);
  for (int i = 0; i < 8; ++i) out[i] = st[i];
}

// Message word g (big-endian) of LEAF_LABEL || data[0..len) || SHA padding, total bytes
// T = 32 + len; `word(j)` returns data word j (bytes 4j..4j+3, little-endian load order).
template <typename DataWord, typename DataByte>
__host__ __device__ inline __attribute__((always_inline)) uint32_t leaf_msg_word(uint32_t g, uint32_t len, uint32_t nblk,
                                                           DataWord&& word, DataByte&& byte) {
  const uint32_t o = 4 * g, T = 32 + len;
  if (o < 32) return kLeafLabel.w[g];
  if (o + 4 <= T) return bswap(word((o - 32) >> 2));
  if (g == 16 * nblk - 1) return T * 8;  // bit length (T < 2^29): low word
  if (g == 16 * nblk - 2) return 0;      // bit length: high word
  uint32_t v = 0;
  for (uint32_t k = 0; k < 4; ++k) {
    const uint32_t ob = o + k;
    uint32_t bv = 0;
    if (ob < T) bv = byte(ob - 32);
    else if (ob == T) bv = 0x80;
    v |= bv << (24 - 8 * k);
  }
  return v;
}

}  // namespace sha

}  // namespace ag
