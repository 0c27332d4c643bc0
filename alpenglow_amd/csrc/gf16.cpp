// GF(2^16) tables (see gf16.hpp).  Table construction follows the crate's
// engine/tables.rs: LFSR log table, conversion to the Cantor basis, FFT skew factors.
#include "gf16.hpp"

#include <algorithm>
#include <memory>
#include <vector>

namespace ag {
namespace {

constexpr uint16_t kCantorBasis[kGfBits] = {
    0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
    0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E};

std::unique_ptr<Gf16Tables> build() {
  auto t = std::make_unique<Gf16Tables>();
  // LFSR: exp[] temporarily holds the polynomial-basis logarithm.
  uint32_t state = 1;
  for (uint32_t i = 0; i < kGfModulus; ++i) {
    t->exp[state] = static_cast<uint16_t>(i);
    state <<= 1;
    if (state >= kGfOrder) state ^= kGfPolynomial;
  }
  t->exp[0] = kGfModulus;
  // Cantor basis: log[x] = polynomial-basis log of the element whose Cantor
  // coordinates are x.
  t->log[0] = 0;
  for (unsigned i = 0; i < kGfBits; ++i) {
    const uint32_t w = 1u << i;
    for (uint32_t j = 0; j < w; ++j) t->log[j + w] = t->log[j] ^ kCantorBasis[i];
  }
  for (uint32_t i = 0; i < kGfOrder; ++i) t->log[i] = t->exp[t->log[i]];
  for (uint32_t i = 0; i < kGfOrder; ++i) t->exp[t->log[i]] = static_cast<uint16_t>(i);
  t->exp[kGfModulus] = t->exp[0];

  // Skew factors of the additive FFT (normalised subspace-polynomial values).
  uint16_t temp[kGfBits - 1];
  for (unsigned i = 1; i < kGfBits; ++i) temp[i - 1] = static_cast<uint16_t>(1u << i);
  for (unsigned m = 0; m < kGfBits - 1; ++m) {
    const size_t step = size_t{1} << (m + 1);
    t->skew[(size_t{1} << m) - 1] = 0;
    for (unsigned i = m; i < kGfBits - 1; ++i) {
      const size_t s = size_t{1} << (i + 1);
      for (size_t j = (size_t{1} << m) - 1; j < s; j += step) t->skew[j + s] = t->skew[j] ^ temp[i];
    }
    temp[m] = static_cast<uint16_t>(kGfModulus - t->log[gf_mul(*t, temp[m], t->log[temp[m] ^ 1])]);
    for (unsigned i = m + 1; i < kGfBits - 1; ++i)
      temp[i] = gf_mul(*t, temp[i], gf_add_mod(t->log[temp[i] ^ 1], temp[m]));
  }
  for (uint32_t i = 0; i < kGfModulus; ++i) t->skew[i] = t->log[t->skew[i]];
  return t;
}

}  // namespace

const Gf16Tables& gf16_tables() {
  static const std::unique_ptr<Gf16Tables> tables = build();
  return *tables;
}

namespace {

// The crate's additive FFT / IFFT over one symbol column (indices relative to pos, skew
// index r + dist + delta - 1).
void ifft_col(const Gf16Tables& t, uint16_t* w, size_t pos, size_t size, size_t trunc, size_t delta) {
  for (size_t dist = 1; dist < size; dist <<= 1)
    for (size_t r = 0; r < trunc; r += 2 * dist) {
      const uint16_t lm = t.skew[r + dist + delta - 1];
      for (size_t i = r; i < r + dist; ++i) {
        uint16_t &x = w[pos + i], &y = w[pos + i + dist];
        y ^= x;
        if (lm != kGfModulus) x ^= gf_mul(t, y, lm);
      }
    }
}
void fft_col(const Gf16Tables& t, uint16_t* w, size_t pos, size_t size, size_t trunc, size_t delta) {
  for (size_t dist = size >> 1; dist >= 1; dist >>= 1)
    for (size_t r = 0; r < trunc; r += 2 * dist) {
      const uint16_t lm = t.skew[r + dist + delta - 1];
      for (size_t i = r; i < r + dist; ++i) {
        uint16_t &x = w[pos + i], &y = w[pos + i + dist];
        if (lm != kGfModulus) x ^= gf_mul(t, y, lm);
        y ^= x;
      }
    }
}

}  // namespace

void hr_generator(size_t k, size_t m, uint16_t* G) {
  const Gf16Tables& t = gf16_tables();
  const size_t chunk = next_pow2(m);
  const size_t rows = std::max(chunk, (k + chunk - 1) / chunk * chunk);
  std::vector<uint16_t> w(rows);
  for (size_t i = 0; i < k; ++i) {
    std::fill(w.begin(), w.end(), uint16_t{0});
    w[i] = 1;
    ifft_col(t, w.data(), 0, chunk, std::min(k, chunk), chunk);
    for (size_t cs = chunk; cs < k; cs += chunk) {  // further (possibly partial) chunks
      ifft_col(t, w.data(), cs, chunk, std::min(chunk, k - cs), cs + chunk);
      for (size_t j = 0; j < chunk; ++j) w[j] ^= w[cs + j];
    }
    fft_col(t, w.data(), 0, chunk, m, 0);
    for (size_t j = 0; j < m; ++j) G[j * k + i] = w[j];
  }
}

int use_high_rate(size_t k, size_t m) {
  if (k > kGfOrder || m > kGfOrder) return -1;
  const size_t pk = next_pow2(k), pm = next_pow2(m);
  const size_t smaller = pk < pm ? pk : pm;
  const size_t larger = k > m ? k : m;
  if (k == 0 || m == 0 || smaller + larger > kGfOrder) return -1;
  if (pk < pm) return 0;
  if (pk > pm) return 1;
  // Equal powers of two: the crate picks HighRate when original_count <= recovery_count.
  return k <= m ? 1 : 0;
}

}  // namespace ag
