// Test infrastructure (not part of the library): the host-only decoder bookkeeping of
// rs_patterns.cpp and the field code of gf16.cpp, built with AddressSanitizer and
// UndefinedBehaviorSanitizer by tests/test_sanitizers.py and checked against the field's own
// definitions -- no GPU, no HIP call.
//   * gf_invert: A * A^-1 = I for random invertible matrices (n = 1..32);
//   * full_window_x32: X * G = I for the 32:32 HighRate generator G;
//   * build_syn_pattern: Minv * (syndromes) restores the erased originals of 16:4 codewords;
//   * build_corr_pattern: (X r')_E + K s restores the erased originals of 32:32 codewords
//     with lost recovery shards (K read back from the kernel's table picks);
//   * window64_masks / window128_masks: exactly k survivors under ANY_K, no erased position
//     loaded, every restored position erased;
//   * pack_flags / count_flags against a byte loop.
// Prints "ok" and exits 0, or names the first failing check and exits 1.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "gf16.hpp"
#include "rs_patterns.hpp"

using namespace ag;

static int g_fail = 0;
#define CHECK(cond, ...)                         \
  do {                                           \
    if (!(cond)) {                               \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);         \
      std::fprintf(stderr, "\n");                \
      ++g_fail;                                  \
      return;                                    \
    }                                            \
  } while (0)

static uint16_t mulv(uint16_t a, uint16_t b) { return gf_mul_elem(gf16_tables(), a, b); }

// y = M x over GF(2^16), M n x n row-major
static void matvec(size_t n, const uint16_t* M, const uint16_t* x, uint16_t* y) {
  for (size_t r = 0; r < n; ++r) {
    uint16_t acc = 0;
    for (size_t c = 0; c < n; ++c) acc ^= mulv(M[r * n + c], x[c]);
    y[r] = acc;
  }
}

static void check_invert(std::mt19937_64& rng) {
  for (size_t n = 1; n <= 32; ++n) {
    std::vector<uint16_t> A(n * n), B;
    for (int attempt = 0;; ++attempt) {
      for (auto& v : A) v = static_cast<uint16_t>(rng());
      B = A;
      if (gf_invert(n, B.data())) break;
      CHECK(attempt < 8, "no invertible random %zux%zu matrix", n, n);
    }
    for (size_t r = 0; r < n; ++r)
      for (size_t c = 0; c < n; ++c) {
        uint16_t acc = 0;
        for (size_t i = 0; i < n; ++i) acc ^= mulv(A[r * n + i], B[i * n + c]);
        CHECK(acc == (r == c ? 1 : 0), "A * A^-1 != I (n=%zu)", n);
      }
  }
  std::vector<uint16_t> Z(9, 0);
  CHECK(!gf_invert(3, Z.data()), "singular matrix inverted");
}

static void check_x32() {
  const uint16_t* X = full_window_x32();
  CHECK(X != nullptr, "full_window_x32 failed");
  std::vector<uint16_t> G(32 * 32);
  hr_generator(32, 32, G.data());
  for (size_t r = 0; r < 32; ++r)
    for (size_t c = 0; c < 32; ++c) {
      uint16_t acc = 0;
      for (size_t i = 0; i < 32; ++i) acc ^= mulv(X[r * 32 + i], G[i * 32 + c]);
      CHECK(acc == (r == c ? 1 : 0), "X * G != I");
    }
}

// 16x16 GF(2) matrix (rows[o] bit i) applied to a field element
static uint16_t bitmat(const uint32_t* rows, uint16_t x) {
  uint16_t y = 0;
  for (unsigned o = 0; o < 16; ++o) y |= static_cast<uint16_t>((__builtin_popcount(rows[o] & x) & 1) << o);
  return y;
}

static void check_syn(std::mt19937_64& rng) {
  const size_t k = 16, m = 4;
  std::vector<uint16_t> G(m * k);
  hr_generator(k, m, G.data());
  for (int it = 0; it < 400; ++it) {
    uint16_t d[16], r[4];
    for (auto& v : d) v = static_cast<uint16_t>(rng());
    for (size_t j = 0; j < m; ++j) {
      r[j] = 0;
      for (size_t i = 0; i < k; ++i) r[j] ^= mulv(G[j * k + i], d[i]);
    }
    uint8_t op[16], rp[4];
    for (auto& v : op) v = 1;
    for (auto& v : rp) v = rng() & 1;
    const size_t e = rng() % 5;
    for (size_t i = 0; i < e; ++i) op[rng() % k] = 0;
    SynPattern sp;
    const size_t ne = k - count_flags(op, k), nr = count_flags(rp, m);
    const bool ok = build_syn_pattern(k, m, op, rp, G.data(), &sp);
    CHECK(ok == (ne <= nr), "build_syn_pattern admitted %d with ne=%zu nr=%zu", ok, ne, nr);
    if (!ok) continue;
    CHECK(sp.e == ne, "syn e");
    // syndromes: received recovery minus the re-encoded present originals at the used rows
    uint16_t S[4] = {};
    for (size_t b = 0; b < sp.e; ++b) {
      const size_t j = sp.rec[b];
      CHECK(rp[j], "syn uses an absent recovery shard");
      uint16_t acc = r[j];
      for (size_t i = 0; i < k; ++i)
        if (op[i]) acc ^= mulv(G[j * k + i], d[i]);
      S[b] = acc;
    }
    for (size_t a = 0; a < sp.e; ++a) {
      uint16_t got = 0;
      for (size_t b = 0; b < sp.e; ++b) got ^= bitmat(sp.rows[a][b], S[b]);
      CHECK(got == d[sp.out[a]], "syn restore mismatch");
    }
  }
}

static void check_corr(std::mt19937_64& rng) {
  const uint16_t* X = full_window_x32();
  std::vector<uint16_t> G(32 * 32);
  hr_generator(32, 32, G.data());
  for (int it = 0; it < 300; ++it) {
    const size_t k = 17 + rng() % 16;  // 17..32
    uint16_t d[32] = {}, r[32];
    for (size_t i = 0; i < k; ++i) d[i] = static_cast<uint16_t>(rng());
    matvec(32, G.data(), d, r);  // the k-code is the 32-code with originals k..31 zero
    uint8_t op[32], rp[32];
    for (size_t i = 0; i < k; ++i) op[i] = 1;
    for (auto& v : rp) v = 1;
    const size_t nl = 1 + rng() % 16;
    for (size_t i = 0; i < nl; ++i) rp[rng() % 32] = 0;
    const size_t ne = 1 + rng() % 16;
    for (size_t i = 0; i < ne; ++i) op[rng() % k] = 0;
    const size_t no = count_flags(op, k), nr = count_flags(rp, 32);
    if (no + nr < k) continue;
    CorrPattern cp;
    std::vector<uint32_t> pool;
    const bool fits = corr_fits(k, no, nr);
    const bool ok = build_corr_pattern(k, op, rp, &cp, pool);
    CHECK(ok == fits, "build_corr_pattern %d vs corr_fits %d", ok, fits);
    if (!ok) continue;
    uint16_t rz[32], xr[32];
    for (size_t j = 0; j < 32; ++j) rz[j] = rp[j] ? r[j] : 0;
    matvec(32, X, rz, xr);
    // syndromes at the points of smask in position order
    uint16_t s[32];
    size_t ns = 0;
    for (size_t i = 0; i < 32; ++i)
      if ((cp.smask >> i) & 1) s[ns++] = static_cast<uint16_t>(d[i] ^ xr[i]);
    CHECK(ns == cp.ns, "corr syndrome count");
    const uint32_t* K = pool.data() + cp.kofs;
    size_t a = 0;
    for (size_t i = 0; i < k; ++i) {
      if (!((cp.emask >> i) & 1)) continue;
      uint16_t got = xr[i];
      for (size_t b = 0; b < ns; ++b) {
        const uint32_t* pk = K + kCorrPairWords * (a * ns + b);
        uint32_t rows[16];
        for (unsigned o = 0; o < 16; ++o)
          rows[o] = pk[2 * o] | (pk[2 * o + 1] << 4) | (pk[32 + 2 * o] << 8) | (pk[32 + 2 * o + 1] << 12);
        got ^= bitmat(rows, s[b]);
      }
      CHECK(got == d[i], "corr restore mismatch (k=%zu |L|=%u |E|=%u)", k, cp.ns, cp.ne);
      ++a;
    }
  }
}

static void check_windows(std::mt19937_64& rng) {
  for (int it = 0; it < 2000; ++it) {
    // HighRate 32:32 (xchunk 32) and the LowRate sub-window of 32:64 (xchunk 32, xm_rec 32)
    const bool hr = it & 1;
    const size_t k = 32, m = hr ? 32 : 64, xchunk = 32, xm_rec = 32;
    uint8_t op[32], rp[64];
    for (auto& v : op) v = rng() & 1;
    for (auto& v : rp) v = (rng() % 3) != 0;
    const size_t no = count_flags(op, k), nr = count_flags(rp, xm_rec);
    if (no + nr < k) continue;
    uint64_t e, in, out;
    window64_masks(hr, k, m, xchunk, xm_rec, op, rp, true, &e, &in, &out);
    CHECK(static_cast<size_t>(__builtin_popcountll(in)) == k, "ANY_K window loads %d, not k", __builtin_popcountll(in));
    CHECK((in & e) == 0, "a loaded position is erased");
    CHECK((out & ~e) == 0, "a restored position is not erased");
    CHECK(static_cast<size_t>(__builtin_popcountll(out)) == k - no, "restored count");
    uint64_t e2, in2, out2;
    window64_masks(hr, k, m, xchunk, xm_rec, op, rp, false, &e2, &in2, &out2);
    CHECK(static_cast<size_t>(__builtin_popcountll(in2)) == no + nr, "EXACT window must load every present shard");
    // W = 128: HighRate 64:64, LowRate 32:64 over both recovery chunks
    const size_t k2 = hr ? 64 : 32, m2 = 64, c128 = 64 / (hr ? 1 : 2);
    uint8_t op2[64], rp2[64];
    for (size_t i = 0; i < k2; ++i) op2[i] = rng() & 1;
    for (auto& v : rp2) v = rng() & 1;
    if (count_flags(op2, k2) + count_flags(rp2, m2) < k2) continue;
    uint64_t q[10];
    window128_masks(hr, k2, m2, hr ? 64 : c128, op2, rp2, q);
    const int nin = __builtin_popcountll(q[2]) + __builtin_popcountll(q[3]);
    CHECK(static_cast<size_t>(nin) == k2, "W=128 loads %d, not k", nin);
    CHECK(((q[2] & q[0]) | (q[3] & q[1])) == 0, "W=128 loaded position erased");
    CHECK(((q[4] & ~q[0]) | (q[5] & ~q[1])) == 0, "W=128 restored position not erased");
  }
}

static void check_flags(std::mt19937_64& rng) {
  for (int it = 0; it < 5000; ++it) {
    const size_t n = rng() % 65;
    std::vector<uint8_t> f(n);
    uint64_t want = 0;
    for (size_t i = 0; i < n; ++i) {
      f[i] = (rng() & 3) ? static_cast<uint8_t>(rng()) : 0;
      if (f[i]) want |= uint64_t{1} << i;
    }
    CHECK(pack_flags(f.data(), n) == want, "pack_flags");
    CHECK(count_flags(f.data(), n) == static_cast<size_t>(__builtin_popcountll(want)), "count_flags");
  }
}

int main() {
  std::mt19937_64 rng(0xA19E);
  check_flags(rng);
  check_invert(rng);
  check_x32();
  check_syn(rng);
  check_corr(rng);
  check_windows(rng);
  if (g_fail) return 1;
  std::printf("ok\n");
  return 0;
}
