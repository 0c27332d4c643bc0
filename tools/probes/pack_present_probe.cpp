// Host-side timing of the present-flag packing of ag_rs_coder_deshred_batch (AVX2 compares over
// 2 x 32 flag bytes per slice, 65 536 slices): is it on the coder deshred's critical path?
// g++ -O2 -o /tmp/pack_probe tools/probes/pack_present_probe.cpp && /tmp/pack_probe
#include <immintrin.h>
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>
__attribute__((target("avx2"))) static inline uint32_t nz(const uint8_t* f) {
  const __m256i x = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(f));
  return ~static_cast<uint32_t>(_mm256_movemask_epi8(_mm256_cmpeq_epi8(x, _mm256_setzero_si256())));
}
__attribute__((target("avx2"),noinline)) bool pack(const uint8_t* d, const uint8_t* c, size_t n, uint64_t* p) {
  bool s = false;
  for (size_t b = 0; b < n; ++b) { p[b] = uint64_t{nz(d + 32*b)} | (uint64_t{nz(c + 32*b)} << 32); s |= __builtin_popcountll(p[b]) > 32; }
  return s;
}
int main() {
  size_t n = 65536; std::vector<uint8_t> d(32*n), c(32*n); std::mt19937 r(1);
  for (auto& x : d) x = r() & 1; for (auto& x : c) x = r() & 1;
  std::vector<uint64_t> p(n);
  for (int it = 0; it < 5; ++it) {
    auto t0 = std::chrono::steady_clock::now(); bool s = pack(d.data(), c.data(), n, p.data());
    auto t1 = std::chrono::steady_clock::now();
    printf("%d %.1f us\n", s, std::chrono::duration<double, std::micro>(t1 - t0).count());
  }
}
