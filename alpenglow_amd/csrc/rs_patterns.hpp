// Host-only pattern bookkeeping of the decoders (no HIP calls): presence flags -> masks, the
// per-pattern tables of the syndrome (decode_syn) and correction (decode_c) decoders, and the
// window masks of the locator decoders (decode_x / decode_h8 / decode_x16).  Split from
// rs_api.cpp so the CPU suite can run it under AddressSanitizer / UndefinedBehaviorSanitizer
// (tests/native/patterns_selfcheck.cpp, tests/test_sanitizers.py).
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <vector>

#include "rs_launch.hpp"

namespace ag {

// Host flag arrays (0 / nonzero bytes, one per shard) -> bit masks, 8 flags per step:
// the per-pattern bookkeeping of a 65 536-slice batch stays well under a millisecond.
inline uint64_t pack_flags(const uint8_t* f, size_t n) {  // n <= 64
  uint64_t bits = 0;
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t x;
    std::memcpy(&x, f + i, 8);
    // high bit of each byte <- byte != 0, then gather the 8 high bits (multiply trick)
    const uint64_t nz = ((((x & 0x7F7F7F7F7F7F7F7Full) + 0x7F7F7F7F7F7F7F7Full) | x) & 0x8080808080808080ull) >> 7;
    bits |= ((nz * 0x0102040810204080ull) >> 56) << i;
  }
  for (; i < n; ++i) bits |= uint64_t{f[i] != 0} << i;
  return bits;
}
inline size_t count_flags(const uint8_t* f, size_t n) {
  if (n <= 64) return static_cast<size_t>(__builtin_popcountll(pack_flags(f, n)));
  size_t c = 0;
  for (size_t i = 0; i < n; ++i) c += f[i] != 0;
  return c;
}

// Syndrome-decoder pattern (decode_syn_kernel): restore the erased originals from the
// first e present recovery shards; G = the k x m HighRate generator (hr_generator).  False
// if the pattern does not fit (more than 4 erased, too few recovery shards) or the e x e
// system is singular (cannot happen for an MDS code); the caller then takes another decoder.
bool build_syn_pattern(size_t k, size_t m, const uint8_t* opres, const uint8_t* rpres, const uint16_t* G,
                       SynPattern* sp);

// In-place Gauss-Jordan inverse of an n x n matrix over GF(2^16) (row-major, stride n).
// Returns false if singular.
bool gf_invert(size_t n, uint16_t* A);

// X = the 32-point full-recovery transform as a matrix (the inverse of the 32:32 encoder).
const uint16_t* full_window_x32();

// decode_c: whether a 32:m=32 pattern takes the correction decoder (no = present originals,
// nr = present recovery shards), and its pattern (K picks appended to `pool`).
bool corr_fits(size_t k, size_t no, size_t nr);
bool build_corr_pattern(size_t k, const uint8_t* opres, const uint8_t* rpres, CorrPattern* cp,
                        std::vector<uint32_t>& pool);

// The W <= 64 locator window of one pattern (decode_x / decode_h8 / decode_x16 PASS 0):
// erased (locator) / present (loaded) / restored position bits.  HighRate (hr): recovery j <
// xchunk at j, original i at xchunk + i; LowRate sub-window: original i at i, recovery j at
// xchunk + j (j < xm_rec).  any_k: exactly k survivors -- the present originals, then the
// recovery shards in index order (the surplus counts as erased).
void window64_masks(bool hr, size_t k, size_t m, size_t xchunk, size_t xm_rec, const uint8_t* opres,
                    const uint8_t* rpres, bool any_k, uint64_t* e, uint64_t* in, uint64_t* out);

// The W = 128 window of one pattern as two 64-point passes (exactly k survivors): q[0..5] =
// {erased, present, restored} as (positions 0..63, 64..127) pairs, q[6..7] = pass 1's (present
// in the loaded half, restored), q[8..9] = pass 2's.  c128 = next_pow2(m) (HighRate, 64) or
// next_pow2(k) (LowRate).
void window128_masks(bool hr, size_t k, size_t m, size_t c128, const uint8_t* opres, const uint8_t* rpres,
                     uint64_t q[10]);

}  // namespace ag
