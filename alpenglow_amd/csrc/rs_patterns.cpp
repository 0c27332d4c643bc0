// Host-only pattern bookkeeping of the decoders (rs_patterns.hpp).  Restates no reference
// code: the window masks follow the crate's decoder window and
// ReedSolomonCoder's any-k-survivors use of it (reed_solomon.rs:150-180); the syndrome and
// correction tables are this build's own decoders.
#include "rs_patterns.hpp"

#include <algorithm>

#include "gf16.hpp"

namespace ag {

bool build_syn_pattern(size_t k, size_t m, const uint8_t* opres, const uint8_t* rpres, const uint16_t* G,
                       SynPattern* sp) {
  const Gf16Tables& t = gf16_tables();
  std::memset(sp, 0, sizeof *sp);
  size_t e = 0, r = 0;
  for (size_t i = 0; i < k; ++i) {
    if (opres[i]) sp->dmask |= uint64_t{1} << i;
    else if (e < 4) sp->out[e++] = static_cast<uint8_t>(i);
    else return false;
  }
  for (size_t j = 0; j < m && r < e; ++j)
    if (rpres[j]) sp->rec[r++] = static_cast<uint8_t>(j);
  if (r < e) return false;
  sp->e = static_cast<uint32_t>(e);
  // A[b][a] = G[rec[b]][out[a]]; Gauss-Jordan inverse over GF(2^16)
  uint16_t A[4][8] = {};
  for (size_t b = 0; b < e; ++b) {
    for (size_t a = 0; a < e; ++a) A[b][a] = G[sp->rec[b] * k + sp->out[a]];
    A[b][e + b] = 1;
  }
  for (size_t col = 0; col < e; ++col) {
    size_t piv = col;
    while (piv < e && A[piv][col] == 0) ++piv;
    if (piv == e) return false;
    if (piv != col)
      for (size_t x = 0; x < 2 * e; ++x) std::swap(A[piv][x], A[col][x]);
    const uint16_t inv = gf_inv(t, A[col][col]);
    for (size_t x = 0; x < 2 * e; ++x) A[col][x] = gf_mul_elem(t, A[col][x], inv);
    for (size_t row = 0; row < e; ++row) {
      if (row == col || A[row][col] == 0) continue;
      const uint16_t f = A[row][col];
      for (size_t x = 0; x < 2 * e; ++x) A[row][x] ^= gf_mul_elem(t, f, A[col][x]);
    }
  }
  // Minv[a][b] = A[a][e + b]; bitsliced matrix rows[o] bit i = bit o of (Minv * 2^i)
  for (size_t a = 0; a < e; ++a)
    for (size_t b = 0; b < e; ++b)
      for (unsigned i = 0; i < 16; ++i) {
        const uint16_t prod = gf_mul_elem(t, A[a][e + b], static_cast<uint16_t>(1u << i));
        for (unsigned o = 0; o < 16; ++o) sp->rows[a][b][o] |= ((prod >> o) & 1u) << i;
      }
  return true;
}

bool gf_invert(size_t n, uint16_t* A) {
  const Gf16Tables& t = gf16_tables();
  std::vector<uint16_t> M(n * 2 * n, 0);
  for (size_t r = 0; r < n; ++r) {
    for (size_t c = 0; c < n; ++c) M[r * 2 * n + c] = A[r * n + c];
    M[r * 2 * n + n + r] = 1;
  }
  for (size_t col = 0; col < n; ++col) {
    size_t piv = col;
    while (piv < n && M[piv * 2 * n + col] == 0) ++piv;
    if (piv == n) return false;
    if (piv != col)
      for (size_t x = 0; x < 2 * n; ++x) std::swap(M[piv * 2 * n + x], M[col * 2 * n + x]);
    const uint16_t inv = gf_inv(t, M[col * 2 * n + col]);
    for (size_t x = 0; x < 2 * n; ++x) M[col * 2 * n + x] = gf_mul_elem(t, M[col * 2 * n + x], inv);
    for (size_t row = 0; row < n; ++row) {
      const uint16_t f = M[row * 2 * n + col];
      if (row == col || f == 0) continue;
      for (size_t x = 0; x < 2 * n; ++x) M[row * 2 * n + x] ^= gf_mul_elem(t, f, M[col * 2 * n + x]);
    }
  }
  for (size_t r = 0; r < n; ++r)
    for (size_t c = 0; c < n; ++c) A[r * n + c] = M[r * 2 * n + n + c];
  return true;
}

// X = the 32-point full-recovery transform as a matrix (d_i = XOR_j X[i][j] * r_j): the
// inverse of the 32:32 HighRate encoder.  A k < 32 code is the 32:32 code with originals
// k..31 zero, so the same X serves every k <= 32 with m = 32.
const uint16_t* full_window_x32() {
  static const std::vector<uint16_t> X = [] {
    std::vector<uint16_t> G(32 * 32);
    hr_generator(32, 32, G.data());
    if (!gf_invert(32, G.data())) G.clear();  // cannot happen: the encoder is invertible
    return G;
  }();
  return X.empty() ? nullptr : X.data();
}

// Correction-decoder pattern (decode_c_kernel): HighRate k <= 32, m = 32, lost recovery
// shards L (1 <= |L| <= kCorrMaxSyn).  Syndrome points: virtual zeros k..31 first (no
// load), then present originals in index order.  False if the pattern does not fit (the
// caller takes another decoder).
// decode_c's balanced correction (rs_decode_c.hip), decided per pattern: layout H0 gives wave
// w the positions 2w, 16 + 2w, 2w + 1, 17 + 2w (slots 0..3).  Every wave keeps at most
// quota = ceil(|E| / 8) of its own restored originals (lowest slots first); the surplus, in
// ascending position order, is dealt to the waves below quota (ascending wave order), which
// accumulate it in their free slots (ascending slot order) and return the sums through LDS
// slot = the output's donation rank.
void corr_assign(CorrPattern* cp) {
  auto pos = [](uint32_t w, uint32_t t) { return (t & 1 ? 16u : 0u) + 2 * w + (t >> 1); };
  const uint64_t em = cp->emask;
  const uint32_t ne = static_cast<uint32_t>(__builtin_popcountll(em & 0xFFFFFFFFull));
  const uint32_t quota = (ne + 7) >> 3;
  auto rank = [&](uint64_t m, uint32_t a) {
    return static_cast<uint32_t>(__builtin_popcountll(m & ((uint64_t{1} << a) - 1)));
  };
  uint32_t own[8], donated[8], cap[8];
  uint64_t dmask = 0;
  for (uint32_t w = 0; w < 8; ++w) {
    own[w] = 0;
    for (uint32_t t = 0; t < 4; ++t)
      if ((em >> pos(w, t)) & 1) own[w] |= 1u << t;
    uint32_t m = own[w];
    for (uint32_t q = 0; q < quota && m; ++q) m &= m - 1;
    donated[w] = m;
    for (uint32_t t = 0; t < 4; ++t)
      if ((m >> t) & 1) dmask |= uint64_t{1} << pos(w, t);
    const uint32_t c = static_cast<uint32_t>(__builtin_popcount(own[w]));
    cap[w] = c < quota ? quota - c : 0;
  }
  const uint32_t nd = static_cast<uint32_t>(__builtin_popcountll(dmask));
  uint64_t rem = dmask;
  uint32_t d = 0;
  for (uint32_t w = 0; w < 8; ++w) {
    uint32_t act = 0, foreign = 0;
    for (uint32_t t = 0; t < 4; ++t) {
      uint32_t a = 64, lds = 0;
      if (((own[w] & ~donated[w]) >> t) & 1) {
        a = pos(w, t);
      } else if ((donated[w] >> t) & 1) {
        lds = rank(dmask, pos(w, t));
      } else if (!((own[w] >> t) & 1) && cap[w] && d < nd) {
        a = static_cast<uint32_t>(__builtin_ctzll(rem));
        rem &= rem - 1;
        lds = d++;
        --cap[w];
        foreign |= 1u << t;
      }
      uint32_t kofs = 0;
      if (a < 64) {
        act |= 1u << t;
        kofs = kCorrPairWords * rank(em, a) * cp->ns;
      }
      cp->wslot[w][t] = kofs | (lds << 20);
    }
    cp->wsum[w] = act | (own[w] << 4) | (donated[w] << 8) | (foreign << 12) | ((nd ? 1u : 0u) << 16);
  }
}

bool build_corr_pattern(size_t k, const uint8_t* opres, const uint8_t* rpres, CorrPattern* cp,
                        std::vector<uint32_t>& pool) {
  const uint16_t* X = full_window_x32();
  if (!X || k > 32) return false;
  const Gf16Tables& t = gf16_tables();
  std::memset(cp, 0, sizeof *cp);
  uint8_t E[32], L[32], D[32];
  size_t ne = 0, nl = 0, nd = 0;
  for (size_t j = 0; j < 32; ++j) {
    if (rpres[j]) cp->rmask |= uint64_t{1} << j;
    else L[nl++] = static_cast<uint8_t>(j);
  }
  for (size_t i = 0; i < k; ++i)
    if (!opres[i]) {
      cp->emask |= uint64_t{1} << i;
      E[ne++] = static_cast<uint8_t>(i);
    }
  if (nl == 0 || nl > static_cast<size_t>(kCorrMaxSyn) || ne == 0 || ne * nl > kCorrMaxPairs) return false;
  for (size_t i = k; i < 32 && nd < nl; ++i) D[nd++] = static_cast<uint8_t>(i);
  for (size_t i = 0; i < k && nd < nl; ++i)
    if (opres[i]) D[nd++] = static_cast<uint8_t>(i);
  if (nd < nl) return false;  // fewer than k survivors
  for (size_t b = 0; b < nd; ++b) cp->smask |= uint64_t{1} << D[b];
  // the syndrome rank b of point D[b] must follow position order (the kernel ranks by popcount)
  std::sort(D, D + nd);
  cp->ne = static_cast<uint32_t>(ne);
  cp->ns = static_cast<uint32_t>(nl);
  corr_assign(cp);
  // N = X[D, L], K = X[E, L] N^-1
  std::vector<uint16_t> N(nl * nl), K(ne * nl, 0);
  for (size_t b = 0; b < nl; ++b)
    for (size_t c = 0; c < nl; ++c) N[b * nl + c] = X[D[b] * 32 + L[c]];
  if (!gf_invert(nl, N.data())) return false;
  for (size_t a = 0; a < ne; ++a)
    for (size_t b = 0; b < nl; ++b) {
      uint16_t acc = 0;
      for (size_t c = 0; c < nl; ++c) acc ^= gf_mul_elem(t, X[E[a] * 32 + L[c]], N[c * nl + b]);
      K[a * nl + b] = acc;
    }
  // table picks: per pair, group pair gp and output plane o, the two nibbles of row o
  // (input planes 8gp..8gp+3, 8gp+4..8gp+7); row o bit i = bit o of K * 2^i
  cp->kofs = pool.size();
  pool.resize(pool.size() + ne * nl * kCorrPairWords);
  uint32_t* dst = pool.data() + cp->kofs;
  for (size_t a = 0; a < ne; ++a)
    for (size_t b = 0; b < nl; ++b, dst += kCorrPairWords) {
      uint32_t rows[16] = {};
      const uint16_t v = K[a * nl + b];
      for (unsigned i = 0; i < 16; ++i) {
        const uint16_t prod = gf_mul_elem(t, v, static_cast<uint16_t>(1u << i));
        for (unsigned o = 0; o < 16; ++o) rows[o] |= ((prod >> o) & 1u) << i;
      }
      for (unsigned gp = 0; gp < 2; ++gp)
        for (unsigned o = 0; o < 16; ++o) {
          dst[32 * gp + 2 * o] = (rows[o] >> (8 * gp)) & 15u;
          dst[32 * gp + 2 * o + 1] = (rows[o] >> (8 * gp + 4)) & 15u;
        }
    }
  return true;
}

// The correction decoder takes a 32:m=32 pattern when 1 <= |L| <= kCorrMaxSyn recovery
// shards are lost and some original is erased (no = present originals, nr = present
// recovery shards; no + nr >= k is checked first).
bool corr_fits(size_t k, size_t no, size_t nr) {
  const size_t nl = 32 - nr, ne = k - no;
  return nl >= 1 && nl <= static_cast<size_t>(kCorrMaxSyn) && ne >= 1 && ne * nl <= kCorrMaxPairs;
}

void window64_masks(bool hr, size_t k, size_t m, size_t xchunk, size_t xm_rec, const uint8_t* opres,
                    const uint8_t* rpres, bool any_k, uint64_t* e, uint64_t* in, uint64_t* out) {
  (void)m;
  const uint64_t ob = pack_flags(opres, k), kmask = k >= 64 ? ~uint64_t{0} : (uint64_t{1} << k) - 1;
  uint64_t rb = pack_flags(rpres, xm_rec);
  // ANY_K: exactly k survivors -- the present originals, then recovery shards in index
  // order; surplus recovery shards count as erased (MDS: any k survivors determine the
  // originals), so only k input multiplies remain.  EXACT: every present shard, as the
  // crate's decoder
  if (any_k) {
    const size_t po = static_cast<size_t>(__builtin_popcountll(ob));
    const size_t budget = k > po ? k - po : 0;
    // keep the lowest `budget` set bits (one pass over the kept bits: a popcount per
    // dropped bit cost ~40 ns per pattern, 5 ms per 131 072-pattern call)
    uint64_t keep = 0;
    for (size_t i = 0; i < budget && rb; ++i, rb &= rb - 1) keep |= rb & (~rb + 1);
    rb = keep;
  }
  const uint64_t cmask = xchunk >= 64 ? ~uint64_t{0} : (uint64_t{1} << xchunk) - 1;  // xchunk <= 32
  if (hr) {
    *in = rb | (ob << xchunk);
    *out = (~ob & kmask) << xchunk;
    *e = (~rb & cmask) | *out;  // lost / surplus recovery, virtual points m..chunk-1
  } else {
    *in = ob | (rb << xchunk);
    *out = ~ob & kmask;                       // the zero padding k..31 is neither loaded nor erased
    *e = *out | ((~rb & cmask) << xchunk);  // lost / surplus recovery, positions past m
  }
}

void window128_masks(bool hr, size_t k, size_t m, size_t c128, const uint8_t* opres, const uint8_t* rpres,
                     uint64_t q[10]) {
  const size_t oh = hr ? 1 : 0;  // the output (originals') window half
  const uint64_t ob = pack_flags(opres, k), kmask = k >= 64 ? ~uint64_t{0} : (uint64_t{1} << k) - 1;
  uint64_t rb[2] = {pack_flags(rpres, std::min<size_t>(m, 64)), m > 64 ? pack_flags(rpres + 64, m - 64) : 0};
  // exactly k survivors: the present originals, then recovery shards in index order
  const size_t po = static_cast<size_t>(__builtin_popcountll(ob));
  size_t budget = k > po ? k - po : 0;
  for (int w = 0; w < 2; ++w) {
    uint64_t keep = 0;
    for (uint64_t b = rb[w]; b && budget; b &= b - 1, --budget) keep |= b & (~b + 1);
    rb[w] = keep;
  }
  uint64_t in[2], out[2], e[2];
  if (hr) {  // recovery j at j (j < m <= 64), original i at 64 + i
    in[0] = rb[0];
    in[1] = ob;
    out[0] = 0;
    out[1] = ~ob & kmask;
    e[0] = ~rb[0];  // lost / surplus recovery and the virtual points m..63
    e[1] = out[1];  // positions 64 + k.. are the encoder's zeros, not erasures
  } else {  // original i at i, zero padding k..c-1, recovery j at c + j, erasures from c + m
    uint64_t rw[2] = {0, 0};  // recovery positions in the window
    for (size_t j = 0; j < m && c128 + j < 128; ++j) {
      const size_t g = c128 + j;
      if ((rb[j >> 6] >> (j & 63)) & 1) rw[g >> 6] |= uint64_t{1} << (g & 63);
    }
    const uint64_t cm = c128 >= 64 ? ~uint64_t{0} : (uint64_t{1} << c128) - 1;  // originals + padding
    in[0] = ob | rw[0];
    in[1] = rw[1];
    out[0] = ~ob & kmask;
    out[1] = 0;
    e[0] = out[0] | (~rw[0] & ~cm);  // lost / surplus recovery, positions past c + m
    e[1] = ~rw[1];
  }
  q[0] = e[0];
  q[1] = e[1];
  q[2] = in[0];
  q[3] = in[1];
  q[4] = out[0];
  q[5] = out[1];
  q[6] = in[1 - oh];  // pass 1: the other half's inputs
  q[7] = out[oh];
  q[8] = in[oh];      // pass 2: the output half's inputs
  q[9] = out[oh];
}

}  // namespace ag
