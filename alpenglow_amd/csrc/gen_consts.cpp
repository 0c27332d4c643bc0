// Build-time generator of the compile-time constants the bitsliced kernels use.
//
// For every FFT skew index s < kCount it emits
//   kSkewLog[s]     the skew factor's logarithm (65535 == "multiply by 0")
//   kMulRow[s][o]   16-bit mask: bit i set <=> output bit o of (x * skew[s]) depends on
//                   input bit i.  Multiplication by a constant is GF(2)-linear, so in the
//                   bitsliced layout it is a 16x16 XOR network over bit-planes.
//   kCse*[s]        the same network with shared sub-sums factored out: temps
//                   t_j = XOR of 2 or 3 earlier signals (one v_xor / v_bitop3 each), then
//                   output o = XOR of the signals in kCseRow[s][o] (signals 0..15 = input
//                   planes, 16+j = t_j).  Greedy on the exact VALU count with 3-input XORs
//                   (cost of a row with n terms plus the accumulator: ceil(n / 2)), with
//                   and without cancellation (cse(), bp_pass()).
//
// Usage: gen_consts <out.inc>
#include <algorithm>
#include <array>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <string>
#include <vector>

#include "gf16.hpp"

namespace {

constexpr int kMaxTemps = 40;

struct CseProgram {
  std::vector<std::array<int, 3>> temps;  // signal ids; [2] = -1 for a pair
  uint64_t rows[16];
};

int row_cost(int n) { return (n + 1) / 2; }

int program_cost(const CseProgram& p) {
  int c = static_cast<int>(p.temps.size());
  for (int o = 0; o < 16; ++o) c += row_cost(__builtin_popcountll(p.rows[o]));
  return c;
}

// One greedy pass: repeatedly factor out the 2- or 3-signal subset with the largest VALU
// gain.  rng == nullptr: the deterministic choice (largest gain, then the larger subset, then
// the first in mask order); otherwise a uniformly random pick among the candidates whose gain
// is within `slack` of the best (randomised restarts, cse() keeps the cheapest program).
CseProgram cse_pass(const uint16_t* mat, uint64_t* rng, int slack) {
  CseProgram prog;
  uint64_t rows[16];
  for (int o = 0; o < 16; ++o) rows[o] = mat[o];
  int nsig = 16;
  while (nsig < 16 + kMaxTemps) {
    std::map<uint64_t, int> uses;  // candidate subset mask -> rows containing it
    for (int o = 0; o < 16; ++o) {
      std::vector<int> ids;
      for (int b = 0; b < 64; ++b)
        if ((rows[o] >> b) & 1) ids.push_back(b);
      const int n = static_cast<int>(ids.size());
      for (int a = 0; a < n; ++a)
        for (int b = a + 1; b < n; ++b) {
          uses[(1ull << ids[a]) | (1ull << ids[b])]++;
          for (int c = b + 1; c < n; ++c) uses[(1ull << ids[a]) | (1ull << ids[b]) | (1ull << ids[c])]++;
        }
    }
    std::vector<std::pair<int, uint64_t>> cands;  // (gain, subset)
    uint64_t best = 0;
    int best_gain = 0;
    for (const auto& [m, cnt] : uses) {
      if (cnt < 2) continue;
      const int k = __builtin_popcountll(m);
      int gain = -1;
      for (int o = 0; o < 16; ++o)
        if ((rows[o] & m) == m) {
          const int n = __builtin_popcountll(rows[o]);
          gain += row_cost(n) - row_cost(n - k + 1);
        }
      if (gain <= 0) continue;
      cands.emplace_back(gain, m);
      if (gain > best_gain || (gain == best_gain && best && k > __builtin_popcountll(best))) {
        best = m;
        best_gain = gain;
      }
    }
    if (!best) break;
    if (rng) {
      std::vector<uint64_t> pool;
      for (const auto& [g, m] : cands)
        if (g >= best_gain - slack) pool.push_back(m);
      *rng = *rng * 6364136223846793005ull + 1442695040888963407ull;
      best = pool[(*rng >> 33) % pool.size()];
    }
    std::array<int, 3> t{-1, -1, -1};
    int j = 0;
    for (int b = 0; b < 64; ++b)
      if ((best >> b) & 1) t[j++] = b;
    prog.temps.push_back(t);
    for (int o = 0; o < 16; ++o)
      if ((rows[o] & best) == best) rows[o] = (rows[o] & ~best) | (1ull << nsig);
    ++nsig;
  }
  for (int o = 0; o < 16; ++o) prog.rows[o] = rows[o];
  return prog;
}

// Boyar-Peralta-style factoring with cancellation: a row may be the XOR of signals whose
// supports overlap.  dist[v] = the fewest signals XOR-ing to v, over all 2^16 vectors, so a
// candidate temp t (the XOR of 2 or 3 signals) is scored exactly: row o's distance becomes
// min(dist[T_o], 1 + dist[T_o ^ t]).  Greedy on the VALU cost (ceil(dist / 2) per row), then on
// the total distance; the cheapest prefix of the temp sequence is kept.  At most kBpMaxTemps
// temps (the subset greedy's peak: no more live VGPRs in the kernels).
constexpr int kBpMaxTemps = 13;
CseProgram bp_pass(const uint16_t* T, uint64_t* rng) {
  std::vector<uint16_t> base;
  for (int i = 0; i < 16; ++i) base.push_back(static_cast<uint16_t>(1u << i));
  std::vector<uint8_t> dist(65536, 255), par(65536, 255);
  // dist over the 16 input planes: popcount, the last step any set bit
  for (uint32_t v = 0; v < 65536; ++v) {
    dist[v] = static_cast<uint8_t>(__builtin_popcount(v));
    par[v] = v ? static_cast<uint8_t>(__builtin_ctz(v)) : 255;
  }
  auto cost_of = [&](size_t ntemps) {
    int c = static_cast<int>(ntemps);
    for (int o = 0; o < 16; ++o) c += row_cost(dist[T[o]]);
    return c;
  };
  std::vector<std::array<int, 3>> temps;
  std::vector<std::vector<uint8_t>> pars;  // par after each temp (the prefix rebuild)
  int best_cost = cost_of(0);
  size_t best_n = 0;
  std::vector<uint8_t> best_par = par;
  while (static_cast<int>(temps.size()) < kBpMaxTemps) {
    const int nb = static_cast<int>(base.size());
    long best_score = 0;
    std::vector<std::pair<long, std::array<int, 3>>> cands;
    for (int a = 0; a < nb; ++a)
      for (int b = a + 1; b < nb; ++b)
        for (int c = b + 1; c <= nb; ++c) {  // c == nb: the pair (a, b)
          const uint16_t t = static_cast<uint16_t>(base[a] ^ base[b] ^ (c < nb ? base[c] : 0));
          if (dist[t] <= 1) continue;
          long gc = 0, gd = 0;
          for (int o = 0; o < 16; ++o) {
            const int od = dist[T[o]];
            const int nd = std::min<int>(od, 1 + dist[T[o] ^ t]);
            gc += row_cost(od) - row_cost(nd);
            gd += od - nd;
          }
          const long score = gc * 64 + gd;
          if (score <= 0) continue;
          cands.push_back({score, {a, b, c < nb ? c : -1}});
          best_score = std::max(best_score, score);
        }
    if (best_score <= 0) break;
    std::vector<std::array<int, 3>> pool;
    const long slack = rng ? static_cast<long>((*rng >> 60) & 3) : 0;
    for (const auto& [sc, tt] : cands)
      if (sc >= best_score - slack) pool.push_back(tt);
    std::array<int, 3> tt = pool[0];
    if (rng) {
      *rng = *rng * 6364136223846793005ull + 1442695040888963407ull;
      tt = pool[(*rng >> 33) % pool.size()];
    }
    temps.push_back(tt);
    const uint16_t tv = static_cast<uint16_t>(base[tt[0]] ^ base[tt[1]] ^ (tt[2] >= 0 ? base[tt[2]] : 0));
    base.push_back(tv);
    // a shortest representation uses the new signal at most once
    const uint8_t ti = static_cast<uint8_t>(base.size() - 1);
    for (uint32_t v = 0; v < 65536; ++v) {
      const uint32_t w = v ^ tv;
      if (v < w) {
        const uint8_t dv = dist[v], dw = dist[w];
        if (dw + 1 < dv) {
          dist[v] = static_cast<uint8_t>(dw + 1);
          par[v] = ti;
        } else if (dv + 1 < dw) {
          dist[w] = static_cast<uint8_t>(dv + 1);
          par[w] = ti;
        }
      }
    }
    const int c = cost_of(temps.size());
    if (c < best_cost) {
      best_cost = c;
      best_n = temps.size();
      best_par = par;
    }
  }
  // the representations of the best prefix: follow the last-step pointers (a later pointer
  // may lead through a shorter path; a signal met twice cancels)
  CseProgram prog;
  prog.temps.assign(temps.begin(), temps.begin() + static_cast<long>(best_n));
  base.resize(16 + best_n);
  for (int o = 0; o < 16; ++o) {
    uint64_t r = 0;
    uint16_t v = T[o];
    for (int guard = 0; v && guard < 64; ++guard) {
      const int i = best_par[v];
      r ^= uint64_t{1} << i;
      v = static_cast<uint16_t>(v ^ base[i]);
    }
    prog.rows[o] = r;
  }
  return prog;
}

// The subset greedy (deterministic and randomised), the cancellation greedy (deterministic and
// randomised); fixed seeds per matrix, so the output is reproducible; the cheapest program
// wins (fewer temps on a tie).  Subset greedy alone: 36.2 VALU per multiply; with its 24
// restarts 35.3; with the cancellation greedy 32.9.
int g_restarts = 24;
CseProgram cse(const uint16_t* mat, bool subset_only = false) {
  CseProgram best = cse_pass(mat, nullptr, 0);
  auto take = [&](const CseProgram& p) {
    const int a = program_cost(p), b = program_cost(best);
    if (a < b || (a == b && p.temps.size() < best.temps.size())) best = p;
  };
  uint64_t rng = 0x9E3779B97F4A7C15ull;
  for (int o = 0; o < 16; ++o) rng = rng * 31 + mat[o];
  for (int r = 0; r < g_restarts; ++r) {
    CseProgram p = cse_pass(mat, &rng, r % 2);
    if (program_cost(p) < program_cost(best)) best = p;
  }
  if (!subset_only) {
    take(bp_pass(mat, nullptr));
    for (int r = 0; r < g_restarts; ++r) take(bp_pass(mat, &rng));
  }
  // self-check: the program computes exactly the matrix
  std::vector<uint16_t> sig(16);
  for (int i = 0; i < 16; ++i) sig[i] = static_cast<uint16_t>(1u << i);
  for (const auto& tt : best.temps)
    sig.push_back(static_cast<uint16_t>(sig[tt[0]] ^ sig[tt[1]] ^ (tt[2] >= 0 ? sig[tt[2]] : 0)));
  for (int o = 0; o < 16; ++o) {
    uint16_t m = 0;
    for (size_t b = 0; b < sig.size(); ++b)
      if ((best.rows[o] >> b) & 1) m ^= sig[b];
    if (m != mat[o]) {
      std::fprintf(stderr, "CSE program mismatch (row %d)\n", o);
      std::exit(1);
    }
  }
  return best;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc == 4 && std::string(argv[2]) == "--restarts") {
    g_restarts = std::atoi(argv[3]);  // diagnostics (the sanitizer build): fewer restarts
  } else if (argc != 2) {
    std::fprintf(stderr, "usage: %s out.inc [--restarts N]\n", argv[0]);
    return 2;
  }
  constexpr int kSkewCount = 256;
  const ag::Gf16Tables& t = ag::gf16_tables();
  const int kCount = kSkewCount;
  std::vector<uint16_t> clog(t.skew, t.skew + kCount);  // log of every constant (65535 = zero)
  FILE* f = std::fopen(argv[1], "w");
  if (!f) return 1;
  std::fprintf(f,
               "// GENERATED by gen_consts.cpp -- do not edit.\n"
               "// FFT skew logs and 16x16 GF(2) multiply matrices (row masks) for skew\n"
               "// indices 0..%d of the GF(2^16) Leopard FFT (poly 0x1002D, Cantor basis).\n"
               "#pragma once\n#include <cstdint>\n\n"
               "namespace ag {\n"
               "constexpr int kSkewConstCount = %d;\n",
               kCount - 1, kCount);
  std::fprintf(f, "constexpr uint16_t kSkewLog[kSkewConstCount] = {\n");
  for (int s = 0; s < kCount; ++s) std::fprintf(f, "%u,%s", clog[s], (s % 16 == 15) ? "\n" : " ");
  std::fprintf(f, "};\n\nconstexpr uint16_t kMulRow[kSkewConstCount][16] = {\n");
  std::vector<std::array<uint16_t, 16>> all(kCount);
  for (int s = 0; s < kCount; ++s) {
    uint16_t* rows = all[s].data();
    std::fill(rows, rows + 16, 0);
    if (clog[s] != ag::kGfModulus) {
      for (int i = 0; i < 16; ++i) {
        const uint16_t col = ag::gf_mul(t, static_cast<uint16_t>(1u << i), clog[s]);
        for (int o = 0; o < 16; ++o)
          if ((col >> o) & 1) rows[o] |= static_cast<uint16_t>(1u << i);
      }
    }
    std::fprintf(f, "{");
    for (int o = 0; o < 16; ++o) std::fprintf(f, "0x%04x%s", rows[o], o == 15 ? "" : ",");
    std::fprintf(f, "},\n");
  }
  std::fprintf(f, "};\n\n");
  // Two program sets: kCse* (the cheapest of both greedies) for every kernel, kCseSub* (the
  // subset greedy only) for decode_c and decode_pk, whose register allocations spill more with
  // the cancellation programs (decode_c 39 VGPRs against 9, decode_pk 14 against 0).  cse()
  // self-checks each.
  auto emit = [&](const char* pfx, bool subset_only) {
    std::vector<CseProgram> progs(kCount);
    size_t max_t = 0;
    for (int s = 0; s < kCount; ++s) {
      progs[s] = cse(all[s].data(), subset_only);
      max_t = std::max(max_t, progs[s].temps.size());
    }
    const size_t mt = max_t ? max_t : 1;
    std::fprintf(f, "constexpr int %sMaxTemps = %zu;\nconstexpr uint8_t %sNTemps[kSkewConstCount] = {\n", pfx, mt, pfx);
    for (int s = 0; s < kCount; ++s) std::fprintf(f, "%zu,%s", progs[s].temps.size(), (s % 16 == 15) ? "\n" : " ");
    std::fprintf(f, "};\n// temp j of skew s: signals a, b, c (c = 255: two-input XOR)\n"
                    "constexpr uint8_t %sTemp[kSkewConstCount][%sMaxTemps][3] = {\n", pfx, pfx);
    for (int s = 0; s < kCount; ++s) {
      std::fprintf(f, "{");
      for (size_t j = 0; j < mt; ++j) {
        std::array<int, 3> tt{255, 255, 255};
        if (j < progs[s].temps.size()) {
          tt = progs[s].temps[j];
          if (tt[2] < 0) tt[2] = 255;
        }
        std::fprintf(f, "{%d,%d,%d}%s", tt[0], tt[1], tt[2], j + 1 == mt ? "" : ",");
      }
      std::fprintf(f, "},\n");
    }
    std::fprintf(f, "};\nconstexpr uint64_t %sRow[kSkewConstCount][16] = {\n", pfx);
    for (int s = 0; s < kCount; ++s) {
      std::fprintf(f, "{");
      for (int o = 0; o < 16; ++o)
        std::fprintf(f, "0x%llxull%s", static_cast<unsigned long long>(progs[s].rows[o]), o == 15 ? "" : ",");
      std::fprintf(f, "},\n");
    }
    std::fprintf(f, "};\n");
  };
  emit("kCse", false);
  emit("kCseSub", true);
  // Basis change between the crate's Cantor-basis coordinates and the polynomial basis of
  // GF(2)[a] / 0x1002D: L(x) = a^log[x] (the LFSR state the crate's exp table inverts).
  // In the polynomial basis a multiply by `a` is a shift plus 3 XORs (a^16 = a^5 + a^3 + a^2 +
  // 1), so a runtime constant multiply is a 16-step Horner scheme (rs_kernels.hip mul_rt_poly).
  // Matrix 0 = L (Cantor -> poly), 1 = L^-1; emitted as CSE programs like the skew constants.
  {
    std::vector<uint16_t> st(ag::kGfModulus);
    uint32_t s = 1;
    for (uint32_t i = 0; i < ag::kGfModulus; ++i) {
      st[i] = static_cast<uint16_t>(s);
      s <<= 1;
      if (s >= ag::kGfOrder) s ^= ag::kGfPolynomial;
    }
    auto L = [&](uint16_t x) -> uint16_t { return x ? st[t.log[x]] : 0; };
    auto pmul = [](uint32_t a, uint32_t b) {
      uint32_t r = 0;
      for (int i = 0; i < 16; ++i)
        if ((b >> i) & 1) r ^= a << i;
      for (int i = 31; i >= 16; --i)
        if ((r >> i) & 1) r ^= ag::kGfPolynomial << (i - 16);
      return static_cast<uint16_t>(r);
    };
    // self-check: L is the field isomorphism (linear, multiplicative)
    uint32_t rnd = 12345;
    for (int n = 0; n < 4096; ++n) {
      rnd = rnd * 1103515245u + 12345u;
      const uint16_t x = static_cast<uint16_t>(rnd >> 8), y = static_cast<uint16_t>(rnd >> 15);
      if (L(x ^ y) != (L(x) ^ L(y)) || L(ag::gf_mul_elem(t, x, y)) != pmul(L(x), L(y))) {
        std::fprintf(stderr, "basis change self-check failed\n");
        return 1;
      }
    }
    uint16_t mat[2][16] = {};
    uint16_t cols[16];
    for (int i = 0; i < 16; ++i) cols[i] = L(static_cast<uint16_t>(1u << i));
    for (int o = 0; o < 16; ++o)
      for (int i = 0; i < 16; ++i) mat[0][o] |= static_cast<uint16_t>(((cols[i] >> o) & 1u) << i);
    // inverse: column i of L^-1 = the Cantor coordinates of a^i
    for (int i = 0; i < 16; ++i) {
      uint16_t x = 0;
      for (uint32_t v = 1; v < ag::kGfOrder; ++v)
        if (L(static_cast<uint16_t>(v)) == (1u << i)) {
          x = static_cast<uint16_t>(v);
          break;
        }
      for (int o = 0; o < 16; ++o) mat[1][o] |= static_cast<uint16_t>(((x >> o) & 1u) << i);
    }
    CseProgram bp[2] = {cse(mat[0]), cse(mat[1])};
    const size_t bmax = std::max(bp[0].temps.size(), bp[1].temps.size());
    std::fprintf(f, "\n// Cantor <-> polynomial basis (0: L, Cantor -> poly; 1: L^-1)\n"
                    "constexpr int kBasisMaxTemps = %zu;\nconstexpr uint8_t kBasisNTemps[2] = {%zu, %zu};\n"
                    "constexpr uint16_t kBasisMat[2][16] = {\n",
                 bmax, bp[0].temps.size(), bp[1].temps.size());
    for (int b = 0; b < 2; ++b) {
      std::fprintf(f, "{");
      for (int o = 0; o < 16; ++o) std::fprintf(f, "0x%04x%s", mat[b][o], o == 15 ? "" : ",");
      std::fprintf(f, "},\n");
    }
    std::fprintf(f, "};\nconstexpr uint8_t kBasisTemp[2][kBasisMaxTemps][3] = {\n");
    for (int b = 0; b < 2; ++b) {
      std::fprintf(f, "{");
      for (size_t j = 0; j < bmax; ++j) {
        std::array<int, 3> tt{255, 255, 255};
        if (j < bp[b].temps.size()) {
          tt = bp[b].temps[j];
          if (tt[2] < 0) tt[2] = 255;
        }
        std::fprintf(f, "{%d,%d,%d}%s", tt[0], tt[1], tt[2], j + 1 == bmax ? "" : ",");
      }
      std::fprintf(f, "},\n");
    }
    std::fprintf(f, "};\nconstexpr uint64_t kBasisRow[2][16] = {\n");
    for (int b = 0; b < 2; ++b) {
      std::fprintf(f, "{");
      for (int o = 0; o < 16; ++o)
        std::fprintf(f, "0x%llxull%s", static_cast<unsigned long long>(bp[b].rows[o]), o == 15 ? "" : ",");
      std::fprintf(f, "},\n");
    }
    std::fprintf(f, "};\n");
  }
  std::fprintf(f, "}  // namespace ag\n");
  std::fclose(f);
  return 0;
}
