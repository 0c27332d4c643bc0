// Test infrastructure: runs the kernels' Ed25519 code (ed25519_core.hpp) on the host so
// tests/test_ed25519.py can check the arithmetic against the oracle without a GPU.  Not
// part of the library.  stdin lines: "pk SEED" | "sign SEED MSG" | "verify PK MSG SIG"
// (hex, MSG may be "-" for empty); stdout: one hex / 0 / 1 line each.  "bench_verify PK MSG
// SIG N" times N verifications on one host thread (bench_sig.py's native CPU baseline leg)
// and prints verifications per second.
#include <chrono>
#include <cstdio>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "ed25519_core.hpp"

using namespace ag::ed;

static std::vector<uint8_t> unhex(const std::string& s) {
  std::vector<uint8_t> v;
  if (s == "-") return v;
  for (size_t i = 0; i + 1 < s.size(); i += 2) v.push_back(static_cast<uint8_t>(std::stoi(s.substr(i, 2), nullptr, 16)));
  return v;
}
static std::string hex(const uint8_t* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s;
  for (size_t i = 0; i < n; ++i) {
    s += d[p[i] >> 4];
    s += d[p[i] & 15];
  }
  return s;
}

int main() {
  std::vector<int32_t> table(64 * 8 * 30);
  for (int r = 0; r < 64; ++r) base_table_row(r, table.data());
  std::string line;
  while (std::getline(std::cin, line)) {
    std::istringstream is(line);
    std::string op, a, b, c;
    is >> op >> a >> b >> c;
    if (op == "pk") {
      auto seed = unhex(a);
      uint8_t pk[32];
      public_key(seed.data(), pk, table.data());
      std::cout << hex(pk, 32) << "\n";
    } else if (op == "sign") {
      auto seed = unhex(a), msg = unhex(b);
      uint8_t pk[32], sig[64];
      public_key(seed.data(), pk, table.data());
      sign(seed.data(), pk, static_cast<uint32_t>(msg.size()), [&](uint32_t i) -> uint32_t { return msg[i]; }, sig,
           table.data());
      std::cout << hex(sig, 64) << "\n";
    } else if (op == "bench_verify") {
      auto pk = unhex(a), msg = unhex(b), sig = unhex(c);
      long n = 0;
      is >> n;
      Cached tab[9];
      int good = 0;
      const auto t0 = std::chrono::steady_clock::now();
      for (long r = 0; r < n; ++r)
        good += verify(pk.data(), sig.data(), static_cast<uint32_t>(msg.size()),
                       [&](uint32_t i) -> uint32_t { return msg[i]; }, table.data(), tab);
      const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      std::cout << (good == n ? n / dt : -1.0) << "\n";
    } else if (op == "verify") {
      auto pk = unhex(a), msg = unhex(b), sig = unhex(c);
      Cached tab[9];
      const bool ok = verify(pk.data(), sig.data(), static_cast<uint32_t>(msg.size()),
                             [&](uint32_t i) -> uint32_t { return msg[i]; }, table.data(), tab);
      std::cout << (ok ? 1 : 0) << "\n";
    }
  }
  return 0;
}
