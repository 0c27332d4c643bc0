// Per-call latency of the crate-API route (INTEGRATION.md Route A) without an interpreter in
// the way: a C++ caller of the C ABI, as the Rust facade would be.  One ReedSolomonCoder with
// a private context, one 32 767-byte slice per call (the reference's shape: block_producer.rs
// :339-345 -> reed_solomon.rs:88-128 shred; slot_block_data.rs:353 -> :140-208 deshred).
// Prints one JSON line: median / p90 / min microseconds per call for
//   shred           payload -> 32 data + 32 coding shreds of 1 KiB
//   deshred_coding  from the 32 coding shreds only (benches/shredder.rs:49-53's shape)
//   deshred_random  from a random 32 of the 64 shreds (the follower's arrival)
//   route_a_*       ReedSolomonEncoder / ReedSolomonDecoder (the facade's entry points): reset,
//                   32 adds, encode / decode, 32 result reads copied out
// Usage: latency_probe [calls]   (built by tools/latency/build.sh against the in-tree library)
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "alpenglow_rs.h"

// diagnostic accessor of the library (not in the header): the last server job's in-kernel ns
extern "C" int ag_rs_internal_coder_last_job_ns(ag_rs_coder* coder, uint64_t* ns);

using clk = std::chrono::steady_clock;

struct Stat {
  double med, p90, min;
};
static Stat stat(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return {v[v.size() / 2], v[v.size() * 9 / 10], v[0]};
}

int main(int argc, char** argv) {
  const int calls = argc > 1 ? std::atoi(argv[1]) : 400;
  ag_rs_coder* coder = nullptr;
  if (ag_rs_coder_new_on_device(0, 32, &coder)) {
    std::fprintf(stderr, "no coder (no device?)\n");
    return 1;
  }
  std::mt19937_64 rng(7);
  std::vector<uint8_t> payload(AG_RS_MAX_DATA_PER_SLICE);
  for (auto& b : payload) b = static_cast<uint8_t>(rng());
  std::vector<uint8_t> data(32 * 1024), coding(32 * 1024), pout(32 * 1024), dout(32 * 1024), cout(32 * 1024);
  size_t S = 0, plen = 0;
  auto shred = [&] { return ag_rs_coder_shred(coder, payload.data(), payload.size(), data.data(), coding.data(), &S); };
  if (shred() || S != 1024) return 1;
  std::vector<const uint8_t*> ptr(64);
  std::vector<size_t> lens(64, S);
  std::vector<uint8_t> is_data(64);
  for (int i = 0; i < 64; ++i) is_data[i] = i < 32;
  auto set_present = [&](const std::vector<int>& keep) {
    std::fill(ptr.begin(), ptr.end(), nullptr);
    for (int i : keep) ptr[i] = i < 32 ? data.data() + i * S : coding.data() + (i - 32) * S;
  };
  auto deshred = [&] {
    return ag_rs_coder_deshred(coder, 32, ptr.data(), lens.data(), is_data.data(), pout.data(), &plen, dout.data(),
                               cout.data(), &S);
  };
  std::vector<double> job;  // the last timed series' server-job microseconds (in-kernel)
  std::vector<double> ph[4];  // and its phases
  auto time = [&](auto&& f) {
    for (int i = 0; i < 20; ++i) f();
    std::vector<double> t;
    job.clear();
    for (auto& v : ph) v.clear();
    for (int i = 0; i < calls; ++i) {
      const auto a = clk::now();
      if (f()) std::exit(2);
      t.push_back(std::chrono::duration<double, std::micro>(clk::now() - a).count());
      uint64_t ns[5] = {};
      if (ag_rs_internal_coder_last_job_ns(coder, ns) == 0) {
        job.push_back(ns[0] * 1e-3);
        for (int k = 0; k < 4; ++k) ph[k].push_back(ns[1 + k] * 1e-3);
      }
    }
    return stat(t);
  };
  const Stat s_shred = time(shred);
  std::vector<int> coding_only;
  for (int i = 32; i < 64; ++i) coding_only.push_back(i);
  set_present(coding_only);
  const Stat s_dc = time(deshred);
  const Stat j_dc = stat(job);
  double p_dc[4];
  for (int k = 0; k < 4; ++k) p_dc[k] = stat(ph[k]).med;
  if (plen != payload.size() || std::memcmp(pout.data(), payload.data(), plen)) return 3;
  std::vector<int> all(64);
  for (int i = 0; i < 64; ++i) all[i] = i;
  std::shuffle(all.begin(), all.end(), rng);
  all.resize(32);
  set_present(all);
  const Stat s_dr = time(deshred);
  const Stat j_dr = stat(job);
  double p_dr[4];
  for (int k = 0; k < 4; ++k) p_dr[k] = stat(ph[k]).med;
  if (plen != payload.size() || std::memcmp(pout.data(), payload.data(), plen) ||
      std::memcmp(cout.data(), coding.data(), 32 * S))
    return 4;
  // Route A's own entry points in the Rust facade's call pattern: the crate's
  // ReedSolomonEncoder / ReedSolomonDecoder as reed_solomon.rs drives them per slice --
  // reset, 32 add_*_shard, encode / decode, 32 result reads (recovery_iter / restored_original)
  ag_rs_encoder* enc = nullptr;
  ag_rs_decoder* dec = nullptr;
  if (ag_rs_encoder_new_on_device(0, 32, 32, S, &enc) || ag_rs_decoder_new_on_device(0, 32, 32, S, &dec)) return 5;
  std::vector<uint8_t> sink(32 * S);
  auto encoder = [&] {
    int st = ag_rs_encoder_reset(enc, 32, 32, S);
    for (int i = 0; i < 32 && !st; ++i) st = ag_rs_encoder_add_original_shard(enc, data.data() + i * S, S);
    if (!st) st = ag_rs_encoder_encode(enc);
    for (int j = 0; j < 32 && !st; ++j) {
      const uint8_t* r = nullptr;
      size_t len = 0;
      st = ag_rs_encoder_recovery(enc, j, &r, &len);
      if (!st) std::memcpy(sink.data() + j * S, r, len);  // the facade's .to_vec()
    }
    return st;
  };
  std::vector<int> keep;  // decoder: the follower's random 32 of 64
  auto decoder = [&] {
    int st = ag_rs_decoder_reset(dec, 32, 32, S);
    for (int i : keep) {
      if (st) break;
      st = i < 32 ? ag_rs_decoder_add_original_shard(dec, i, data.data() + i * S, S)
                  : ag_rs_decoder_add_recovery_shard(dec, i - 32, coding.data() + (i - 32) * S, S);
    }
    if (!st) st = ag_rs_decoder_decode(dec);
    for (int i = 0; i < 32 && !st; ++i) {
      const uint8_t* r = nullptr;
      size_t len = 0;
      if (ag_rs_decoder_restored_original(dec, i, &r, &len) == 0) std::memcpy(sink.data() + i * S, r, len);
    }
    return st;
  };
  const Stat s_enc = time(encoder);
  if (std::memcmp(sink.data(), coding.data(), 32 * S)) return 6;
  keep.assign(coding_only.begin(), coding_only.end());
  const Stat s_dec_c = time(decoder);
  if (std::memcmp(sink.data(), data.data(), 32 * S)) return 7;
  keep.assign(all.begin(), all.end());
  const Stat s_dec_r = time(decoder);
  for (int i = 0; i < 32; ++i)
    if (std::find(keep.begin(), keep.end(), i) == keep.end() && std::memcmp(sink.data() + i * S, data.data() + i * S, S))
      return 8;
  std::printf("{\"unit\": \"us per call\", \"caller\": \"C++ through the C ABI\", \"calls\": %d, "
              "\"shred\": {\"median\": %.2f, \"p90\": %.2f, \"min\": %.2f}, "
              "\"deshred_coding_only\": {\"median\": %.2f, \"p90\": %.2f, \"min\": %.2f}, "
              "\"deshred_random_32_of_64\": {\"median\": %.2f, \"p90\": %.2f, \"min\": %.2f}, "
              "\"route_a_encoder\": {\"median\": %.2f, \"p90\": %.2f, \"min\": %.2f}, "
              "\"route_a_decoder_coding_only\": {\"median\": %.2f, \"p90\": %.2f, \"min\": %.2f}, "
              "\"route_a_decoder_random_32_of_64\": {\"median\": %.2f, \"p90\": %.2f, \"min\": %.2f}, "
              "\"server_job_in_kernel\": {\"phases\": [\"kind read\", \"parameters + invalidate\", \"tile\", \"release\"], "
              "\"deshred_coding_only\": {\"median\": %.2f, \"min\": %.2f, \"phase_medians\": [%.2f, %.2f, %.2f, %.2f]}, "
              "\"deshred_random_32_of_64\": {\"median\": %.2f, \"min\": %.2f, \"phase_medians\": [%.2f, %.2f, %.2f, %.2f]}}}\n",
              calls, s_shred.med, s_shred.p90, s_shred.min, s_dc.med, s_dc.p90, s_dc.min, s_dr.med, s_dr.p90, s_dr.min,
              s_enc.med, s_enc.p90, s_enc.min, s_dec_c.med, s_dec_c.p90, s_dec_c.min, s_dec_r.med, s_dec_r.p90,
              s_dec_r.min, j_dc.med, j_dc.min, p_dc[0], p_dc[1], p_dc[2], p_dc[3], j_dr.med, j_dr.min, p_dr[0], p_dr[1],
              p_dr[2], p_dr[3]);
  ag_rs_encoder_free(enc);
  ag_rs_decoder_free(dec);
  ag_rs_coder_free(coder);
  return 0;
}
