// Where a single-slice call's microseconds go (diagnostic; tools/latency/build.sh): one 32:32
// codeword of 1 KiB shreds encoded through the public C ABI in three ways, median of N calls:
//   device   ag_rs_encode_batch on device-resident buffers + stream sync (launch + kernel floor)
//   dma      pinned host -> hipMemcpyAsync H2D -> ag_rs_encode_batch -> D2H -> sync
//   zerocopy ag_rs_encode_batch(AG_RS_MEM_HOST)? no: ag_rs_coder_shred, the product per-call path
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "alpenglow_rs.h"

using clk = std::chrono::steady_clock;

template <typename F>
static double median_us(int n, F&& f) {
  for (int i = 0; i < 20; ++i) f();
  std::vector<double> t;
  for (int i = 0; i < n; ++i) {
    const auto a = clk::now();
    f();
    t.push_back(std::chrono::duration<double, std::micro>(clk::now() - a).count());
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 300;
  const size_t k = 32, m = 32, S = 1024, ob = k * S, rb = m * S;
  ag_rs_ctx* ctx = nullptr;
  if (ag_rs_ctx_create(0, &ctx)) return 1;
  hipStream_t st = static_cast<hipStream_t>(ag_rs_ctx_stream(ctx));
  uint8_t *d_o, *d_r, *h;
  if (hipMalloc(&d_o, ob) || hipMalloc(&d_r, rb) || hipHostMalloc(&h, ob + rb)) return 2;
  for (size_t i = 0; i < ob; ++i) h[i] = static_cast<uint8_t>(i * 131 + 7);
  (void)hipMemcpy(d_o, h, ob, hipMemcpyHostToDevice);
  auto enc = [&] { return ag_rs_encode_batch(ctx, k, m, S, 1, d_o, ob, d_r, rb, AG_RS_MEM_DEVICE); };
  const double t_dev = median_us(n, [&] {
    if (enc() || ag_rs_ctx_synchronize(ctx)) std::exit(3);
  });
  const double t_launch = median_us(n, [&] {
    if (enc()) std::exit(3);
  });
  (void)ag_rs_ctx_synchronize(ctx);
  const double t_dma = median_us(n, [&] {
    if (hipMemcpyAsync(d_o, h, ob, hipMemcpyHostToDevice, st) || enc() ||
        hipMemcpyAsync(h + ob, d_r, rb, hipMemcpyDeviceToHost, st) || hipStreamSynchronize(st))
      std::exit(4);
  });
  ag_rs_coder* coder = nullptr;
  if (ag_rs_coder_new(ctx, 32, &coder)) return 5;
  std::vector<uint8_t> data(ob), coding(rb);
  size_t sb = 0;
  const double t_zero = median_us(n, [&] {
    if (ag_rs_coder_shred(coder, h, 32767, data.data(), coding.data(), &sb)) std::exit(6);
  });
  std::printf("{\"unit\": \"us median\", \"device_encode_plus_sync\": %.2f, \"launch_only_async\": %.2f, "
              "\"dma_h2d_encode_d2h\": %.2f, \"coder_shred_zero_copy\": %.2f}\n", t_dev, t_launch, t_dma, t_zero);
  ag_rs_coder_free(coder);
  (void)hipFree(d_o);
  (void)hipFree(d_r);
  (void)hipHostFree(h);
  ag_rs_ctx_destroy(ctx);
  return 0;
}
