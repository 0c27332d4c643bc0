// Diagnostic: the 32:32 encode's memory skeleton at each block size (the 256 KiB
// dip).  A 512-thread workgroup per tile of 64 chunks copies its 32 input shard pieces (4 KiB
// each, stride S) to the same pieces of 32 output shards in a second buffer, with the
// transform kernels' lane-linear 16-byte nt accesses and XCD-contiguous tile order.  Usage: membench7 [GiB per side]
// Build: hipcc -O3 --offload-arch=gfx950 tools/membench/membench7.hip -o tools/latency/_build/membench7
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t g) {
  const uint32_t x = b & 7, q = g >> 3, r = g & 7;
  return x * q + (x < r ? x : r) + (b >> 3);
}

// NW waves of 64 lanes, 32 / NW shards per wave (NW = 4: xform<4>'s skeleton, NW = 8:
// xform8's); 64 KiB of dynamic LDS caps residency at two workgroups per CU like the kernels.
template <int NW>
__global__ __launch_bounds__(64 * NW) void tile_copy(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                     uint32_t S, uint32_t K) {
  extern __shared__ int pad[];
  constexpr int SH = 32 / NW;
  const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x);
  const uint32_t tps = S / 4096;  // tiles per shard
  const uint32_t blk = tile / tps, tt = tile % tps;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t bstride = static_cast<size_t>(K) * S;
  const uint8_t* src = in + blk * bstride + static_cast<size_t>(tt) * 4096 + lane * 16;
  uint8_t* dst = out + blk * bstride + static_cast<size_t>(tt) * 4096 + lane * 16;
  u32x4 v[SH][4];
#pragma unroll
  for (int s = 0; s < SH; ++s)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      v[s][q] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + static_cast<size_t>(wave * SH + s) * S + q * 1024));
  if (v[0][0].x == 0xdeadbeef && threadIdx.x == 1000) pad[0] = 1;
#pragma unroll
  for (int s = 0; s < SH; ++s)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_nontemporal_store(v[s][q], reinterpret_cast<u32x4*>(dst + static_cast<size_t>(wave * SH + s) * S + q * 1024));
}

int main(int argc, char** argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 4.0;
  const size_t bytes = static_cast<size_t>(gib * (1ull << 30));
  uint8_t *in, *out;
  if (hipMalloc(&in, bytes) != hipSuccess || hipMalloc(&out, bytes) != hipSuccess) return 1;
  (void)hipMemset(in, 1, bytes);
  (void)hipMemset(out, 0, bytes);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const uint32_t K = 32;
  for (uint32_t S : {4096u, 8192u, 16384u, 32768u, 131072u}) {
    for (int nw : {4, 8}) {
      const size_t nblk = bytes / (static_cast<size_t>(K) * S);
      const uint32_t tiles = static_cast<uint32_t>(nblk * (S / 4096));
      auto launch = [&] {
        if (nw == 4)
          hipLaunchKernelGGL(tile_copy<4>, dim3(tiles), dim3(256), 65536, 0, in, out, S, K);
        else
          hipLaunchKernelGGL(tile_copy<8>, dim3(tiles), dim3(512), 65536, 0, in, out, S, K);
      };
      for (int w = 0; w < 5; ++w) launch();
      (void)hipEventRecord(a);
      const int reps = 20;
      for (int r = 0; r < reps; ++r) launch();
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, a, b);
      const double tbs = 2.0 * static_cast<double>(tiles) * K * 4096 * reps / (ms * 1e-3) / 1e12;
      std::printf("{\"block_bytes\": %zu, \"shard_bytes\": %u, \"waves\": %d, \"copy_TBps\": %.3f}\n",
                  static_cast<size_t>(K) * S, S, nw, tbs);
    }
  }
  return 0;
}
