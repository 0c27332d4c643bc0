// Streaming ceiling exploration (diagnostic): read-only, write-only, copy; per-thread
// depth, occupancy, non-temporal hints.  Usage: membench2 [GiB]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int DEPTH, int NT>
__global__ void rd(const u32x4* __restrict__ in, u32x4* __restrict__ sink, size_t n16) {
  size_t i = (size_t)blockIdx.x * blockDim.x * DEPTH + threadIdx.x;
  u32x4 acc = {0, 0, 0, 0};
  for (; i < n16; i += (size_t)gridDim.x * blockDim.x * DEPTH) {
#pragma unroll
    for (int k = 0; k < DEPTH; ++k) {
      size_t j = i + (size_t)k * blockDim.x;
      if (j < n16) acc ^= NT ? __builtin_nontemporal_load(in + j) : in[j];
    }
  }
  if (acc.x == 0x12345678 && acc.y == 0x9abcdef) sink[threadIdx.x] = acc;
}

template <int DEPTH, int NT>
__global__ void wr(u32x4* __restrict__ out, size_t n16) {
  size_t i = (size_t)blockIdx.x * blockDim.x * DEPTH + threadIdx.x;
  u32x4 v = {1u, 2u, 3u, (uint32_t)threadIdx.x};
  for (; i < n16; i += (size_t)gridDim.x * blockDim.x * DEPTH) {
#pragma unroll
    for (int k = 0; k < DEPTH; ++k) {
      size_t j = i + (size_t)k * blockDim.x;
      if (j < n16) {
        if (NT) __builtin_nontemporal_store(v, out + j); else out[j] = v;
      }
    }
  }
}

template <int DEPTH, int NTL, int NTS>
__global__ void cp(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t n16) {
  size_t i = (size_t)blockIdx.x * blockDim.x * DEPTH + threadIdx.x;
  for (; i < n16; i += (size_t)gridDim.x * blockDim.x * DEPTH) {
    u32x4 v[DEPTH];
#pragma unroll
    for (int k = 0; k < DEPTH; ++k) {
      size_t j = i + (size_t)k * blockDim.x;
      v[k] = j < n16 ? (NTL ? __builtin_nontemporal_load(in + j) : in[j]) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int k = 0; k < DEPTH; ++k) {
      size_t j = i + (size_t)k * blockDim.x;
      if (j < n16) {
        if (NTS) __builtin_nontemporal_store(v[k], out + j); else out[j] = v[k];
      }
    }
  }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

static hipEvent_t e0, e1;
template <typename F>
static void timeit(const char* name, double bytes_moved, F f) {
  f();
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipEventRecord(e0));
    f();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  printf("%-44s %8.3f ms  %6.0f GB/s\n", name, best, bytes_moved / (best * 1e-3) / 1e9);
}

int main(int argc, char** argv) {
  double gib = argc > 1 ? atof(argv[1]) : 4.0;
  size_t bytes = (size_t)(gib * (1ull << 30));
  size_t n16 = bytes / 16;
  u32x4 *a, *b, *sink;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&sink, 4096 * 16));
  CK(hipMemset(a, 1, bytes));
  CK(hipMemset(b, 0, bytes));
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double B = (double)bytes;
  for (int bs : {256, 512}) {
    for (int gridmul : {0, 4, 8, 16}) {
      char nm[128];
      auto grid = [&](int depth) {
        size_t full = (n16 + (size_t)bs * depth - 1) / ((size_t)bs * depth);
        return gridmul == 0 ? full : (size_t)(256 * gridmul) < full ? (size_t)(256 * gridmul) : full;
      };
      snprintf(nm, sizeof nm, "read  d8  bs%d grid%s%d", bs, gridmul ? "256x" : "full", gridmul);
      timeit(nm, B, [&] { hipLaunchKernelGGL((rd<8, 0>), dim3(grid(8)), dim3(bs), 0, 0, a, sink, n16); });
      snprintf(nm, sizeof nm, "readNT d8 bs%d grid%s%d", bs, gridmul ? "256x" : "full", gridmul);
      timeit(nm, B, [&] { hipLaunchKernelGGL((rd<8, 1>), dim3(grid(8)), dim3(bs), 0, 0, a, sink, n16); });
      snprintf(nm, sizeof nm, "write d8  bs%d grid%s%d", bs, gridmul ? "256x" : "full", gridmul);
      timeit(nm, B, [&] { hipLaunchKernelGGL((wr<8, 0>), dim3(grid(8)), dim3(bs), 0, 0, b, n16); });
      snprintf(nm, sizeof nm, "copy d4  bs%d grid%s%d", bs, gridmul ? "256x" : "full", gridmul);
      timeit(nm, 2 * B, [&] { hipLaunchKernelGGL((cp<4, 0, 0>), dim3(grid(4)), dim3(bs), 0, 0, a, b, n16); });
      snprintf(nm, sizeof nm, "copy d8  bs%d grid%s%d", bs, gridmul ? "256x" : "full", gridmul);
      timeit(nm, 2 * B, [&] { hipLaunchKernelGGL((cp<8, 0, 0>), dim3(grid(8)), dim3(bs), 0, 0, a, b, n16); });
      snprintf(nm, sizeof nm, "copy d16 bs%d grid%s%d", bs, gridmul ? "256x" : "full", gridmul);
      timeit(nm, 2 * B, [&] { hipLaunchKernelGGL((cp<16, 0, 0>), dim3(grid(16)), dim3(bs), 0, 0, a, b, n16); });
      snprintf(nm, sizeof nm, "copy d8 NTload bs%d grid%s%d", bs, gridmul ? "256x" : "full", gridmul);
      timeit(nm, 2 * B, [&] { hipLaunchKernelGGL((cp<8, 1, 0>), dim3(grid(8)), dim3(bs), 0, 0, a, b, n16); });
    }
  }
  return 0;
}
