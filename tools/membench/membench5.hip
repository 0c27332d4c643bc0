// Encode-shaped tile copies at 8 GiB (diagnostic for the transform kernel's tile shape).
// Blocks of 64 shards x S = 32 KiB; a tile is NC 64-byte chunks of the 32 data shards,
// copied to the same chunks of the 32 coding shards.  A workgroup of NWV waves copies one
// tile, each wave 32 / NWV shards (NC / 16 lane-linear 1 KiB accesses per shard).  XCD-
// contiguous tile order.  D: dependent VALU rounds over the loaded registers between the
// loads and the stores (stands in for the transform's arithmetic).
// Usage: membench5 [GiB]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t g) {
  const uint32_t x = b & 7, q = g >> 3, r = g & 7;
  return x * q + (x < r ? x : r) + (b >> 3);
}

template <int NC, int NWV, int WPE, int D, int QM = 0>
__global__ __launch_bounds__(64 * NWV, WPE) void tile_copy(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                           uint32_t S) {
  extern __shared__ int pad[];
  constexpr int K = 32, SH = K / NWV, Q = NC / 16;
  const uint32_t L = xcd_tile(blockIdx.x, gridDim.x);
  const uint32_t tiles_per_shard = S / (64 * NC);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t bstride = (size_t)2 * K * S;
  const uint32_t blk = L / tiles_per_shard, tt = L % tiles_per_shard;
  const uint8_t* src = in + blk * bstride + (size_t)tt * NC * 64 + lane * 16;
  uint8_t* dst = out + blk * bstride + (size_t)K * S + (size_t)tt * NC * 64 + lane * 16;
  u32x4 v[SH][Q];
  if constexpr (QM) {  // q-major: every shard's q-th KiB before the next KiB
#pragma unroll
    for (int q = 0; q < Q; ++q)
#pragma unroll
      for (int s = 0; s < SH; ++s) v[s][q] = *reinterpret_cast<const u32x4*>(src + (size_t)(wave * SH + s) * S + q * 1024);
  } else {
#pragma unroll
    for (int s = 0; s < SH; ++s)
#pragma unroll
      for (int q = 0; q < Q; ++q) v[s][q] = *reinterpret_cast<const u32x4*>(src + (size_t)(wave * SH + s) * S + q * 1024);
  }
#pragma unroll 1
  for (int d = 0; d < D; ++d) {
#pragma unroll
    for (int s = 0; s < SH; ++s)
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        v[s][q].x = __builtin_amdgcn_bitop3_b32(v[s][q].x, v[s][q].y, v[s][q].z, 0x96);
        v[s][q].y = __builtin_amdgcn_bitop3_b32(v[s][q].y, v[s][q].z, v[s][q].w, 0x96);
        v[s][q].z = __builtin_amdgcn_bitop3_b32(v[s][q].z, v[s][q].w, v[s][q].x, 0x96);
        v[s][q].w = __builtin_amdgcn_bitop3_b32(v[s][q].w, v[s][q].x, v[s][q].y, 0x96);
      }
  }
  if (v[0][0].x == 0xdeadbeef && threadIdx.x == 100000) pad[0] = 1;
  if constexpr (QM & 2) {
#pragma unroll
    for (int q = 0; q < Q; ++q)
#pragma unroll
      for (int s = 0; s < SH; ++s) *reinterpret_cast<u32x4*>(dst + (size_t)(wave * SH + s) * S + q * 1024) = v[s][q];
  } else {
#pragma unroll
    for (int s = 0; s < SH; ++s)
#pragma unroll
      for (int q = 0; q < Q; ++q) *reinterpret_cast<u32x4*>(dst + (size_t)(wave * SH + s) * S + q * 1024) = v[s][q];
  }
}

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);                \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

static hipEvent_t e0, e1;
template <typename F>
static void timeit(const char* name, double bytes_moved, F f) {
  f();
  CK(hipDeviceSynchronize());
  float best = 1e30f, sum = 0;
  const int reps = 10;
  for (int rep = 0; rep < reps; ++rep) {
    CK(hipEventRecord(e0));
    f();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
    sum += ms;
  }
  printf("%-44s best %7.3f ms %6.0f GB/s  mean %6.0f GB/s\n", name, best, bytes_moved / (best * 1e-3) / 1e9,
         bytes_moved / (sum / reps * 1e-3) / 1e9);
  fflush(stdout);
}

int main(int argc, char** argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 8.0;
  const size_t bytes = (size_t)(gib * (1ull << 30));
  uint8_t* a;
  CK(hipMalloc(&a, bytes));
  CK(hipMemset(a, 1, bytes));
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const uint32_t S = 32768;
  const size_t nblk = bytes / (64 * (size_t)S);
  const double moved = (double)nblk * 64 * S;
  char nm[128];
  // LDS per workgroup that caps the workgroups per CU at W (160 KiB LDS per CU)
  auto lds_cap = [](int w) { return w <= 0 ? 0 : (160 << 10) / w - 1024; };
#define TQ(NC, NWV, WPE, D, WGCU, QM)                                                                 \
  snprintf(nm, sizeof nm, "NC%d waves%d wpe%d D%d wg/cu<=%d qm%d", NC, NWV, WPE, D, WGCU, QM);         \
  timeit(nm, moved, [&] {                                                                              \
    hipLaunchKernelGGL((tile_copy<NC, NWV, WPE, D, QM>), dim3(nblk * (S / (64 * NC))), dim3(64 * NWV), \
                       lds_cap(WGCU), 0, (const uint8_t*)a, a, S);                                     \
  });
#define T(NC, NWV, WPE, D, WGCU) TQ(NC, NWV, WPE, D, WGCU, 0)
  // current transform shape: NC64, 4 waves x 8 shards, 2 WG/CU
  T(64, 4, 2, 0, 2)
  TQ(64, 4, 2, 0, 2, 1)
  TQ(64, 4, 2, 0, 2, 3)
  TQ(64, 4, 2, 43, 2, 1)
  TQ(64, 4, 2, 43, 2, 3)
  T(64, 8, 2, 0, 1)
  TQ(64, 8, 4, 0, 2, 0)
  TQ(64, 8, 4, 0, 2, 3)
  TQ(64, 8, 4, 43, 2, 3)
  TQ(32, 4, 2, 43, 4, 3)
  TQ(32, 8, 2, 43, 2, 3)
  // NC16 shapes
  T(16, 4, 2, 0, 2)
  T(16, 4, 2, 0, 0)
  T(16, 2, 2, 0, 4)
  T(16, 2, 2, 0, 0)
  T(16, 1, 2, 0, 8)
  T(16, 1, 2, 0, 4)
  T(16, 1, 2, 0, 0)
  // NC32
  T(32, 4, 2, 0, 2)
  T(32, 2, 2, 0, 2)
  T(32, 1, 1, 0, 4)
  // with arithmetic between loads and stores (D rounds x 4 VALU per 16-byte register)
  // the transform does ~43 rounds' worth (5.5k VALU per 32 KiB wave tile, PMC)
  T(64, 4, 2, 20, 2)
  T(64, 4, 2, 43, 2)
  T(16, 4, 2, 20, 2)
  T(16, 4, 2, 43, 2)
  T(16, 1, 2, 20, 8)
  T(16, 1, 2, 43, 8)
  T(16, 1, 2, 43, 4)
  T(16, 2, 2, 43, 4)
  return 0;
}
