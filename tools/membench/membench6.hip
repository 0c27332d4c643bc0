// Issue-order experiments on the encode-shaped tile copy (diagnostic for xform<4>).
// Blocks of 64 shards x S = 32 KiB; a tile is NC 64-byte chunks of the 32 data shards,
// copied to the same chunks of the 32 coding shards; NWV waves, each 32 / NWV shards.
// ORD selects the order in which a wave issues its loads (and stores):
//   0 shard-major (s, q)            1 q-major (q, s)
//   2 q rotated by the tile         3 shard rotated by the tile
//   4 both rotated                  5 shard rotated by tile, q rotated by shard
// The register a piece lands in never depends on ORD (static indices); only the address
// does, so this is exactly a change of issue order.  D: dependent VALU rounds.
// Usage: membench6 [GiB]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t g) {
  const uint32_t x = b & 7, q = g >> 3, r = g & 7;
  return x * q + (x < r ? x : r) + (b >> 3);
}

template <int NC, int NWV, int WPE, int D, int ORD, int WR = 32>
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
  const uint32_t rq = (ORD == 2 || ORD == 4) ? (L & (Q - 1)) : 0;
  const uint32_t rs = (ORD == 3 || ORD == 4 || ORD == 5) ? (L % SH) : 0;
  auto sidx = [&](int s) { return (uint32_t)(wave * SH) + ((uint32_t)s + rs) % SH; };
  auto qidx = [&](int s, int q) { return ORD == 5 ? ((uint32_t)q + (uint32_t)s) & (Q - 1) : ((uint32_t)q + rq) & (Q - 1); };
  u32x4 v[SH][Q];
  if constexpr (ORD == 1) {
#pragma unroll
    for (int q = 0; q < Q; ++q)
#pragma unroll
      for (int s = 0; s < SH; ++s) v[s][q] = *reinterpret_cast<const u32x4*>(src + (size_t)sidx(s) * S + qidx(s, q) * 1024);
  } else {
#pragma unroll
    for (int s = 0; s < SH; ++s)
#pragma unroll
      for (int q = 0; q < Q; ++q) v[s][q] = *reinterpret_cast<const u32x4*>(src + (size_t)sidx(s) * S + qidx(s, q) * 1024);
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
  if constexpr (WR < SH) {  // keep the unstored shards' loads live
#pragma unroll
    for (int s = WR; s < SH; ++s)
#pragma unroll
      for (int q = 0; q < Q; ++q) v[s % WR][q] ^= v[s][q];
  }
  if constexpr (ORD == 1) {
#pragma unroll
    for (int q = 0; q < Q; ++q)
#pragma unroll
      for (int s = 0; s < SH; ++s) *reinterpret_cast<u32x4*>(dst + (size_t)sidx(s) * S + qidx(s, q) * 1024) = v[s][q];
  } else {
#pragma unroll
    for (int s = 0; s < (WR < SH ? WR : SH); ++s)
#pragma unroll
      for (int q = 0; q < Q; ++q) *reinterpret_cast<u32x4*>(dst + (size_t)sidx(s) * S + qidx(s, q) * 1024) = v[s][q];
  }
}


// Split tiles: a workgroup copies TWO 32-chunk column ranges (regions A and B) of the 32
// data shards; lanes 0..31 of every 1 KiB wave access take 512 B of region A, lanes 32..63
// 512 B of region B (4 accesses per shard per region = 2 KiB each).  MAP: 0 A = 2u, B = 2u + 1
// (the NC64 footprint), 1 A = u, B = u + N (far), 2 the same column range of blocks 2j, 2j + 1.
template <int NWV, int WPE, int D, int MAP>
__global__ __launch_bounds__(64 * NWV, WPE) void split_copy(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                            uint32_t S) {
  extern __shared__ int pad[];
  constexpr int K = 32, SH = K / NWV, Q = 4;
  const uint32_t u = xcd_tile(blockIdx.x, gridDim.x), N = gridDim.x;
  const uint32_t tps = S / 2048;  // 32-chunk ranges per shard
  uint32_t A, B;
  if (MAP == 0) { A = 2 * u; B = 2 * u + 1; }
  else if (MAP == 1) { A = u; B = u + N; }
  else { const uint32_t j = u / tps, c = u % tps; A = 2 * j * tps + c; B = (2 * j + 1) * tps + c; }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t R = lane < 32 ? A : B;
  const size_t bstride = (size_t)2 * K * S;
  const uint32_t blk = R / tps, tt = R % tps;
  const uint8_t* src = in + blk * bstride + (size_t)tt * 2048 + (lane & 31) * 16;
  uint8_t* dst = out + blk * bstride + (size_t)K * S + (size_t)tt * 2048 + (lane & 31) * 16;
  u32x4 v[SH][Q];
#pragma unroll
  for (int s = 0; s < SH; ++s)
#pragma unroll
    for (int q = 0; q < Q; ++q) v[s][q] = *reinterpret_cast<const u32x4*>(src + (size_t)(wave * SH + s) * S + q * 512);
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
#pragma unroll
  for (int s = 0; s < SH; ++s)
#pragma unroll
    for (int q = 0; q < Q; ++q) *reinterpret_cast<u32x4*>(dst + (size_t)(wave * SH + s) * S + q * 512) = v[s][q];
}

// plain one-shot copy, U 16-byte pieces per thread (the copy ceiling)
template <int U>
__global__ void cp1(const u32x4* __restrict__ in, u32x4* __restrict__ out) {
  const size_t base = (size_t)blockIdx.x * blockDim.x * U + threadIdx.x;
  u32x4 v[U];
#pragma unroll
  for (int k = 0; k < U; ++k) v[k] = in[base + (size_t)k * blockDim.x];
#pragma unroll
  for (int k = 0; k < U; ++k) out[base + (size_t)k * blockDim.x] = v[k];
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
  for (int w = 0; w < 3; ++w) f();
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
  printf("%-40s best %7.3f ms %6.0f GB/s  mean %6.0f GB/s\n", name, best, bytes_moved / (best * 1e-3) / 1e9,
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
  auto lds_cap = [](int w) { return w <= 0 ? 0 : (160 << 10) / w - 1024; };
#define T(NC, NWV, WPE, D, WGCU, ORD)                                                                  \
  snprintf(nm, sizeof nm, "NC%d w%d D%d wg/cu<=%d ord%d", NC, NWV, D, WGCU, ORD);                      \
  timeit(nm, moved, [&] {                                                                              \
    hipLaunchKernelGGL((tile_copy<NC, NWV, WPE, D, ORD>), dim3(nblk * (S / (64 * NC))), dim3(64 * NWV), \
                       lds_cap(WGCU), 0, (const uint8_t*)a, a, S);                                     \
  });
  timeit("cp1 U1 bs256", (double)bytes, [&] {
    hipLaunchKernelGGL((cp1<1>), dim3(bytes / 2 / 16 / 256), dim3(256), 0, 0, (const u32x4*)a,
                       (u32x4*)(a + bytes / 2));
  });
#define TW(NC, NWV, WPE, D, WGCU, WR)                                                                  \
  snprintf(nm, sizeof nm, "NC%d w%d D%d wg/cu<=%d write %d of %d", NC, NWV, D, WGCU, WR, 32 / NWV);    \
  timeit(nm, movedw(WR, 32 / NWV), [&] {                                                               \
    hipLaunchKernelGGL((tile_copy<NC, NWV, WPE, D, 0, WR>), dim3(nblk * (S / (64 * NC))), dim3(64 * NWV), \
                       lds_cap(WGCU), 0, (const uint8_t*)a, a, S);                                     \
  });
  // reconstruct shape: read 32 shards, write 16 (bytes counted: 1.5 x the data shards)
  auto movedw = [&](int wr, int sh) { return (double)nblk * 32 * S * (1.0 + (double)wr / sh); };
  for (int rep = 0; rep < 2; ++rep) {
    T(64, 4, 2, 43, 2, 0)
    TW(64, 8, 4, 20, 2, 2)
    TW(64, 8, 4, 10, 2, 2)
    TW(64, 8, 4, 0, 2, 2)
    TW(64, 4, 2, 20, 2, 4)
    TW(32, 8, 4, 20, 2, 2)
    TW(32, 4, 2, 20, 2, 4)
  }
  return 0;
}
