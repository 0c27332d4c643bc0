// Copy ceiling vs bytes in flight per CU (diagnostic).  One-shot copies of U 16-byte
// pieces per thread; dynamic LDS caps the workgroups per CU.  Usage: membench4 [GiB]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U>
__global__ void cp1(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t n16) {
  extern __shared__ int pad[];
  const size_t base = (size_t)blockIdx.x * blockDim.x * U + threadIdx.x;
  u32x4 v[U];
#pragma unroll
  for (int k = 0; k < U; ++k) v[k] = in[base + (size_t)k * blockDim.x];
  if (v[0].x == 0xdeadbeef && threadIdx.x == 1000) pad[0] = 1;
#pragma unroll
  for (int k = 0; k < U; ++k) out[base + (size_t)k * blockDim.x] = v[k];
}

// tile-shaped copy: blocks of 2*K shards of S bytes; a workgroup of 4 waves copies tile t
// (NC 64-byte chunks of each of the K data shards) into the same chunks of the K coding
// shards; each wave owns K/4 shards, one 1 KiB lane-linear access per 16 chunks.
template <int NC, int K>
__global__ void tcp(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, uint32_t S) {
  extern __shared__ int pad[];
  const uint32_t tiles_per_shard = S / (64 * NC);
  const uint32_t blk = blockIdx.x / tiles_per_shard, tt = blockIdx.x % tiles_per_shard;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t bstride = (size_t)2 * K * S;
  const uint8_t* src = in + blk * bstride + (size_t)tt * NC * 64 + lane * 16;
  uint8_t* dst = out + blk * bstride + (size_t)K * S + (size_t)tt * NC * 64 + lane * 16;
  constexpr int SH = K / 4, Q = NC / 16;
  u32x4 v[SH][Q];
#pragma unroll
  for (int s = 0; s < SH; ++s)
#pragma unroll
    for (int q = 0; q < Q; ++q) v[s][q] = *reinterpret_cast<const u32x4*>(src + (size_t)(wave * SH + s) * S + q * 1024);
  if (v[0][0].x == 0xdeadbeef && threadIdx.x == 1000) pad[0] = 1;
#pragma unroll
  for (int s = 0; s < SH; ++s)
#pragma unroll
    for (int q = 0; q < Q; ++q) *reinterpret_cast<u32x4*>(dst + (size_t)(wave * SH + s) * S + q * 1024) = v[s][q];
}


// NC = 64 tile copy with the loads / stores issued in groups of G instructions, D dependent
// VALU ops between groups (mimics compute spread between load groups)
template <int G, int D, int PIPE>
__global__ void tcpg(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, uint32_t S) {
  extern __shared__ int pad[];
  constexpr int NC = 64, K = 32;
  const uint32_t tiles_per_shard = S / (64 * NC);
  const uint32_t blk = blockIdx.x / tiles_per_shard, tt = blockIdx.x % tiles_per_shard;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t bstride = (size_t)2 * K * S;
  const uint8_t* src = in + blk * bstride + (size_t)tt * NC * 64 + lane * 16;
  uint8_t* dst = out + blk * bstride + (size_t)K * S + (size_t)tt * NC * 64 + lane * 16;
  constexpr int SH = K / 4, Q = NC / 16, N = SH * Q;
  u32x4 v[N];
  uint32_t acc = threadIdx.x;
  auto addr = [&](int i) { return (size_t)(wave * SH + i / Q) * S + (i % Q) * 1024; };
  if constexpr (PIPE) {
    // software pipeline: load group g, then store group g - 1
#pragma unroll
    for (int g = 0; g <= N / G; ++g) {
      if (g < N / G) {
#pragma unroll
        for (int j = 0; j < G; ++j) v[g * G + j] = *reinterpret_cast<const u32x4*>(src + addr(g * G + j));
      }
#pragma unroll
      for (int d = 0; d < D; ++d) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(acc) : "v"(lane));
      if (g > 0) {
#pragma unroll
        for (int j = 0; j < G; ++j) *reinterpret_cast<u32x4*>(dst + addr((g - 1) * G + j)) = v[(g - 1) * G + j];
      }
    }
  } else {
#pragma unroll
    for (int g = 0; g < N / G; ++g) {
#pragma unroll
      for (int j = 0; j < G; ++j) v[g * G + j] = *reinterpret_cast<const u32x4*>(src + addr(g * G + j));
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int d = 0; d < D; ++d) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(acc) : "v"(lane));
      __builtin_amdgcn_sched_barrier(0);
    }
    if (v[0].x == 0xdeadbeef && threadIdx.x == 1000) pad[0] = 1;
#pragma unroll
    for (int g = 0; g < N / G; ++g) {
#pragma unroll
      for (int j = 0; j < G; ++j) *reinterpret_cast<u32x4*>(dst + addr(g * G + j)) = v[g * G + j];
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int d = 0; d < D; ++d) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(acc) : "v"(lane));
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (acc == 0x12345) pad[1] = acc;
}

// NC = 16 tile copies, T tiles per workgroup in sequence (persistent-ish)
template <int T>
__global__ void tcp16t(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, uint32_t S) {
  extern __shared__ int pad[];
  constexpr int NC = 16, K = 32, SH = 8;
  const uint32_t tiles_per_shard = S / (64 * NC);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t bstride = (size_t)2 * K * S;
#pragma unroll 1
  for (int t = 0; t < T; ++t) {
    const uint32_t tile = blockIdx.x * T + t;
    const uint32_t blk = tile / tiles_per_shard, tt = tile % tiles_per_shard;
    const uint8_t* src = in + blk * bstride + (size_t)tt * NC * 64 + lane * 16;
    uint8_t* dst = out + blk * bstride + (size_t)K * S + (size_t)tt * NC * 64 + lane * 16;
    u32x4 v[SH];
#pragma unroll
    for (int s = 0; s < SH; ++s) v[s] = *reinterpret_cast<const u32x4*>(src + (size_t)(wave * SH + s) * S);
#pragma unroll
    for (int s = 0; s < SH; ++s) *reinterpret_cast<u32x4*>(dst + (size_t)(wave * SH + s) * S) = v[s];
  }
}

// WG copies SUB sub-tiles of NC chunks x 32 shards (lane-linear 1 KiB per instruction).
// Sub-tile j of workgroup b is logical NC-tile L (block-major order):
//   SPREAD 0: L = b' * SUB + j        SPREAD 1: L = j * G + b'
// with b' = b (XCD 0) or the XCD-major remap b' = (b % 8) * (G / 8) + b / 8 (XCD 1).
template <int NC, int SUB, int SPREAD, int XCD>
__global__ void tcpx(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, uint32_t S) {
  extern __shared__ int pad[];
  constexpr int K = 32, SH = 8, Q = NC / 16;
  const uint32_t G = gridDim.x, b = blockIdx.x;
  const uint32_t bb = XCD ? (b % 8) * (G / 8) + b / 8 : b;
  const uint32_t tiles_per_shard = S / (64 * NC);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t bstride = (size_t)2 * K * S;
  u32x4 v[SUB][SH][Q];
#pragma unroll
  for (int j = 0; j < SUB; ++j) {
    const uint32_t L = SPREAD ? j * G + bb : bb * SUB + j;
    const uint32_t blk = L / tiles_per_shard, tt = L % tiles_per_shard;
    const uint8_t* src = in + blk * bstride + (size_t)tt * NC * 64 + lane * 16;
#pragma unroll
    for (int s = 0; s < SH; ++s)
#pragma unroll
      for (int q = 0; q < Q; ++q) v[j][s][q] = *reinterpret_cast<const u32x4*>(src + (size_t)(wave * SH + s) * S + q * 1024);
  }
  if (v[0][0][0].x == 0xdeadbeef && threadIdx.x == 1000) pad[0] = 1;
#pragma unroll
  for (int j = 0; j < SUB; ++j) {
    const uint32_t L = SPREAD ? j * G + bb : bb * SUB + j;
    const uint32_t blk = L / tiles_per_shard, tt = L % tiles_per_shard;
    uint8_t* dst = out + blk * bstride + (size_t)K * S + (size_t)tt * NC * 64 + lane * 16;
#pragma unroll
    for (int s = 0; s < SH; ++s)
#pragma unroll
      for (int q = 0; q < Q; ++q) *reinterpret_cast<u32x4*>(dst + (size_t)(wave * SH + s) * S + q * 1024) = v[j][s][q];
  }
}

// XCD-remapped tile copy: NC chunks x 32 shards per workgroup of NWV waves, each wave
// copying 32 / NWV shards (NC / 16 lane-linear 1 KiB loads per shard); ROWS: read/write
// shard counts (decode shape: read 32, write 16).
template <int NC, int NWV, int NWR>
__global__ void tcpw(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, uint32_t S) {
  extern __shared__ int pad[];
  constexpr int K = 32, SH = K / NWV, Q = NC / 16;
  const uint32_t G = gridDim.x, b = blockIdx.x;
  const uint32_t x = b & 7, q8 = G >> 3, r8 = G & 7;
  const uint32_t L = x * q8 + (x < r8 ? x : r8) + (b >> 3);
  const uint32_t tiles_per_shard = S / (64 * NC);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t bstride = (size_t)2 * K * S;
  const uint32_t blk = L / tiles_per_shard, tt = L % tiles_per_shard;
  const uint8_t* src = in + blk * bstride + (size_t)tt * NC * 64 + lane * 16;
  uint8_t* dst = out + blk * bstride + (size_t)K * S + (size_t)tt * NC * 64 + lane * 16;
  u32x4 v[SH][Q];
#pragma unroll
  for (int s = 0; s < SH; ++s)
#pragma unroll
    for (int q = 0; q < Q; ++q) v[s][q] = *reinterpret_cast<const u32x4*>(src + (size_t)(wave * SH + s) * S + q * 1024);
  if (v[0][0].x == 0xdeadbeef && threadIdx.x == 1000) pad[0] = 1;
  if (wave * SH < NWR) {
#pragma unroll
    for (int s = 0; s < SH; ++s)
#pragma unroll
      for (int q = 0; q < Q; ++q) *reinterpret_cast<u32x4*>(dst + (size_t)(wave * SH + s) * S + q * 1024) = v[s][q];
  }
}

// Persistent XCD-aware tile copy with prefetch: grid = 256 * WPC workgroups of NWV waves;
// the workgroups of XCD x walk that XCD's contiguous tile range with stride 32 * WPC, so
// the tiles in flight on an XCD are neighbours; the next tile's loads are issued before
// the current tile's D dependent VALU ops and stores.
template <int NWV, int WPC, int D, int NWR>
__global__ void tcpp(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, uint32_t S, uint32_t ntiles) {
  extern __shared__ int pad[];
  constexpr int NC = 64, K = 32, SH = K / NWV, Q = 4;
  const uint32_t b = blockIdx.x, x = b & 7, j = b >> 3;
  const uint32_t per = ntiles / 8, lo = x * per, hi = lo + per;  // ntiles % 8 == 0 here
  const uint32_t tiles_per_shard = S / (64 * NC);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t bstride = (size_t)2 * K * S;
  auto src_of = [&](uint32_t L) {
    const uint32_t blk = L / tiles_per_shard, tt = L % tiles_per_shard;
    return in + blk * bstride + (size_t)tt * NC * 64 + lane * 16;
  };
  auto dst_of = [&](uint32_t L) {
    const uint32_t blk = L / tiles_per_shard, tt = L % tiles_per_shard;
    return out + blk * bstride + (size_t)K * S + (size_t)tt * NC * 64 + lane * 16;
  };
  u32x4 v[2][SH][Q];
  uint32_t acc = lane;
  uint32_t L = lo + j;
  if (L >= hi) return;
  {
    const uint8_t* src = src_of(L);
#pragma unroll
    for (int s = 0; s < SH; ++s)
#pragma unroll
      for (int q = 0; q < Q; ++q) v[0][s][q] = *reinterpret_cast<const u32x4*>(src + (size_t)(wave * SH + s) * S + q * 1024);
  }
  int cur = 0;
  for (;;) {
    const uint32_t Ln = L + 32 * WPC;
    const bool more = Ln < hi;
    if (more) {
      const uint8_t* src = src_of(Ln);
#pragma unroll
      for (int s = 0; s < SH; ++s)
#pragma unroll
        for (int q = 0; q < Q; ++q)
          v[cur ^ 1][s][q] = *reinterpret_cast<const u32x4*>(src + (size_t)(wave * SH + s) * S + q * 1024);
    }
#pragma unroll
    for (int d = 0; d < D; ++d) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(acc) : "v"(v[cur][d % SH][d % Q].x));
    uint8_t* dst = dst_of(L);
    if (wave * SH < NWR) {
#pragma unroll
      for (int s = 0; s < SH; ++s)
#pragma unroll
        for (int q = 0; q < Q; ++q) *reinterpret_cast<u32x4*>(dst + (size_t)(wave * SH + s) * S + q * 1024) = v[cur][s][q];
    }
    if (!more) break;
    L = Ln;
    cur ^= 1;
  }
  if (acc == 0x12345) pad[0] = acc;
}

// NC64 tile copy (4 or 8 waves), XCD-contiguous tile ranges with an in-XCD order MODE:
//   0: consecutive tiles;  1: block-strided (consecutive workgroups take the same tile of
//   consecutive blocks);  2: consecutive, stores non-temporal;  3: consecutive, loads nt
template <int NWV, int NWR, int MODE>
__global__ void tcpm(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, uint32_t S) {
  extern __shared__ int pad[];
  constexpr int NC = 64, K = 32, SH = K / NWV, Q = 4;
  const uint32_t G = gridDim.x, b = blockIdx.x;
  const uint32_t x = b & 7, q8 = G >> 3;
  const uint32_t i = b >> 3;  // G % 8 == 0 here
  const uint32_t tiles_per_shard = S / (64 * NC);
  uint32_t L;
  if (MODE == 1) {
    const uint32_t nb = q8 / tiles_per_shard;  // blocks per XCD
    L = x * q8 + (i % nb) * tiles_per_shard + i / nb;
  } else {
    L = x * q8 + i;
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t bstride = (size_t)2 * K * S;
  const uint32_t blk = L / tiles_per_shard, tt = L % tiles_per_shard;
  const uint8_t* src = in + blk * bstride + (size_t)tt * NC * 64 + lane * 16;
  uint8_t* dst = out + blk * bstride + (size_t)K * S + (size_t)tt * NC * 64 + lane * 16;
  u32x4 v[SH][Q];
#pragma unroll
  for (int s = 0; s < SH; ++s)
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const u32x4* ptr = reinterpret_cast<const u32x4*>(src + (size_t)(wave * SH + s) * S + q * 1024);
      v[s][q] = MODE == 3 ? __builtin_nontemporal_load(ptr) : *ptr;
    }
  if (v[0][0].x == 0xdeadbeef && threadIdx.x == 1000) pad[0] = 1;
  if (wave * SH < NWR) {
#pragma unroll
    for (int s = 0; s < SH; ++s)
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        u32x4* ptr = reinterpret_cast<u32x4*>(dst + (size_t)(wave * SH + s) * S + q * 1024);
        if (MODE == 2) __builtin_nontemporal_store(v[s][q], ptr); else *ptr = v[s][q];
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
  printf("%-44s %7.3f ms %6.0f GB/s\n", name, best, bytes_moved / (best * 1e-3) / 1e9);
  fflush(stdout);
}

int main(int argc, char** argv) {
  double gib = argc > 1 ? atof(argv[1]) : 4.0;
  size_t bytes = (size_t)(gib * (1ull << 30));
  size_t n16 = bytes / 16;
  u32x4 *a, *b;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMemset(a, 1, bytes));
  CK(hipMemset(b, 0, bytes));
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double B2 = 2.0 * (double)bytes;
  char nm[128];
  const int lds_for_wg[] = {0, 100 << 10, 64 << 10, 0, 36 << 10, 0, 0, 0, 18 << 10};
#define ONE(U, BS, W)                                                                                  \
  snprintf(nm, sizeof nm, "cp1 U%d bs%d wg/cu<=%d", U, BS, W);                                        \
  timeit(nm, B2, [&] { hipLaunchKernelGGL((cp1<U>), dim3(n16 / (BS * U)), dim3(BS), lds_for_wg[W], 0, a, b, n16); });
  const uint32_t S = 32768;
  const size_t nblk = bytes / (2 * 32 * (size_t)S);
  const double TB = (double)nblk * 2 * 32 * S;
#define TW(NC, NWV, NWR, W)                                                                           \
  snprintf(nm, sizeof nm, "tcpw NC%d waves%d write%d wg/cu<=%d", NC, NWV, NWR, W);                    \
  timeit(nm, (double)nblk * (32 + NWR) * S, [&] { hipLaunchKernelGGL((tcpw<NC, NWV, NWR>), dim3(nblk * (S / (64 * NC))), \
                                          dim3(64 * NWV), lds_for_wg[W], 0, (const uint8_t*)a, (uint8_t*)a, S); });
#define TP(NWV, WPC, D, NWR)                                                                           \
  snprintf(nm, sizeof nm, "tcpp waves%d wg/cu=%d D%d write%d", NWV, WPC, D, NWR);                     \
  timeit(nm, (double)nblk * (32 + NWR) * S, [&] { hipLaunchKernelGGL((tcpp<NWV, WPC, D, NWR>), dim3(256 * WPC), \
                                          dim3(64 * NWV), lds_for_wg[WPC], 0, (const uint8_t*)a, (uint8_t*)a, S, (uint32_t)(nblk * (S / 4096))); });
#define TM(NWV, NWR, MODE, W)                                                                          \
  snprintf(nm, sizeof nm, "tcpm waves%d write%d mode%d wg/cu<=%d", NWV, NWR, MODE, W);                 \
  timeit(nm, (double)nblk * (32 + NWR) * S, [&] { hipLaunchKernelGGL((tcpm<NWV, NWR, MODE>), dim3(nblk * (S / 4096)), \
                                          dim3(64 * NWV), lds_for_wg[W], 0, (const uint8_t*)a, (uint8_t*)a, S); });
  TM(4, 32, 0, 2) TM(4, 32, 1, 2) TM(4, 32, 2, 2) TM(4, 32, 3, 2) TM(8, 32, 0, 2) TM(8, 32, 1, 2) TM(8, 32, 2, 2)
  TM(4, 16, 0, 2) TM(4, 16, 1, 2) TM(8, 16, 0, 2) TM(8, 16, 1, 2) TM(8, 16, 3, 2)
  return 0;
}
