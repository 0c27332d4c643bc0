// Copy-ceiling exploration (diagnostic): one-shot vs grid-stride copies, unroll depth,
// block size, non-temporal / sc bits on buffer loads and stores, buffer size.
// Usage: membench3 [GiB]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// one-shot: each thread copies U 16-byte pieces, block-strided (lane-linear per instruction)
template <int U, int NTL, int NTS>
__global__ void cp1(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t n16) {
  const size_t base = (size_t)blockIdx.x * blockDim.x * U + threadIdx.x;
  u32x4 v[U];
#pragma unroll
  for (int k = 0; k < U; ++k) {
    const size_t j = base + (size_t)k * blockDim.x;
    v[k] = NTL ? __builtin_nontemporal_load(in + j) : in[j];
  }
#pragma unroll
  for (int k = 0; k < U; ++k) {
    const size_t j = base + (size_t)k * blockDim.x;
    if (NTS) __builtin_nontemporal_store(v[k], out + j); else out[j] = v[k];
  }
}

// buffer-instruction copy with cache-policy aux bits (gfx950: bit0 sc0, bit1 nt, bit4 sc1 ...)
template <int U, int AL, int AS>
__global__ void cpb(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t n16) {
  const size_t blk_bytes = (size_t)blockDim.x * U * 16;
  const char* ib = reinterpret_cast<const char*>(in) + blockIdx.x * blk_bytes;
  char* ob = reinterpret_cast<char*>(out) + blockIdx.x * blk_bytes;
  auto ri = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(ib), 0, (int)blk_bytes, 0x00020000);
  auto ro = __builtin_amdgcn_make_buffer_rsrc(ob, 0, (int)blk_bytes, 0x00020000);
  u32x4 v[U];
#pragma unroll
  for (int k = 0; k < U; ++k)
    v[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ri, (threadIdx.x + k * blockDim.x) * 16, 0, AL));
#pragma unroll
  for (int k = 0; k < U; ++k)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, v[k]), ro,
                                           (threadIdx.x + k * blockDim.x) * 16, 0, AS);
}

// grid-stride persistent copy
template <int U>
__global__ void cpg(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t n16) {
  for (size_t base = (size_t)blockIdx.x * blockDim.x * U + threadIdx.x; base < n16;
       base += (size_t)gridDim.x * blockDim.x * U) {
    u32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = in[base + (size_t)k * blockDim.x];
#pragma unroll
    for (int k = 0; k < U; ++k) out[base + (size_t)k * blockDim.x] = v[k];
  }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

static hipEvent_t e0, e1;
template <typename F>
static void timeit(const char* name, double bytes_moved, F f) {
  f();
  CK(hipDeviceSynchronize());
  float best = 1e30f, sum = 0;
  for (int rep = 0; rep < 7; ++rep) {
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
         bytes_moved / (sum / 7 * 1e-3) / 1e9);
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
#define ONE(U, L, S, BS)                                                                                 \
  snprintf(nm, sizeof nm, "cp1 U%d ntl%d nts%d bs%d", U, L, S, BS);                                     \
  timeit(nm, B2, [&] { hipLaunchKernelGGL((cp1<U, L, S>), dim3(n16 / (BS * U)), dim3(BS), 0, 0, a, b, n16); });
  ONE(1, 0, 0, 256) ONE(2, 0, 0, 256) ONE(4, 0, 0, 256) ONE(8, 0, 0, 256) ONE(16, 0, 0, 256)
  ONE(4, 0, 0, 64) ONE(4, 0, 0, 128) ONE(4, 0, 0, 512) ONE(4, 0, 0, 1024)
  ONE(8, 0, 0, 512) ONE(8, 0, 0, 1024)
  ONE(4, 1, 0, 256) ONE(4, 0, 1, 256) ONE(4, 1, 1, 256) ONE(8, 1, 1, 256) ONE(8, 1, 0, 512)
#define BUF(U, L, S, BS)                                                                                 \
  snprintf(nm, sizeof nm, "cpb U%d auxL%d auxS%d bs%d", U, L, S, BS);                                   \
  timeit(nm, B2, [&] { hipLaunchKernelGGL((cpb<U, L, S>), dim3(n16 / (BS * U)), dim3(BS), 0, 0, a, b, n16); });
  BUF(4, 0, 0, 256) BUF(4, 2, 0, 256) BUF(4, 0, 2, 256) BUF(4, 2, 2, 256) BUF(4, 1, 0, 256) BUF(4, 0, 1, 256)
  BUF(4, 16, 0, 256) BUF(4, 0, 16, 256) BUF(4, 3, 3, 256) BUF(8, 2, 2, 256) BUF(8, 0, 0, 256) BUF(4, 17, 17, 256)
#define GS(U, BS, G)                                                                                     \
  snprintf(nm, sizeof nm, "cpg U%d bs%d grid%d", U, BS, G);                                             \
  timeit(nm, B2, [&] { hipLaunchKernelGGL((cpg<U>), dim3(G), dim3(BS), 0, 0, a, b, n16); });
  GS(4, 256, 1024) GS(4, 256, 2048) GS(4, 256, 4096) GS(8, 256, 2048) GS(4, 512, 2048) GS(2, 1024, 2048)
  return 0;
}
