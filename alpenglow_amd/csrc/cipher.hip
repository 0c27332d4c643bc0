// All-or-nothing payload transforms of the AONT and PETS shredders.
//
// What it replaces (per slice, before ReedSolomonCoder::shred / after ::deshred):
//   AontShredder::shred    payload := AES-128-CTR_key(payload) || key ^ SHA-256(ciphertext)[0..16)
//                          (shredder.rs:463-470)
//   PetsShredder::shred    payload := AES-128-CTR_key(payload) || key      (shredder.rs:414-418)
//   decrypt_payload        split the 16-byte tail, derive the key (AONT: tail ^ SHA-256 of the
//                          ciphertext; PETS: the tail), decrypt in place (shredder.rs:509-528)
//   cipher::apply_keystream  ctr::Ctr64LE<Aes128>, all-zero IV (crypto/cipher.rs:25-30):
//                          keystream block i = AES_key(LE64(i) || 0^8)
//   hash::hash             SHA-256 (crypto/hash.rs:64-67; sha256.hpp)
// The random key itself comes from the host (encrypt_with_random_key, cipher.rs:35-40).
//
// Kernels
//   aes_ctr_kernel      one workgroup per 32 KiB segment of a buffer, eight 16-byte blocks per
//                       thread: AES-128 with Te0 in LDS, one copy per bank (conflict-free
//                       lookups; rotations for Te1..3, byte 1 as the S-box), round keys
//                       expanded per workgroup and held in scalar registers.
//   sha256_buf_kernel   one thread per buffer (SHA-256 is sequential within a message), the
//                       next block's loads in flight during each block's rounds.
//   key tail / derive   one thread per buffer.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "cipher.hpp"
#include "sha256.hpp"
#include "unaligned.hpp"

namespace ag {
namespace aes {

// ---- tables (FIPS-197 §5.1.1: S-box = affine(GF(2^8) inverse), poly 0x11B) ----------
constexpr uint8_t gmul(uint8_t a, uint8_t b) {
  uint8_t p = 0;
  for (int i = 0; i < 8; ++i) {
    if (b & 1) p ^= a;
    const bool hi = a & 0x80;
    a = static_cast<uint8_t>(a << 1);
    if (hi) a ^= 0x1B;
    b >>= 1;
  }
  return p;
}
constexpr uint8_t ginv(uint8_t a) {  // a^254
  uint8_t r = 1, x = a;
  for (int e = 254; e; e >>= 1) {
    if (e & 1) r = gmul(r, x);
    x = gmul(x, x);
  }
  return a ? r : 0;
}
constexpr uint8_t rotl8(uint8_t x, int n) { return static_cast<uint8_t>((x << n) | (x >> (8 - n))); }
struct Tables {
  uint8_t sbox[256];
  uint32_t te0[256];  // big-endian column (2s, s, s, 3s)
};
constexpr Tables make_tables() {
  Tables t{};
  for (int i = 0; i < 256; ++i) {
    const uint8_t b = ginv(static_cast<uint8_t>(i));
    const uint8_t s = static_cast<uint8_t>(b ^ rotl8(b, 1) ^ rotl8(b, 2) ^ rotl8(b, 3) ^ rotl8(b, 4) ^ 0x63);
    t.sbox[i] = s;
    t.te0[i] = (uint32_t(gmul(s, 2)) << 24) | (uint32_t(s) << 16) | (uint32_t(s) << 8) | uint32_t(gmul(s, 3));
  }
  return t;
}
constexpr Tables kTables = make_tables();
static_assert(kTables.sbox[0] == 0x63 && kTables.sbox[1] == 0x7C && kTables.sbox[0x53] == 0xED, "AES S-box");
__constant__ Tables kDevTables = make_tables();

__host__ __device__ inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
__host__ __device__ inline uint32_t getu32(const uint8_t* p) {
  return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | uint32_t(p[3]);
}

// AES-128 key schedule (FIPS-197 §5.2): 44 words.
template <typename SBOX>
__host__ __device__ inline void expand(const uint8_t key[16], uint32_t rk[44], SBOX&& sb) {
  constexpr uint32_t rcon[10] = {0x01000000, 0x02000000, 0x04000000, 0x08000000, 0x10000000,
                                 0x20000000, 0x40000000, 0x80000000, 0x1B000000, 0x36000000};
  for (int i = 0; i < 4; ++i) rk[i] = getu32(key + 4 * i);
  for (int r = 0; r < 10; ++r) {
    const uint32_t t = rk[4 * r + 3];
    rk[4 * r + 4] = rk[4 * r] ^ (uint32_t(sb((t >> 16) & 0xFF)) << 24) ^ (uint32_t(sb((t >> 8) & 0xFF)) << 16) ^
                    (uint32_t(sb(t & 0xFF)) << 8) ^ uint32_t(sb(t >> 24)) ^ rcon[r];
    rk[4 * r + 5] = rk[4 * r + 1] ^ rk[4 * r + 4];
    rk[4 * r + 6] = rk[4 * r + 2] ^ rk[4 * r + 5];
    rk[4 * r + 7] = rk[4 * r + 3] ^ rk[4 * r + 6];
  }
}

// One block: state words (big-endian byte order) in s[4], out in s[4].
template <typename TE, typename SBOX>
__host__ __device__ inline void encrypt(uint32_t s[4], const uint32_t* rk, TE&& te, SBOX&& sb) {
  uint32_t s0 = s[0] ^ rk[0], s1 = s[1] ^ rk[1], s2 = s[2] ^ rk[2], s3 = s[3] ^ rk[3];
  for (int r = 1; r < 10; ++r) {
    const uint32_t* k = rk + 4 * r;
    const uint32_t t0 = te(s0 >> 24) ^ rotr(te((s1 >> 16) & 0xFF), 8) ^ rotr(te((s2 >> 8) & 0xFF), 16) ^
                        rotr(te(s3 & 0xFF), 24) ^ k[0];
    const uint32_t t1 = te(s1 >> 24) ^ rotr(te((s2 >> 16) & 0xFF), 8) ^ rotr(te((s3 >> 8) & 0xFF), 16) ^
                        rotr(te(s0 & 0xFF), 24) ^ k[1];
    const uint32_t t2 = te(s2 >> 24) ^ rotr(te((s3 >> 16) & 0xFF), 8) ^ rotr(te((s0 >> 8) & 0xFF), 16) ^
                        rotr(te(s1 & 0xFF), 24) ^ k[2];
    const uint32_t t3 = te(s3 >> 24) ^ rotr(te((s0 >> 16) & 0xFF), 8) ^ rotr(te((s1 >> 8) & 0xFF), 16) ^
                        rotr(te(s2 & 0xFF), 24) ^ k[3];
    s0 = t0;
    s1 = t1;
    s2 = t2;
    s3 = t3;
  }
  const uint32_t* k = rk + 40;
  auto last = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return (uint32_t(sb(a >> 24)) << 24) | (uint32_t(sb((b >> 16) & 0xFF)) << 16) |
           (uint32_t(sb((c >> 8) & 0xFF)) << 8) | uint32_t(sb(d & 0xFF));
  };
  s[0] = last(s0, s1, s2, s3) ^ k[0];
  s[1] = last(s1, s2, s3, s0) ^ k[1];
  s[2] = last(s2, s3, s0, s1) ^ k[2];
  s[3] = last(s3, s0, s1, s2) ^ k[3];
}

}  // namespace aes

void aes128_encrypt_block(const uint8_t key[16], const uint8_t in[16], uint8_t out[16]) {
  auto sb = [](uint32_t i) { return aes::kTables.sbox[i]; };
  auto te = [](uint32_t i) { return aes::kTables.te0[i]; };
  uint32_t rk[44];
  aes::expand(key, rk, sb);
  uint32_t s[4] = {aes::getu32(in), aes::getu32(in + 4), aes::getu32(in + 8), aes::getu32(in + 12)};
  aes::encrypt(s, rk, te, sb);
  for (int i = 0; i < 4; ++i)
    for (int b = 0; b < 4; ++b) out[4 * i + b] = static_cast<uint8_t>(s[i] >> (24 - 8 * b));
}

namespace {

constexpr uint32_t kAesThreads = 256, kAesPer = 8;           // 16-byte blocks per thread
constexpr uint32_t kSegBytes = kAesThreads * kAesPer * 16;  // 32 KiB per workgroup
constexpr uint32_t kTeCopies = 32;                          // one Te0 copy per LDS bank of ds_read_b32

// Te0 entry of the byte at bit `sh` of s, from the lane's own bank copy: byte address
// byte * 128 + (lane & 31) * 4, so the 32 lanes of a ds_read_b32 group never share a bank (a
// random lookup into one shared table costs ~3.5 LDS cycles per group instead of 1).
template <int SH>
__device__ __forceinline__ uint32_t te_at(const uint32_t* te, uint32_t s, uint32_t lane4) {
  const uint32_t a = (SH >= 7 ? (s >> (SH - 7)) : (s << (7 - SH))) & 0x7F80u;
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(te) + (a | lane4));
}

__global__ __launch_bounds__(256) void aes_ctr_kernel(const BufferBatch bb, const uint8_t* __restrict__ keys,
                                                      uint32_t lens_delta, uint32_t segs) {
  __shared__ uint32_t te[256 * kTeCopies];  // entry i, copy c at i * 32 + c (32 KiB)
  __shared__ uint32_t rk_s[44];
  const uint64_t b = blockIdx.x / segs;
  const uint32_t seg = blockIdx.x - static_cast<uint32_t>(b * segs);
  if (b >= bb.n) return;
  const uint32_t lenb = bb.lens[b];
  const uint32_t len = lenb > lens_delta ? lenb - lens_delta : 0;
  if (static_cast<uint64_t>(seg) * kSegBytes >= len) return;  // whole workgroup
#pragma unroll
  for (uint32_t k = 0; k < kTeCopies; ++k) {  // lane-consecutive words: conflict-free stores
    const uint32_t w = threadIdx.x + kAesThreads * k;
    te[w] = aes::kDevTables.te0[w / kTeCopies];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint8_t key[16];
    for (int i = 0; i < 16; ++i) key[i] = keys[16 * b + i];
    aes::expand(key, rk_s, [&](uint32_t i) { return (te[i * kTeCopies] >> 8) & 0xFFu; });  // S-box = byte 1
  }
  __syncthreads();
  uint32_t rk[44];
#pragma unroll
  for (int i = 0; i < 44; ++i) rk[i] = __builtin_amdgcn_readfirstlane(rk_s[i]);
  const uint32_t l4 = (threadIdx.x & 31) * 4;
  uint8_t* const base = bb.base + b * bb.stride;
  for (uint32_t k = 0; k < kAesPer; ++k) {
    const uint64_t blk = static_cast<uint64_t>(seg) * (kSegBytes / 16) + k * kAesThreads + threadIdx.x;  // counter
    const uint64_t off = 16 * blk;
    if (off >= len) break;
    // Ctr64LE with a zero IV: block = LE64(counter) || 0^8 (state words big-endian)
    uint32_t s0 = sha::bswap(static_cast<uint32_t>(blk)) ^ rk[0], s1 = sha::bswap(static_cast<uint32_t>(blk >> 32)) ^ rk[1];
    uint32_t s2 = rk[2], s3 = rk[3];
#pragma unroll
    for (int r = 1; r < 10; ++r) {
      const uint32_t t0 = te_at<24>(te, s0, l4) ^ aes::rotr(te_at<16>(te, s1, l4), 8) ^
                          aes::rotr(te_at<8>(te, s2, l4), 16) ^ aes::rotr(te_at<0>(te, s3, l4), 24) ^ rk[4 * r];
      const uint32_t t1 = te_at<24>(te, s1, l4) ^ aes::rotr(te_at<16>(te, s2, l4), 8) ^
                          aes::rotr(te_at<8>(te, s3, l4), 16) ^ aes::rotr(te_at<0>(te, s0, l4), 24) ^ rk[4 * r + 1];
      const uint32_t t2 = te_at<24>(te, s2, l4) ^ aes::rotr(te_at<16>(te, s3, l4), 8) ^
                          aes::rotr(te_at<8>(te, s0, l4), 16) ^ aes::rotr(te_at<0>(te, s1, l4), 24) ^ rk[4 * r + 2];
      const uint32_t t3 = te_at<24>(te, s3, l4) ^ aes::rotr(te_at<16>(te, s0, l4), 8) ^
                          aes::rotr(te_at<8>(te, s1, l4), 16) ^ aes::rotr(te_at<0>(te, s2, l4), 24) ^ rk[4 * r + 3];
      s0 = t0;
      s1 = t1;
      s2 = t2;
      s3 = t3;
    }
    // last round: SubBytes + ShiftRows; the S-box value is byte 1 of the Te0 entry
    auto last = [&](uint32_t a, uint32_t bq, uint32_t c, uint32_t d) __attribute__((always_inline)) {
      return ((te_at<24>(te, a, l4) & 0xFF00u) << 16) | (te_at<16>(te, bq, l4) & 0xFF0000u) |
             (te_at<8>(te, c, l4) & 0xFF00u) | ((te_at<0>(te, d, l4) >> 8) & 0xFFu);
    };
    const uint32_t k0 = sha::bswap(last(s0, s1, s2, s3) ^ rk[40]), k1 = sha::bswap(last(s1, s2, s3, s0) ^ rk[41]);
    const uint32_t k2 = sha::bswap(last(s2, s3, s0, s1) ^ rk[42]), k3 = sha::bswap(last(s3, s0, s1, s2) ^ rk[43]);
    uint8_t* p = base + off;
    if (len - off >= 16) {
      uint4 x = ld16u(p);
      x.x ^= k0;
      x.y ^= k1;
      x.z ^= k2;
      x.w ^= k3;
      st16u(p, x);
    } else {
      const uint32_t ks[4] = {k0, k1, k2, k3};
      for (uint32_t i = 0; i < len - off; ++i) p[i] ^= static_cast<uint8_t>(ks[i >> 2] >> (8 * (i & 3)));
    }
  }
}

// SHA-256 of p[0..L) (message words big-endian; any alignment).  One message per lane (a
// batch's messages are the parallelism): the next whole block's four 16-byte loads are issued
// before this block's rounds, so the rounds hide the load latency.
__device__ void sha256_bytes(const uint8_t* __restrict__ p, uint32_t L, uint32_t out[8]) {
  uint32_t st[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) st[i] = sha::kIv[i];
  const uint32_t nblk = (L + 9 + 63) / 64, nfull = L / 64;
  uint4 nx[4];
  auto fetch = [&](uint32_t b) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 4; ++q) nx[q] = ld16u(p + 64 * b + 16 * q);
  };
  if (nfull) fetch(0);
  for (uint32_t b = 0; b < nfull; ++b) {
    uint32_t w[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      w[4 * q] = sha::bswap(nx[q].x);
      w[4 * q + 1] = sha::bswap(nx[q].y);
      w[4 * q + 2] = sha::bswap(nx[q].z);
      w[4 * q + 3] = sha::bswap(nx[q].w);
    }
    if (b + 1 < nfull) fetch(b + 1);
    sha::compress(st, w);
  }
  for (uint32_t b = nfull; b < nblk; ++b) {  // the padding blocks
    uint32_t w[16];
    const uint32_t o0 = 64 * b;
    for (int i = 0; i < 16; ++i) {
      const uint32_t o = o0 + 4 * i;
      uint32_t v = 0;
      if (b == nblk - 1 && i == 15) {
        v = L * 8;
      } else if (!(b == nblk - 1 && i == 14)) {
        for (uint32_t k = 0; k < 4; ++k) {
          const uint32_t ob = o + k;
          const uint32_t bv = ob < L ? p[ob] : (ob == L ? 0x80u : 0u);
          v |= bv << (24 - 8 * k);
        }
      }
      w[i] = v;
    }
    sha::compress(st, w);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) out[i] = st[i];
}

__global__ __launch_bounds__(64) void sha256_buf_kernel(const BufferBatch bb, uint32_t lens_delta,
                                                        uint8_t* __restrict__ digests) {
  const uint64_t b = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b >= bb.n) return;
  const uint32_t lenb = bb.lens[b];
  uint32_t h[8];
  sha256_bytes(bb.base + b * bb.stride, lenb > lens_delta ? lenb - lens_delta : 0, h);
  for (int i = 0; i < 8; ++i)
    for (int k = 0; k < 4; ++k) digests[32 * b + 4 * i + k] = static_cast<uint8_t>(h[i] >> (24 - 8 * k));
}

__global__ __launch_bounds__(256) void key_tail_kernel(const BufferBatch bb, int aont, const uint8_t* __restrict__ keys,
                                                       const uint8_t* __restrict__ digests) {
  const uint64_t b = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b >= bb.n) return;
  uint8_t* tail = bb.base + b * bb.stride + bb.lens[b];
  for (int i = 0; i < 16; ++i) tail[i] = static_cast<uint8_t>(keys[16 * b + i] ^ (aont ? digests[32 * b + i] : 0));
}

__global__ __launch_bounds__(256) void derive_keys_kernel(const BufferBatch bb, int aont,
                                                          const uint8_t* __restrict__ digests, uint8_t* keys) {
  const uint64_t b = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b >= bb.n) return;
  const uint32_t len = bb.lens[b];
  const uint8_t* tail = bb.base + b * bb.stride + (len - 16);
  for (int i = 0; i < 16; ++i) keys[16 * b + i] = static_cast<uint8_t>(tail[i] ^ (aont ? digests[32 * b + i] : 0));
}

dim3 grid_for(uint64_t threads, uint32_t per) { return dim3(static_cast<unsigned>((threads + per - 1) / per)); }

}  // namespace

hipError_t launch_apply_keystream(const BufferBatch& b, const uint8_t* keys, uint32_t lens_delta, hipStream_t stream) {
  if (b.n == 0 || b.max_len <= lens_delta) return hipSuccess;
  const uint32_t segs = (b.max_len - lens_delta + kSegBytes - 1) / kSegBytes;
  if (b.n * segs > 0x7FFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(aes_ctr_kernel, dim3(static_cast<unsigned>(b.n * segs)), dim3(256), 0, stream, b, keys,
                     lens_delta, segs);
  return hipGetLastError();
}

hipError_t launch_sha256(const BufferBatch& b, uint32_t lens_delta, uint8_t* digests, hipStream_t stream) {
  if (b.n == 0) return hipSuccess;
  hipLaunchKernelGGL(sha256_buf_kernel, grid_for(b.n, 64), dim3(64), 0, stream, b, lens_delta, digests);
  return hipGetLastError();
}

hipError_t launch_write_key_tail(const BufferBatch& b, int aont, const uint8_t* keys, const uint8_t* digests,
                                 hipStream_t stream) {
  if (b.n == 0) return hipSuccess;
  hipLaunchKernelGGL(key_tail_kernel, grid_for(b.n, 256), dim3(256), 0, stream, b, aont, keys, digests);
  return hipGetLastError();
}

hipError_t launch_derive_keys(const BufferBatch& b, int aont, const uint8_t* digests, uint8_t* keys,
                              hipStream_t stream) {
  if (b.n == 0) return hipSuccess;
  hipLaunchKernelGGL(derive_keys_kernel, grid_for(b.n, 256), dim3(256), 0, stream, b, aont, digests, keys);
  return hipGetLastError();
}

}  // namespace ag
