// Ed25519 shred signatures on the device.
//
// What it replaces
//   SecretKey::to_pk / sign_bytes, Signature::verify_bytes (crypto/signature.rs:54-104) --
//   ed25519-zebra 4.2.0: RFC 8032 keygen and signing, ZIP-215 verification;
//   ValidatedShred::try_new (shredder/validated_shred.rs:52-81): the per-shred check on the
//   receive path (every shred that arrives through the disseminator or repair);
//   the shred side's signature over SliceCommitment (shredder.rs:206-215, :540).
// The arithmetic (field, group, SHA-512, scalars) is ed25519_core.hpp.
//
// Kernels (one thread per signature; the work is long integer-multiply chains, VALU-bound)
//   ed_init_kernel        64 threads: the fixed-base table rows j * 16^i * B (once per context)
//   ed_verify_kernel      decompress A and R, k = SHA-512(R || A || M) mod l, joint signed
//                         radix-16 [k](-A) + [s]B (the -A table in per-lane scratch, the B
//                         row in global memory), [8](R - R') == identity
//   ed_pubkey_kernel      [a]B with the fixed-base table (64 mixed additions)
//   ed_sign_kernel        RFC 8032 signing, R = [r]B with the fixed-base table
//   shred_commit_kernel   SliceCommitment per shred, cached-commitment compare, compacted
//                         list of the shreds that need a signature check
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "ed25519.hpp"
#include "ed25519_core.hpp"

namespace ag {

namespace {

__global__ __launch_bounds__(64) void ed_init_kernel(int32_t* table) {
  const int row = threadIdx.x;
  if (row < static_cast<int>(kEdBaseRows)) ed::base_table_row(row, table);
}

// WPE: waves per SIMD the register budget is sized for (1: 313 VGPRs, no spills; 2: 256
// VGPRs, 48 spilled; 3: 168, 220 spilled); 2 is launched (kVerifyWpe).
template <int WPE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void ed_verify_kernel(
    const EdVerifyParams p) {
  uint64_t t = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (p.list) {
    if (t >= *p.list_count) return;
    t = p.list[t];
  } else if (t >= p.n) {
    return;
  }
  const uint8_t* pk = p.pks + t * p.pk_stride;
  const uint8_t* sig = p.sigs + t * p.sig_stride;
  const uint8_t* msg = p.msgs + t * p.msg_stride;
  const uint32_t mlen = p.msg_lens ? p.msg_lens[t] : p.msg_len;
  ed::Cached tab[9];
  const bool ok = ed::verify(pk, sig, mlen, [&](uint32_t i) -> uint32_t { return msg[i]; }, p.base_table, tab);
  if (p.ok) p.ok[t] = ok ? 1 : 0;
  else p.status[t] = ok ? p.on_valid[t] : kShredInvalidSignature;
}

__global__ __launch_bounds__(64) void ed_pubkey_kernel(const uint8_t* seeds, uint8_t* pks, uint64_t n,
                                                       const int32_t* table) {
  const uint64_t t = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= n) return;
  ed::public_key(seeds + 32 * t, pks + 32 * t, table);
}

__global__ __launch_bounds__(64) void ed_sign_kernel(const EdSignParams p) {
  const uint64_t t = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= p.n) return;
  const uint8_t* msg = p.msgs + t * p.msg_stride;
  ed::sign(p.seeds + t * p.seed_stride, p.pks + t * p.pk_stride, p.msg_len,
           [&](uint32_t i) -> uint32_t { return msg[i]; }, p.sigs + 64 * t, p.base_table);
}

__global__ __launch_bounds__(256) void shred_commit_kernel(const ShredCommitParams p) {
  const uint64_t t = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= p.n) return;
  if (p.active && !p.active[t]) {
    p.status[t] = kShredInvalidSignature;
    return;
  }
  uint8_t c[kSliceCommitmentLen];
  const uint64_t slot = p.slots[t], si = p.slice_indices[t];
  for (int i = 0; i < 8; ++i) {
    c[i] = static_cast<uint8_t>(slot >> (8 * i));
    c[8 + i] = static_cast<uint8_t>(si >> (8 * i));
  }
  c[16] = p.is_last[t] ? 1 : 0;
  for (int i = 0; i < 32; ++i) c[17 + i] = p.roots[32 * t + i];
  uint8_t* out = p.commitments + kSliceCommitmentLen * t;
  for (uint32_t i = 0; i < kSliceCommitmentLen; ++i) out[i] = c[i];
  const uint64_t ci = p.cached_group > 1 ? t / p.cached_group : t;
  const bool cached = p.cached && p.has_cached && p.has_cached[ci];
  if (cached) {
    const uint8_t* cc = p.cached + kSliceCommitmentLen * ci;
    uint32_t diff = 0;
    for (uint32_t i = 0; i < kSliceCommitmentLen; ++i) diff |= c[i] ^ cc[i];
    if (diff == 0) {  // validated_shred.rs:62-64: same commitment, no signature check
      p.status[t] = kShredOk;
      return;
    }
  }
  // validated_shred.rs:65-77: a valid signature is OK without a cache, Equivocation with one
  p.on_valid[t] = cached ? kShredEquivocation : kShredOk;
  p.status[t] = kShredInvalidSignature;
  const uint32_t slot_idx = atomicAdd(p.list_count, 1u);
  p.list[slot_idx] = static_cast<uint32_t>(t);
}

constexpr int kVerifyWpe = 2;  // measured: 1 -> 41.9, 2 -> 46.2, 3 -> 45.8 M verifications/s

dim3 grid_for(uint64_t n, unsigned block) { return dim3(static_cast<unsigned>((n + block - 1) / block)); }

}  // namespace

hipError_t launch_ed25519_init(int32_t* base_table, hipStream_t stream) {
  hipLaunchKernelGGL(ed_init_kernel, dim3(1), dim3(64), 0, stream, base_table);
  return hipGetLastError();
}

hipError_t launch_ed25519_verify(const EdVerifyParams& p, hipStream_t stream) {
  if (p.n == 0) return hipSuccess;
  if ((p.n + 63) / 64 > 0x7FFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ed_verify_kernel<kVerifyWpe>, grid_for(p.n, 64), dim3(64), 0, stream, p);
  return hipGetLastError();
}

hipError_t launch_ed25519_public_key(const uint8_t* seeds, uint8_t* pks, uint64_t n, const int32_t* base_table,
                                     hipStream_t stream) {
  if (n == 0) return hipSuccess;
  if ((n + 63) / 64 > 0x7FFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ed_pubkey_kernel, grid_for(n, 64), dim3(64), 0, stream, seeds, pks, n, base_table);
  return hipGetLastError();
}

hipError_t launch_ed25519_sign(const EdSignParams& p, hipStream_t stream) {
  if (p.n == 0) return hipSuccess;
  if ((p.n + 63) / 64 > 0x7FFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ed_sign_kernel, grid_for(p.n, 64), dim3(64), 0, stream, p);
  return hipGetLastError();
}

hipError_t launch_shred_commit(const ShredCommitParams& p, hipStream_t stream) {
  if (p.n == 0) return hipSuccess;
  if ((p.n + 255) / 256 > 0x7FFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(shred_commit_kernel, grid_for(p.n, 256), dim3(256), 0, stream, p);
  return hipGetLastError();
}

}  // namespace ag
