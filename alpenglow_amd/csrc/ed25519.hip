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
#include "unaligned.hpp"
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
  static_assert(kSliceCommitmentLen == 49, "slot | slice_index | is_last | root");
  // the 49 commitment bytes as 12 little-endian words + 1 byte: slot, slice index, then
  // is_last and the root shifted up one byte (v_alignbyte); rows of 49 bytes take unaligned
  // 16-byte accesses (byte loops cost ~130 memory instructions per shred)
  uint32_t w[12];
  const uint64_t slot = p.slots[t], si = p.slice_indices[t];
  w[0] = static_cast<uint32_t>(slot);
  w[1] = static_cast<uint32_t>(slot >> 32);
  w[2] = static_cast<uint32_t>(si);
  w[3] = static_cast<uint32_t>(si >> 32);
  uint32_t r[8];
  if ((reinterpret_cast<uintptr_t>(p.roots) & 15) == 0) {
    const uint4 a = *reinterpret_cast<const uint4*>(p.roots + 32 * t);
    const uint4 b = *reinterpret_cast<const uint4*>(p.roots + 32 * t + 16);
    r[0] = a.x; r[1] = a.y; r[2] = a.z; r[3] = a.w;
    r[4] = b.x; r[5] = b.y; r[6] = b.z; r[7] = b.w;
  } else {
    for (int i = 0; i < 8; ++i) {
      const uint8_t* q = p.roots + 32 * t + 4 * i;
      r[i] = q[0] | (uint32_t{q[1]} << 8) | (uint32_t{q[2]} << 16) | (uint32_t{q[3]} << 24);
    }
  }
  w[4] = (p.is_last[t] ? 1u : 0u) | (r[0] << 8);
  for (int k = 1; k < 8; ++k) w[4 + k] = __builtin_amdgcn_alignbyte(r[k], r[k - 1], 3);
  const uint8_t last = static_cast<uint8_t>(r[7] >> 24);
  uint8_t* out = p.commitments + kSliceCommitmentLen * t;
  for (int q = 0; q < 3; ++q)
    st16u(out + 16 * q, make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]));
  out[48] = last;
  const uint64_t ci = p.cached_group > 1 ? t / p.cached_group : t;
  const bool cached = p.cached && p.has_cached && p.has_cached[ci];
  if (cached) {
    const uint8_t* cc = p.cached + kSliceCommitmentLen * ci;
    uint32_t diff = static_cast<uint32_t>(cc[48] ^ last);
    for (int q = 0; q < 3; ++q) {
      const uint4 x = ld16u(cc + 16 * q);
      diff |= (x.x ^ w[4 * q]) | (x.y ^ w[4 * q + 1]) | (x.z ^ w[4 * q + 2]) | (x.w ^ w[4 * q + 3]);
    }
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
