// All-or-nothing payload transforms of the AONT / PETS shredders (cipher.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace ag {

constexpr uint32_t kCipherKeyBytes = 16;  // cipher::KEY_BYTES (crypto/cipher.rs:16)

// n buffers: buffer b at base + b*stride, lens[b] bytes (device array).
struct BufferBatch {
  uint8_t* base;
  uint64_t stride;
  const uint32_t* lens;
  uint64_t n;
  uint32_t max_len;  // max over lens (grid sizing)
};

// cipher::apply_keystream (crypto/cipher.rs:25-30): AES-128-CTR (ctr::Ctr64LE, zero IV)
// keystream XORed into buffer b under keys + 16*b.  lens_delta is subtracted from every
// length (the decrypt side excludes the 16-byte key tail).
hipError_t launch_apply_keystream(const BufferBatch& b, const uint8_t* keys, uint32_t lens_delta, hipStream_t stream);
// hash::hash (crypto/hash.rs:64-67): SHA-256 of buffer b's first lens[b] - lens_delta bytes.
hipError_t launch_sha256(const BufferBatch& b, uint32_t lens_delta, uint8_t* digests, hipStream_t stream);
// Encrypt side tail at buffer + lens[b]: AONT key ^ digest[0..16) (shredder.rs:467-469),
// PETS the key (shredder.rs:416-417).
hipError_t launch_write_key_tail(const BufferBatch& b, int aont, const uint8_t* keys, const uint8_t* digests,
                                 hipStream_t stream);
// Decrypt side: keys[b] = tail ^ digest (AONT, shredder.rs:481-488) or the tail (PETS,
// shredder.rs:430); the tail is the last 16 of lens[b] bytes.
hipError_t launch_derive_keys(const BufferBatch& b, int aont, const uint8_t* digests, uint8_t* keys,
                              hipStream_t stream);

// Host AES-128 block encryption (same tables as the kernels; tests / known answers).
void aes128_encrypt_block(const uint8_t key[16], const uint8_t in[16], uint8_t out[16]);

}  // namespace ag
