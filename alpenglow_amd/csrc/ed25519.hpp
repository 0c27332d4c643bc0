// Ed25519 shred signatures on the device (ed25519.hip): parameter blocks and launchers.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace ag {

constexpr uint32_t kSliceCommitmentLen = 8 + 8 + 1 + 32;  // SLICE_COMMITMENT_LEN (shredder.rs:188)

// Device-side constant tables built once per context by launch_ed25519_init:
//   base  [64][8] multiples j*16^i*B (j = 1..8), affine "precomp" form
//         (y+x, y-x, 2d*x*y), 10 int32 limbs each -- fixed-base scalar multiples (sign,
//         public keys) with no doublings.  Row 0 is also the verify loop's B table.
constexpr uint32_t kEdBaseRows = 64, kEdBaseCols = 8, kEdPrecompInts = 30;
constexpr size_t kEdBaseTableBytes = size_t{kEdBaseRows} * kEdBaseCols * kEdPrecompInts * 4;
hipError_t launch_ed25519_init(int32_t* base_table, hipStream_t stream);

// Signature::verify_bytes (signature.rs:100-103; ed25519-zebra 4.2 ZIP-215 rules) for n
// (pk, msg, sig) triples.  pk: pks + t*pk_stride (stride 0 = one key for the batch);
// msg: msgs + t*msg_stride, msg_lens[t] bytes (msg_lens null: msg_len for every t);
// sig: sigs + t*64.  Optional list: verify only t = list[0 .. *list_count) (compacted
// work lists).  ok[t] = 1 / 0 (or status[t] via the shred path below).
struct EdVerifyParams {
  const uint8_t* pks;
  uint64_t pk_stride;
  const uint8_t* msgs;
  uint64_t msg_stride;
  const uint32_t* msg_lens;
  uint32_t msg_len;
  const uint8_t* sigs;
  uint64_t sig_stride;
  uint64_t n;
  const uint32_t* list;        // may be null
  const uint32_t* list_count;  // device counter when list != null
  uint8_t* ok;                 // ok[t]: 1 valid, 0 invalid
  // shred mode (ok == null): status[t] = valid ? on_valid[t] : kShredInvalidSignature
  uint8_t* status;
  const uint8_t* on_valid;
  const int32_t* base_table;
};
hipError_t launch_ed25519_verify(const EdVerifyParams& p, hipStream_t stream);

// SecretKey::to_pk (signature.rs:54-58) for n 32-byte seeds -> 32-byte keys.
hipError_t launch_ed25519_public_key(const uint8_t* seeds, uint8_t* pks, uint64_t n, const int32_t* base_table,
                                     hipStream_t stream);

// SecretKey::sign_bytes (signature.rs:69-72; RFC 8032 §5.1.6) for n messages.  seed / pk:
// seeds + t*seed_stride, pks + t*pk_stride (stride 0 = one key); msg t at msgs +
// t*msg_stride, msg_len bytes; signature -> sigs + t*64.
struct EdSignParams {
  const uint8_t* seeds;
  uint64_t seed_stride;
  const uint8_t* pks;
  uint64_t pk_stride;
  const uint8_t* msgs;
  uint64_t msg_stride;
  uint32_t msg_len;
  uint8_t* sigs;
  uint64_t n;
  const int32_t* base_table;
};
hipError_t launch_ed25519_sign(const EdSignParams& p, hipStream_t stream);

// ValidatedShred::try_new (validated_shred.rs:52-81), stage 1 (after the Merkle root of each
// shred has been derived into roots + 32*t): build the SliceCommitment (shredder.rs:206-215)
// into commitments + 49*t, compare with the cached commitment (if has_cached[t]), set
// status[t] = OK on a cache hit, and append t to the verify list otherwise (on_valid[t] =
// OK without a cache, EQUIVOCATION with one).
enum : uint8_t { kShredOk = 0, kShredInvalidSignature = 1, kShredEquivocation = 2 };
struct ShredCommitParams {
  const uint64_t* slots;
  const uint64_t* slice_indices;
  const uint8_t* is_last;
  const uint8_t* roots;            // 32 B per shred
  const uint8_t* cached;           // 49 B per shred (nullable)
  const uint8_t* has_cached;       // per shred (nullable: no cache)
  uint32_t cached_group;           // > 1: cached / has_cached entry t / cached_group (one per slice)
  const uint8_t* active;           // nullable: shreds with active[t] == 0 get kShredInvalidSignature
                                   // without a signature check (absent / malformed datagrams)
  uint64_t n;
  uint8_t* commitments;            // 49 B per shred (out)
  uint8_t* status;                 // out
  uint8_t* on_valid;               // out
  uint32_t* list;                  // out: shreds that need a signature check
  uint32_t* list_count;            // device counter (zeroed by the caller)
};
hipError_t launch_shred_commit(const ShredCommitParams& p, hipStream_t stream);

}  // namespace ag
