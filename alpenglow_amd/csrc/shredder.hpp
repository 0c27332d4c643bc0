// Composed Shredder pipeline (shredder.hip): the glue kernels between the batched stages
// (slice framing, ReedSolomonCoder, Merkle trees, signatures, wire format) that
// ag_shredder_shred_batch / ag_shredder_deshred_batch chain on the device.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "wire.hpp"

namespace ag {

constexpr uint32_t kPipeShreds = 64;   // TOTAL_SHREDS (shredder.rs:47)
constexpr uint32_t kPipeData = 32;     // DATA_SHREDS (shredder.rs:43)
constexpr uint32_t kPipeHeight = 6;    // Merkle path length of a 64-leaf slice tree
constexpr uint32_t kPipeNone = 0xFFu;  // no shred picked

// Per-shred columns of the shred side / fill side: kind (data shreds first), shred_index,
// data_len = S and height; rows whose skip bit is set get data_len = ~0 (the serializer then
// leaves their packet alone).  skip: per slice, a 64-bit mask of rows to skip (nullable).
struct PipeExpandParams {
  uint64_t nslices;
  uint32_t shred_bytes;
  uint32_t num_data;      // data output shreds (kind Data below it): 32 Regular / AONT, 31 PETS, 0 CodingOnly
  const uint64_t* skip;   // [nslices] (nullable)
  const uint8_t* slice_ok;  // [nslices] (nullable): rows of slices with 0 are skipped too
  uint8_t* kind;          // [nslices * 64]
  uint32_t* shred_index;
  uint32_t* data_len;
  uint32_t* height;
};
hipError_t launch_pipe_expand(const PipeExpandParams& p, hipStream_t stream);

// Deshred side, per slice: the first shred (by index) whose datagram parsed and whose fields
// fit the slice layout (shred_index = its slot, kind matches, data_len = S, height = 6); its
// payload row, proof and header are gathered into compact per-slice arrays so that one
// signature check per slice establishes the slice's commitment (the blockstore's cached
// commitment, validated_shred.rs:57-64).
struct PipePickParams {
  uint64_t nslices;
  uint32_t shred_bytes;
  uint32_t num_data;            // data output shreds: slot j < num_data holds a Data shred
  const uint8_t* wire_status;   // [nslices * 64]
  ShredColumns cols;            // deserialized columns (per shred)
  uint8_t* pick;                // [nslices]: picked shred index or kPipeNone
  uint8_t* g_data;              // [nslices][S]
  uint8_t* g_proof;             // [nslices][6 * 32]
  uint64_t* g_slot;
  uint64_t* g_slice_index;
  uint8_t* g_is_last;
  uint32_t* g_shred_index;
  uint8_t* g_sig;               // [nslices][64]
  uint8_t* has_cached;          // [nslices]: filled by launch_pipe_cache_flags
  uint8_t* plausible;           // [nslices * 64] out: shred t parsed and fits its slot
};
hipError_t launch_pipe_pick(const PipePickParams& p, hipStream_t stream);
// has_cached[s] = the picked shred of slice s passed its signature check.
hipError_t launch_pipe_cache_flags(const uint8_t* pick, const uint8_t* pick_status, uint64_t nslices,
                                   uint8_t* has_cached, hipStream_t stream);

// Per slice after the full validation: the shreds kept (parsed, layout-consistent,
// ValidatedShred::try_new OK, same commitment as the first kept one), and that shred's root,
// header and signature (the ReconstructedSlice's header and the slice_sig that
// fill_missing_shreds copies, shredder.rs:296-299).
struct PipeCheckParams {
  uint64_t nslices;
  uint32_t shred_bytes;
  uint32_t num_data;           // data output shreds (PipePickParams)
  const uint8_t* wire_status;  // [nslices * 64]
  const uint8_t* val_status;   // [nslices * 64]
  const uint8_t* roots;        // [nslices * 64][32]
  ShredColumns cols;
  uint64_t* present;           // [nslices] out
  uint8_t* root;               // [nslices][32] out
  uint64_t* slot;              // [nslices] out
  uint64_t* slice_index;
  uint8_t* is_last;
  uint8_t* sig;                // [nslices][64] out
};
hipError_t launch_pipe_check(const PipeCheckParams& p, hipStream_t stream);

// same[s] = (a + 32 s) and (b + 32 s) hold the same 32 bytes.
hipError_t launch_pipe_root_cmp(const uint8_t* a, const uint8_t* b, uint64_t nslices, uint8_t* same,
                                hipStream_t stream);
// packet_lens[t] = fresh[t] for the rows the fill step serialized (absent rows of slices
// with slice_ok), unchanged elsewhere.
hipError_t launch_pipe_merge_lens(const uint32_t* fresh, const uint64_t* present, const uint8_t* slice_ok,
                                  uint64_t nslices, uint32_t* packet_lens, hipStream_t stream);

// The ReedSolomonCoder::deshred patterns of the kept shreds on the device (32:32 HighRate,
// window W = 64: recovery j at position j, original i at 32 + i), for the per-lane decode_x
// kernel (the patterns rs_api.cpp's decode_device builds on the host for ANY_K):
//   xm[s] = erased positions (locator), xm[n + 2 s] = survivors loaded (the present originals,
//   then recovery shards in index order up to 32), xm[n + 2 s + 1] = originals restored.
// Slices with fewer than 32 kept shreds, or nothing to restore, get empty masks (no loads, no
// stores); few[s] = 1 for the former (NotEnoughShreds, reed_solomon.rs:144).
// fuse (the packed window decoder, decode_pk<-1>): a slice with exactly 32 kept shreds also
// restores its absent coding shreds in the decode (xm[n + 2 s + 1] = every erased position)
// and gets few[s] = 2, so the re-encode's store mask skips it.
hipError_t launch_pipe_patterns(const uint64_t* present, uint64_t nslices, uint64_t* xm, uint8_t* few, bool fuse,
                                hipStream_t stream);
// The same for CodingOnly slices (LowRate 32:64) in the W = 128 window of the two-pass decoder:
// present[2 s] = data bits | coding 0..31 << 32, present[2 s + 1] = coding 32..63; xm =
// decode_rows128's m6 [n][6], then the pass-1 and pass-2 (survivors, restored) pairs [n][2]
// each (rs_api.cpp's class-8 layout).
hipError_t launch_pipe_patterns128(const uint64_t* present, uint64_t nslices, uint64_t* xm, uint8_t* few,
                                   hipStream_t stream);
// mask[s] = ~0 (store every coding shard of the re-encode) when the slice decoded and its
// padding stripped (few[s] == 0 and strip[s] >= 0), else 0 (the coding shreds stay as they
// are, like the reference's early returns; few[s] == 2: the decode restored them).
// present: the kept-shred words (wps per slice, launch_pipe_patterns / 128): a slice with
// exactly 32 kept shreds re-encodes only its absent coding shreds (bit j: coding shred j).
// strip[s] then becomes the slice's result: its payload length, err_few (fewer than 32 kept
// shreds) or err_padding (the strip failed).
hipError_t launch_pipe_store_masks(const uint8_t* few, int64_t* strip, const uint64_t* present, uint32_t wps,
                                   uint64_t nslices, uint64_t* mask, int64_t err_few, int64_t err_padding,
                                   hipStream_t stream);

// flags[64 s + j] = 1: leaf j of slice s is hashed again by the deshred's Merkle rebuild (shred
// not kept, or a coding shred the coder may have rewritten: surplus slices, or all with
// reencode_all); 0: its digest from the proof check stands.
hipError_t launch_pipe_leaf_flags(const uint64_t* present, uint64_t nslices, bool reencode_all, uint8_t* flags,
                                  hipStream_t stream);

}  // namespace ag
