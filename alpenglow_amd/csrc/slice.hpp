// Slice payload framing: Slice::payload_bytes and
// SlicePayload::try_from (/root/reference/src/types/slice.rs:73-84, :211-218) over batches
// of slices in the coder's codeword buffers.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace ag {

constexpr uint32_t kSliceMaxData = 32 * 1024 - 1;  // MAX_DATA_PER_SLICE (shredder.rs:54)
constexpr uint32_t kBlockIdBytes = 8 + 32;         // BlockId = (Slot u64, BlockHash [u8; 32])

// payload_bytes: codeword b's first bytes <- tag || [slot || hash] || u64 LE len || data
struct SliceFrameParams {
  const uint8_t* parent_flags;  // [n] 0 = None, 1 = Some
  const uint8_t* parent_ids;    // [n][40] slot (LE) then block hash
  const uint8_t* data;          // slice data bytes, data_stride apart
  uint64_t data_stride;
  const uint32_t* data_lens;    // [n]
  uint8_t* cw;                  // codewords, cw_stride apart
  uint64_t cw_stride;
  uint64_t n;
};
hipError_t launch_slice_frame(const SliceFrameParams& p, hipStream_t stream);

// try_from on the first payload_lens[b] bytes of codeword b (< 0: no payload)
struct SliceParseParams {
  const uint8_t* cw;
  uint64_t cw_stride;
  const int64_t* payload_lens;
  uint8_t* status;        // [n] AG_SLICE_* codes
  uint8_t* parent_flags;  // [n]
  uint8_t* parent_ids;    // [n][40]
  uint32_t* data_offsets;  // [n] data starts at codeword + offset
  uint32_t* data_lens;     // [n]
  uint64_t n;
};
hipError_t launch_slice_parse(const SliceParseParams& p, hipStream_t stream);

}  // namespace ag
