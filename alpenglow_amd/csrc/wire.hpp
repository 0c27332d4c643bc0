// Shred wire format (wire.hip): column layout and launchers.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "merkle.hpp"  // grouped_row_offset

namespace ag {

// network.rs:45 / types/slice_index.rs:15 / shredder.rs:47
constexpr uint32_t kMtuBytes = 1500, kMaxSlicesPerBlock = 1024, kTotalShreds = 64;
// fixed part of a serialized Shred: u32 + u64 + u64 + u8 + u64 + u64 (data len)
constexpr uint32_t kShredHeadBytes = 4 + 8 + 8 + 1 + 8 + 8;
enum : uint8_t { kWireOk = 0, kWireMalformed = 1, kWireTooLarge = 2 };

// One column per Shred field (device arrays, n entries each).
struct ShredColumns {
  uint8_t* kind;         // ShredPayloadType: 0 Data, 1 Coding
  uint64_t* slot;
  uint64_t* slice_index;
  uint8_t* is_last;
  uint32_t* shred_index;
  uint8_t* data;         // data + t*data_stride
  uint64_t data_stride;  // capacity of one data row
  uint32_t* data_len;
  uint8_t* sig;          // 64 B each
  uint8_t* proof;        // proof + t*proof_stride, height digests
  uint64_t proof_stride;
  uint32_t* height;
  uint32_t hdr_group;    // serialize only: > 1 reads slot / slice_index / is_last / sig of row
                         // t / hdr_group (one header per slice); 0 or 1: per shred
  uint64_t group_stride;  // data row t at data + grouped_row_offset(t, data_stride, group_stride,
  uint32_t skip_row;      // skip_row) (group_stride 0: t * data_stride)
  uint32_t skip_sig;      // serialize only: leave the 64 signature bytes for launch_shred_sig_patch
};
__host__ __device__ inline uint64_t data_row_offset(const ShredColumns& c, uint64_t t) {
  return grouped_row_offset(t, c.data_stride, c.group_stride, c.skip_row);
}

// network::deserialize::<Shred> for n packets (packet t at packets + t*packet_stride,
// packet_lens[t] bytes) into the columns; status[t] = kWireOk / kWireMalformed (wincode
// rejects it) / kWireTooLarge (valid but wider than the caller's data / proof rows).
hipError_t launch_shred_deserialize(const uint8_t* packets, uint64_t packet_stride, const uint32_t* packet_lens,
                                    uint64_t n, const ShredColumns& c, uint8_t* status, hipStream_t stream);
// wincode::serialize(&Shred) for n shreds; packet_lens[t] gets the byte count (0, packet
// untouched, when the shred does not fit packet_stride or its columns' rows).
hipError_t launch_shred_serialize(const ShredColumns& c, uint64_t n, uint8_t* packets, uint64_t packet_stride,
                                  uint32_t* packet_lens, hipStream_t stream);
// The signatures of datagrams serialized with skip_sig: packet t (packet_lens[t] != 0) gets the
// 64 bytes of c.sig row t / hdr_group (or t) at its signature offset (37 + data_len[t]); one
// thread per datagram.  Lets the signing overlap the bulk of the serialization.
hipError_t launch_shred_sig_patch(const ShredColumns& c, uint64_t n, uint8_t* packets, uint64_t packet_stride,
                                  const uint32_t* packet_lens, hipStream_t stream);

}  // namespace ag
