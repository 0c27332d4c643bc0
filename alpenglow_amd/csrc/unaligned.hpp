// Unaligned 16 / 8 / 4-byte global accesses (device code).
//
// gfx950 under ROCm runs global memory in unaligned mode: a global_load/store_dwordx4 at any
// byte address is split by the hardware.  Dereferencing a `uint4*` at such an address would
// still tell the compiler the address is 16-byte aligned, which is undefined behaviour and
// unsafe if the backend ever turned a provably uniform access into a scalar-memory one (those
// drop the low address bits).  These helpers access through types of alignment 1, which assert no
// alignment, and the backend still emits the one vector instruction.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace ag {

// (clang vector types of alignment 1: one vector access, no alignment asserted; HIP's uint4
// class cannot carry a reduced-alignment typedef)
typedef uint32_t u32x4_u __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t u32x2_u __attribute__((ext_vector_type(2), aligned(1)));
typedef uint32_t u32_u __attribute__((aligned(1)));

__device__ __forceinline__ uint4 ld16u(const void* p) {
  const u32x4_u v = *static_cast<const u32x4_u*>(p);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st16u(void* p, uint4 v) { *static_cast<u32x4_u*>(p) = u32x4_u{v.x, v.y, v.z, v.w}; }
__device__ __forceinline__ void st8u(void* p, uint2 v) { *static_cast<u32x2_u*>(p) = u32x2_u{v.x, v.y}; }
__device__ __forceinline__ void st4u(void* p, uint32_t v) { *static_cast<u32_u*>(p) = v; }
typedef uint16_t u16_u __attribute__((aligned(1)));
__device__ __forceinline__ uint2 ld8u(const void* p) {
  const u32x2_u v = *static_cast<const u32x2_u*>(p);
  return make_uint2(v.x, v.y);
}
__device__ __forceinline__ uint32_t ld4u(const void* p) { return *static_cast<const u32_u*>(p); }
__device__ __forceinline__ uint32_t ld2u(const void* p) { return *static_cast<const u16_u*>(p); }
__device__ __forceinline__ void st2u(void* p, uint32_t v) { *static_cast<u16_u*>(p) = static_cast<uint16_t>(v); }

}  // namespace ag
