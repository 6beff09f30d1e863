// Host build of the lane rules (coup_host.cpp, compiled with g++): the few
// HIP names coup_lane.h / coup_tensor.h use, as plain host C++.  The device
// build includes the real <hip/hip_runtime.h>; this directory is on the
// include path of coup_host.cpp only.
#pragma once
#include <stdint.h>

#define COUP_HOST_STANDIN 1  // device-only helpers (cross-lane builtins) are left out of the host build

#define __device__
#define __host__
#define __forceinline__ inline __attribute__((always_inline))
#define __noinline__ __attribute__((noinline))

struct uint2 { uint32_t x, y; };
struct uint4 { uint32_t x, y, z, w; };
struct float4 { float x, y, z, w; };
inline uint2 make_uint2(uint32_t x, uint32_t y) { return uint2{x, y}; }
inline uint4 make_uint4(uint32_t x, uint32_t y, uint32_t z, uint32_t w) { return uint4{x, y, z, w}; }
inline float4 make_float4(float x, float y, float z, float w) { return float4{x, y, z, w}; }
inline uint32_t __umulhi(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }
inline int __popc(uint32_t v) { return __builtin_popcount(v); }
