// Host-only stand-in for <hip/hip_runtime.h> so tools/lane_host_check.cpp can
// compile this project's device rules (open_spiel_coup_amd/csrc/coup_lane.h)
// with g++ for debugging.  Test tooling only; never used by the product build.
#pragma once
#include <stdint.h>
#define COUP_HOST_STANDIN 1  // device-only helpers (cross-lane builtins) are left out
#define __device__
#define __host__
#define __forceinline__ inline
struct uint4 { uint32_t x, y, z, w; };
inline uint4 make_uint4(uint32_t x, uint32_t y, uint32_t z, uint32_t w) { return uint4{x, y, z, w}; }
inline uint32_t __umulhi(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }
inline int __popc(uint32_t v) { return __builtin_popcount(v); }
