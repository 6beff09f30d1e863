// coup_tensor.h -- the ObservationTensor / InformationStateTensor element
// decoders of a packed lane, shared by the device kernels (coup_kernels.hip:
// the per-lane, wave-cooperative and k_info_elems writers) and the host
// build of the per-game State ops (coup_host.cpp), so both write the same
// floats from the same code.  Reference: CoupObserver::WriteTensor
// (coup.cc:248-287, 230-245) with kDefaultObsType / kInfoStateObsType
// (observer.h:287-297) through ContiguousAllocator (observer.h:173-176).
#pragma once

#include "coup_lane.h"
#include "coup_mi355x.h"

namespace coup {

constexpr int kObsSize = COUP_OBS_SIZE;

// CoupObserver::WriteTensor with kDefaultObsType (coup.cc:248-287,
// observer.h:287-290) through ContiguousAllocator (zero-filled, blocks laid
// out back to back, observer.h:173-176):
//   [0:2] observer one-hot          [2:22] P1 cards [4][5]   [22:42] P2 cards
//   [42:44] cur_move_player one-hot (zeros when terminal)
//   [44:60] cards_state [2][4][2]   [60:62] coins           [62:98] last_action [2][18]
// A card's type is visible for the owner's face-down cards and for every
// face-up card.  `f` is a compile-time constant after unrolling, so every
// element folds to one or two compares on a nibble.
template <int P>
__device__ __forceinline__ float obs_at(const Lane& L, bool term, const int f) {
  if (f < 2) return f == P ? 1.0f : 0.0f;
  if (f < 42) {
    const int q = (f - 2) / 20, i = ((f - 2) % 20) / 5, t = (f - 2) % 5;
    const uint32_t n = nib(q ? L.h1 : L.h0, (uint32_t)i);
    const bool v = (n == (uint32_t)(2 * t + 1)) || (q == P && n == (uint32_t)(2 * t));
    return v ? 1.0f : 0.0f;
  }
  if (f < 44) return (!term && L.M == (uint32_t)(f - 42)) ? 1.0f : 0.0f;
  if (f < 60) {
    const int q = (f - 44) / 8, i = ((f - 44) % 8) / 2, s = (f - 44) % 2;
    const uint32_t n = nib(q ? L.h1 : L.h0, (uint32_t)i);
    return (n != 0xFu && (n & 1u) == (uint32_t)s) ? 1.0f : 0.0f;
  }
  if (f < 62) return (float)(f == 60 ? L.c0 : L.c1);
  const int q = (f - 62) / 18, a = (f - 62) % 18;
  return ((q ? L.l1 : L.l0) == (uint32_t)a) ? 1.0f : 0.0f;
}

__device__ __forceinline__ float obs_pair_at(const Lane& L, bool term, const int g) {
  return g < kObsSize ? obs_at<0>(L, term, g) : obs_at<1>(L, term, g - kObsSize);
}

// One observer's 98-bit row (bit f = element f of ObservationTensor(P)).
template <int P>
__device__ __forceinline__ void obs_row_bits(const Lane& L, bool term, uint64_t& lo, uint64_t& hi) {
  lo = 1ull << P;  // observer one-hot
#pragma unroll
  for (uint32_t k = 0; k < 8; ++k) {
    const uint32_t q = k >> 2, i = k & 3u;
    const uint32_t n = nib(q ? L.h1 : L.h0, i);
    const bool exists = n != 0xFu;
    const bool visible = exists && (q == (uint32_t)P || (n & 1u));
    lo |= (uint64_t)visible << (2u + 20u * q + 5u * i + (n >> 1));
    lo |= (uint64_t)exists << (44u + 8u * q + 2u * i + (n & 1u));
  }
  lo |= (uint64_t)(!term) << (42u + L.M);
  hi = 0;
#pragma unroll
  for (uint32_t q = 0; q < 2; ++q) {
    const uint32_t a = q ? L.l1 : L.l0;
    const uint32_t p = 62u + 18u * q + a;
    const bool has = a != kNoAction;
    lo |= (uint64_t)(has && p < 64u) << (p & 63u);
    hi |= (uint64_t)(has && p >= 64u) << ((p - 64u) & 63u);
  }
}

// obs_row_bits with the observer as a run-time value (the same bits): the
// split observation writer decodes a lane's two rows on two threads.
__device__ __forceinline__ void obs_row_bits_rt(const Lane& L, bool term, uint32_t P, uint64_t& lo, uint64_t& hi) {
  lo = 1ull << P;  // observer one-hot
#pragma unroll
  for (uint32_t k = 0; k < 8; ++k) {
    const uint32_t q = k >> 2, i = k & 3u;
    const uint32_t n = nib(q ? L.h1 : L.h0, i);
    const bool exists = n != 0xFu;
    const bool visible = exists && (q == P || (n & 1u));
    lo |= (uint64_t)visible << (2u + 20u * q + 5u * i + (n >> 1));
    lo |= (uint64_t)exists << (44u + 8u * q + 2u * i + (n & 1u));
  }
  lo |= (uint64_t)(!term) << (42u + L.M);
  hi = 0;
#pragma unroll
  for (uint32_t q = 0; q < 2; ++q) {
    const uint32_t a = q ? L.l1 : L.l0;
    const uint32_t p = 62u + 18u * q + a;
    const bool has = a != kNoAction;
    lo |= (uint64_t)(has && p < 64u) << (p & 63u);
    hi |= (uint64_t)(has && p >= 64u) << ((p - 64u) & 63u);
  }
}

// InformationStateTensor layout (see coup_kernels.hip's write_info_wave):
constexpr int kInfoSize = COUP_INFO_STATE_SIZE;  // 2492
constexpr int kInfoHalfF4 = kInfoSize / 4;       // 623 float4 per player
constexpr int kInfoF4 = 2 * kInfoHalfF4;         // 1246 float4 per lane
constexpr int kPreWords = 6;
constexpr int kHist = (int)kHistoryBytes;

__device__ __forceinline__ void info_prefix_to_lds(const Lane& L, uint32_t* __restrict__ pre) {
  const bool term = is_terminal(L);
  uint64_t a_lo, a_hi, b_lo, b_hi;
  obs_row_bits<0>(L, term, a_lo, a_hi);
  obs_row_bits<1>(L, term, b_lo, b_hi);
  const uint64_t m62 = (1ull << 62) - 1ull;  // drop the observation's last_action bits
  // 32-bit stores only: the uint2 form (a <2 x i32> value) gave wrong prefix
  // bits in k_info_sweep
  pre[0] = (uint32_t)a_lo;
  pre[1] = (uint32_t)((a_lo & m62) >> 32);
  pre[2] = (uint32_t)b_lo;
  pre[3] = (uint32_t)((b_lo & m62) >> 32);
  pre[4] = L.c0 | (L.c1 << 8) | (L.move << 16);
  pre[5] = 0;
}

// One InformationStateTensor float4 (element c of [2][2492] / 4) of the lane
// whose record is L and whose history bytes are h; k_info_elems' decode.
__device__ __forceinline__ float4 info_f4(const uint32_t* pre, const uint8_t* h, uint32_t c) {
  const uint32_t p = c >= (uint32_t)kInfoHalfF4 ? 1u : 0u;
  const int f0 = 4 * (int)(c - p * (uint32_t)kInfoHalfF4);
  const uint32_t meta = pre[4];
  const uint32_t len = meta >> 16;
  if (f0 >= 62 + 18 * (int)len) return make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  const uint64_t prefix = (uint64_t)pre[2 * p] | ((uint64_t)pre[2 * p + 1] << 32);
  const int t0 = f0 - 62;
  const uint32_t r0 = t0 < 0 ? 0u : (uint32_t)t0 / 18u;
  const int col0 = t0 - 18 * (int)r0;
  uint32_t va[2];
#pragma unroll
  for (uint32_t k = 0; k < 2; ++k) {
    const uint32_t r = r0 + k;
    const uint32_t e = h[r < (uint32_t)kHist ? r : 0u];
    const bool seen = (e & 0x20u) == 0u || ((e >> 6) & 1u) == p;  // deals: observer's only
    va[k] = (r < len && seen) ? (e & 0x1Fu) : 31u;
  }
  float v[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int f = f0 + e;
    const int col = col0 + e;
    const uint32_t row_act = col >= 18 ? va[1] : va[0];
    const float hv = (row_act == (uint32_t)(col >= 18 ? col - 18 : col)) ? 1.0f : 0.0f;
    const float pb = (float)((uint32_t)(prefix >> (f & 63)) & 1u);
    const float coin = (float)(f == 60 ? (meta & 0xFFu) : ((meta >> 8) & 0xFFu));
    v[e] = f < 60 ? pb : (f < 62 ? coin : hv);
  }
  return make_float4(v[0], v[1], v[2], v[3]);
}

}  // namespace coup
