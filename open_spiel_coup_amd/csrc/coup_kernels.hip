// coup_kernels.hip -- gfx950 kernels of the batched Coup environment and the
// C ABI declared in include/coup_mi355x.h.
//
// One thread = one lane (game).  A lane's 16-byte record is loaded with one
// dwordx4 per thread (1 KiB contiguous per wave instruction), the step runs
// in registers (coup_lane.h), and the record is stored back the same way.
// Integer/branching work only: no MFMA, no LDS.  The HBM-heavy output is
// the optional ObservationTensor write-out (784 B per lane and step).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#ifdef COUP_COUNT_PHILOX
// Measurement builds: [0] wave-level Philox evaluations, [1] lanes active in
// them (coup_debug_philox_counts).
__device__ unsigned long long g_philox_counts[2];
__device__ __forceinline__ void count_philox_eval() {
  const uint64_t ex = __builtin_amdgcn_read_exec();
  if ((threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(ex)) {
    atomicAdd(&g_philox_counts[0], 1ull);
    atomicAdd(&g_philox_counts[1], (unsigned long long)__builtin_popcountll(ex));
  }
}
#define COUP_PHILOX_HOOK() count_philox_eval()
#endif
#ifdef COUP_TRAJ_PHASES
__device__ unsigned long long g_traj_phases[7];  // coup_traj_phases.h
#endif
#include "coup_traj_phases.h"
#include "coup_lane.h"
#include "coup_launch_log.h"
#include "coup_mi355x.h"
#include "coup_np.h"
#include "coup_regroup.h"
#include "coup_tensor.h"

namespace coup {

constexpr int kThreads = 256;
// the 2-player sorted kernels' bin prefix (coup_regroup.h): per wave in DPP
// (bins_below_dpp; the bare rules trajectory at 2^20 lanes 18.52-18.57 ->
// 16.59-17.24 us per step, c3 -0.7..-1.0 us per step, alternating builds,
// call r06e) or, in -DCOUP_BINS_LANE A/B builds, per lane (bins_below)
#ifdef COUP_BINS_LANE
#define COUP_BINS_BELOW(bin, key) bins_below<7>(bin, key)
#else
#define COUP_BINS_BELOW(bin, key) bins_below_dpp(bin, key)
#endif
// lanes per regrouping block of the 2-player sorted step / rollout
// (profiles/r02/ab/sort_block_size_2p.log)
constexpr int kStepSortLanes = 512;
constexpr int kRolloutSortLanes = 1024;

// The per-thread launch log (coup_launch_log.h): distinct (format, values)
// entries in first-launch order.
namespace {
struct LaunchNote {
  const char* fmt;
  int v[5];
};
constexpr int kLaunchNotes = 32;
thread_local LaunchNote g_launch_notes[kLaunchNotes];
thread_local int g_launch_count = 0;
}  // namespace

void note_launch(const char* fmt, int v0, int v1, int v2, int v3, int v4) {
  const int v[5] = {v0, v1, v2, v3, v4};
  for (int i = 0; i < g_launch_count; ++i)
    if (g_launch_notes[i].fmt == fmt && std::memcmp(g_launch_notes[i].v, v, sizeof(v)) == 0) return;
  if (g_launch_count == kLaunchNotes) return;
  LaunchNote& e = g_launch_notes[g_launch_count++];
  e.fmt = fmt;
  std::memcpy(e.v, v, sizeof(v));
}

std::string launch_log_text() {
  std::string out;
  for (int i = 0; i < g_launch_count; ++i) {
    if (i) out += " + ";
    const LaunchNote& e = g_launch_notes[i];
    int k = 0;
    for (const char* c = e.fmt; *c; ++c) {
      if (c[0] == '{' && c[1] == '}') {
        out += std::to_string(k < 5 ? e.v[k] : 0);
        ++k;
        ++c;
      } else if (c[0] == '{' && c[1] == 'b' && c[2] == '}') {
        out += (k < 5 && e.v[k]) ? "true" : "false";
        ++k;
        c += 2;
      } else {
        out += *c;
      }
    }
  }
  return out;
}

void clear_launch_log() { g_launch_count = 0; }

// The RNG key of lane i (global env id).  A measurement
// build with -DCOUP_ABLATE_SAME_STREAM gives every lane the same stream, so
// all lanes play the same game and the waves do not diverge (wrong results;
// it times the step without divergence).
__device__ __forceinline__ uint32_t lane_stream_id(uint32_t env_id_base, int64_t i) {
#ifdef COUP_ABLATE_SAME_STREAM
  (void)i;
  return env_id_base;
#else
  return env_id_base + (uint32_t)i;
#endif
}

// ------------------------------------------------------- observation tensor


// Both players' 98-float rows of one lane: 784 contiguous bytes = 49 float4.
__device__ __forceinline__ void write_obs_pair(float* __restrict__ dst, const Lane& L) {
  const bool term = is_terminal(L);
  typedef float v4f __attribute__((ext_vector_type(4)));
  v4f* d4 = reinterpret_cast<v4f*>(dst);
#pragma unroll
  for (int j = 0; j < 2 * kObsSize / 4; ++j) {
    v4f v;
    v.x = obs_pair_at(L, term, 4 * j + 0);
    v.y = obs_pair_at(L, term, 4 * j + 1);
    v.z = obs_pair_at(L, term, 4 * j + 2);
    v.w = obs_pair_at(L, term, 4 * j + 3);
    __builtin_nontemporal_store(v, d4 + j);
  }
}

// ---- wave-cooperative write-out ------------------------------------------
//
// A wave's 64 lanes own 64 consecutive rows of 196 floats = 3136 float4
// (50,176 contiguous bytes).  Iteration j of 49 stores float4 number
// 64*j + lane of that chunk, so every store instruction writes 1 KiB
// contiguous.  The float4 belongs to lane o = x / 49 (x = 64*j + lane), at
// float offset 4*(x % 49) of o's row; its four values are decoded from o's
// observation KEY (3 u32 fetched with ds_bpermute) through a per-offset
// DESCRIPTOR table held in LDS.
//
// Key words (per lane; only K0 depends on the observer P):
//   K0_P: [0] P, [1+3k .. 3+3k] visible type of card slot k = 4*owner+slot
//         (7 = hidden or empty), [25:26] mover (3 when terminal),
//         [27+2k .. 28+2k] face of slot k < 2 (0 down, 1 up, 3 empty)
//   K1:   [2(k-2) ..] face of slots k = 2..7, [12:15] P1 coins,
//         [16:19] P2 coins, [20:24] P1 last action, [25:29] P2 last action
// Descriptor of float g in [0,196): [4:0] bit offset, [12:8] width,
//   [20:16] value compared against, [24] raw (coins: the field itself),
//   [25] field in K1, [26] observer P = g >= 98.
constexpr int kRowF4 = 2 * kObsSize / 4;  // 49 float4 per lane row

__device__ __forceinline__ uint32_t obs_desc(int g) {
  const uint32_t P = g >= kObsSize;
  const int f = g - (int)P * kObsSize;
  uint32_t off, width, cmp = 0, raw = 0, k1 = 0;
  if (f < 2) {
    off = 0, width = 1, cmp = f;
  } else if (f < 42) {
    const int k = (f - 2) / 5;  // 4*owner + slot
    off = 1 + 3 * k, width = 3, cmp = (f - 2) % 5;
  } else if (f < 44) {
    off = 25, width = 2, cmp = f - 42;
  } else if (f < 60) {
    const int k = (f - 44) / 2;
    width = 2, cmp = (f - 44) % 2;
    if (k < 2) {
      off = 27 + 2 * k;
    } else {
      off = 2 * (k - 2), k1 = 1;
    }
  } else if (f < 62) {
    off = 12 + 4 * (f - 60), width = 4, raw = 1, k1 = 1;
  } else {
    const int q = (f - 62) / 18;
    off = 20 + 5 * q, width = 5, cmp = (f - 62) % 18, k1 = 1;
  }
  return off | (width << 8) | (cmp << 16) | (raw << 24) | (k1 << 25) | (P << 26);
}

struct ObsKey {
  uint32_t k0p0, k0p1, k1;
};

__device__ __forceinline__ ObsKey obs_key(const Lane& L) {
  const bool term = is_terminal(L);
  uint32_t vis0 = 0, vis1 = 0, face_lo = 0, k1 = 0;
#pragma unroll
  for (uint32_t k = 0; k < 8; ++k) {
    const uint32_t n = nib(k < 4 ? L.h0 : L.h1, k & 3u);
    const uint32_t up = n & 1u;
    const uint32_t own = n == 0xFu ? 7u : (n >> 1);          // owner sees every card
    const uint32_t pub = (n == 0xFu || !up) ? 7u : (n >> 1); // others see face-up cards
    vis0 |= (k < 4 ? own : pub) << (1u + 3u * k);
    vis1 |= (k < 4 ? pub : own) << (1u + 3u * k);
    const uint32_t face = n == 0xFu ? 3u : up;
    if (k < 2)
      face_lo |= face << (27u + 2u * k);
    else
      k1 |= face << (2u * (k - 2u));
  }
  const uint32_t cur = (term ? 3u : L.M) << 25;
  ObsKey K;
  K.k0p0 = vis0 | cur | face_lo;
  K.k0p1 = 1u | vis1 | cur | face_lo;
  K.k1 = k1 | (L.c0 << 12) | (L.c1 << 16) | (L.l0 << 20) | (L.l1 << 25);
  return K;
}

__device__ __forceinline__ float obs_decode(uint32_t d, uint32_t k0p0, uint32_t k0p1, uint32_t k1) {
  const uint32_t w = (d & (1u << 25)) ? k1 : ((d & (1u << 26)) ? k0p1 : k0p0);
  const uint32_t v = __builtin_amdgcn_ubfe(w, d & 31u, (d >> 8) & 31u);
  const uint32_t c = (d >> 16) & 31u;
  return (d & (1u << 24)) ? (float)v : (v == c ? 1.0f : 0.0f);
}

// All 64 lanes of the wave must call this (no lane may have exited).
// wave_obs: the wave's first row; n_valid: rows of this wave that exist.
template <bool NT>
__device__ __forceinline__ void write_obs_wave(float* __restrict__ wave_obs, const ObsKey& K, uint32_t n_valid,
                                               const uint4* __restrict__ desc_lds) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  v4f* dst = reinterpret_cast<v4f*>(wave_obs);
  const uint32_t lane = threadIdx.x & 63u;
#pragma unroll 7
  for (uint32_t j = 0; j < (uint32_t)kRowF4; ++j) {
    const uint32_t x = 64u * j + lane;
    const uint32_t o = x / (uint32_t)kRowF4;
    const uint32_t c = x - o * (uint32_t)kRowF4;
    const uint32_t a0 = (uint32_t)__shfl((int)K.k0p0, (int)o);
    const uint32_t a1 = (uint32_t)__shfl((int)K.k0p1, (int)o);
    const uint32_t b = (uint32_t)__shfl((int)K.k1, (int)o);
    const uint4 d = desc_lds[c];
    v4f v;
    v.x = obs_decode(d.x, a0, a1, b);
    v.y = obs_decode(d.y, a0, a1, b);
    v.z = obs_decode(d.z, a0, a1, b);
    v.w = obs_decode(d.w, a0, a1, b);
    if (o < n_valid) {
      if (NT)
        __builtin_nontemporal_store(v, dst + x);
      else
        dst[x] = v;
    }
  }
}

// ---- bitmap variant -------------------------------------------------------
//
// Every element of the two observation rows is 0 or 1 except the four coin
// counts, so a lane's 196 floats are a 196-bit string plus two coin values.
// Each lane builds that string once (one row as a 98-bit (lo, hi) pair per
// observer, concatenated), stores it with the coins as 8 words in LDS, and
// the coalesced store loop turns nibble c of the owner's string into the
// float4 at offset 4c.  Coins sit at row offsets 60-61: float4 15 (.x, .y)
// of the P1 row and float4 39 (.z, .w) of the P2 row.


// 8 LDS words of a lane: the 196-bit string (row P1 at bits 0..97, row P2
// at 98..195) in words 0..6, coins (P1 | P2 << 8) in word 7.

__device__ __forceinline__ void obs_bits_to_lds(const Lane& L, uint32_t* __restrict__ w) {
  const bool term = is_terminal(L);
  uint64_t a_lo, a_hi, b_lo, b_hi;
  obs_row_bits<0>(L, term, a_lo, a_hi);
  obs_row_bits<1>(L, term, b_lo, b_hi);
  uint4 x, y;
  x.x = (uint32_t)a_lo;
  x.y = (uint32_t)(a_lo >> 32);
  x.z = (uint32_t)a_hi;
  x.w = (uint32_t)((a_hi >> 32) & 3u) | (uint32_t)(b_lo << 2);
  y.x = (uint32_t)(b_lo >> 30);
  y.y = (uint32_t)(b_lo >> 62) | (uint32_t)(b_hi << 2);
  y.z = (uint32_t)(b_hi >> 30) & 0xFu;
  y.w = L.c0 | (L.c1 << 8);
  reinterpret_cast<uint4*>(w)[0] = x;
  reinterpret_cast<uint4*>(w)[1] = y;
}

// wave_bits: this wave's 64 x 8 LDS words, written by obs_bits_to_lds and
// made visible by a barrier before the call.
// Store policy of the wave-bitmap writer: 0 plain, 1 non-temporal (global
// stores), 2 sc1 write-through (buffer stores through a wave-uniform
// resource whose range ends at the wave's last row, so rows past the batch
// are dropped by the range check instead of a per-store predicate), 3 the
// same with sc0 sc1 (system scope: the op server's stores into mapped host
// memory, which need no L2 write-back afterwards).
template <int POL, class V>
__device__ __forceinline__ void store_f4(V* p, const V& v) {
  if (POL == 0)
    *p = v;
  else
    __builtin_nontemporal_store(v, p);
}

// FULL: all 64 rows of the wave exist (no per-store predicate, so the
// unrolled iterations' LDS reads can be hoisted ahead of their stores).
// (x, o, c) = (64 j + lane, x / 49, x % 49) advance incrementally: x += 64
// is one row (49) plus 15.
template <int POL, bool FULL>
__device__ __forceinline__ void write_obs_wave_bits(float* __restrict__ wave_obs, const uint32_t* __restrict__ wave_bits,
                                                    uint32_t n_valid) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const uint32_t lane = threadIdx.x & 63u;
  v4f* dst = reinterpret_cast<v4f*>(wave_obs) + lane;
  __amdgpu_buffer_rsrc_t rsrc;
  if (POL >= 2) rsrc = __builtin_amdgcn_make_buffer_rsrc(wave_obs, (short)0, (int)(n_valid * 2u * kObsSize * 4u), 0x00020000);
  uint32_t o = lane >= (uint32_t)kRowF4 ? 1u : 0u;
  uint32_t c = lane - o * (uint32_t)kRowF4;
#pragma unroll 7
  for (uint32_t j = 0; j < (uint32_t)kRowF4; ++j) {
    const uint32_t word = wave_bits[8u * o + (c >> 3)];
    const uint32_t coins = wave_bits[8u * o + 7u];
    const uint32_t nb = word >> (4u * (c & 7u));
    v4f v;
    v.x = (float)(nb & 1u);
    v.y = (float)((nb >> 1) & 1u);
    v.z = (float)((nb >> 2) & 1u);
    v.w = (float)((nb >> 3) & 1u);
    const float c0 = (float)(coins & 0xFFu), c1 = (float)(coins >> 8);
    v.x = c == 15u ? c0 : v.x;
    v.y = c == 15u ? c1 : v.y;
    v.z = c == 39u ? c0 : v.z;
    v.w = c == 39u ? c1 : v.w;
    if (POL >= 2)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), rsrc, (int)(16u * (64u * j + lane)), 0,
                                             POL == 3 ? 17 : 16);
    else if (FULL || o < n_valid)
      store_f4<POL>(dst + 64u * j, v);
    c += 15u;
    o += 1u;
    const bool wrap = c >= (uint32_t)kRowF4;
    c = wrap ? c - (uint32_t)kRowF4 : c;
    o += wrap ? 1u : 0u;
  }
}

// Block-cooperative form: the T lanes of a block own T consecutive rows
// (T x 784 B contiguous) and iteration j stores float4 T*j + t, so each
// iteration of the block writes T x 16 contiguous bytes (16 KiB at T=1024).
// Measured with no compute (tools/hbm_probe.hip), this order streams ~8%
// faster than per-wave chunks.
template <int T, bool NT>
__device__ __forceinline__ void write_obs_block_bits(float* __restrict__ block_obs, const uint32_t* __restrict__ bits,
                                                     uint32_t n_valid) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  v4f* dst = reinterpret_cast<v4f*>(block_obs);
#pragma unroll 7
  for (uint32_t j = 0; j < (uint32_t)kRowF4; ++j) {
    const uint32_t x = (uint32_t)T * j + threadIdx.x;
    const uint32_t o = x / (uint32_t)kRowF4;
    const uint32_t c = x - o * (uint32_t)kRowF4;
    const uint32_t word = bits[8u * o + (c >> 3)];
    const uint32_t coins = bits[8u * o + 7u];
    const uint32_t nb = word >> (4u * (c & 7u));
    v4f v;
    v.x = (float)(nb & 1u);
    v.y = (float)((nb >> 1) & 1u);
    v.z = (float)((nb >> 2) & 1u);
    v.w = (float)((nb >> 3) & 1u);
    const float c0 = (float)(coins & 0xFFu), c1 = (float)(coins >> 8);
    v.x = c == 15u ? c0 : v.x;
    v.y = c == 15u ? c1 : v.y;
    v.z = c == 39u ? c0 : v.z;
    v.w = c == 39u ? c1 : v.w;
    if (o < n_valid) {
      if (NT)
        __builtin_nontemporal_store(v, dst + x);
      else
        dst[x] = v;
    }
  }
}

// ---- InformationStateTensor ----------------------------------------------
//
// CoupObserver::WriteTensor with kInfoStateObsType (perfect recall,
// coup.cc:248-287, 230-245; observer.h:294-297): the first 62 elements are
// the observation's (observer, cards, mover, card faces, coins), then the
// history block [135][18] with row i = history index i, one-hot at the
// action id for player actions and at the card type for chance deals to the
// observer only.  2492 floats per player, both players per lane = 1246
// float4 (19,936 B).  Written wave-cooperatively like the observation: the
// wave's 64 lanes own 1.27 MB contiguous, iteration j stores float4 64*j+lane.
//
// Per-lane LDS inputs: the 96-byte history (hist_lds, the lane's bytes of
// the global history buffer) and 6 words of prefix (pre_lds): [0..1] the
// P1-view prefix bits (element f of 0..61 at bit f), [2..3] the P2 view,
// [4] coins (P1 | P2 << 8) | move_number << 16.
#ifndef COUP_INFO_STORE_POLICY
#define COUP_INFO_STORE_POLICY 2  // 2 sc1 buffer stores (4% faster than 1, non-temporal: DESIGN.md section 5)
#endif
constexpr int kInfoStorePolicy = COUP_INFO_STORE_POLICY;


// All 64 lanes of the wave must call this.  (x, o, c) = (64 j + lane,
// x / 1246, x % 1246) advance incrementally.  A float4 whose first element
// lies in a history row at or past the lane's history length is zero (most
// of the [135][18] block: a uniform-random game is ~21 moves long), and the
// 64 float4 of one store mostly belong to one lane, so the decode below is
// skipped wave-wide for those stores (the writer was VALU-bound: 85% busy).
template <int POL>
__device__ __forceinline__ void write_info_wave(float* __restrict__ wave_info, const uint8_t* __restrict__ hist,
                                                const uint32_t* __restrict__ pre, uint32_t n_valid) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const uint32_t lane = threadIdx.x & 63u;
  v4f* dst = reinterpret_cast<v4f*>(wave_info) + lane;
  __amdgpu_buffer_rsrc_t rsrc;
  if (POL == 2)
    rsrc = __builtin_amdgcn_make_buffer_rsrc(wave_info, (short)0, (int)(n_valid * 2u * kInfoSize * 4u), 0x00020000);
  uint32_t o = 0u, c = lane;
#pragma unroll 2
  for (uint32_t j = 0; j < (uint32_t)kInfoF4; ++j) {
    const uint32_t p = c >= (uint32_t)kInfoHalfF4;
    const int f0 = 4 * (int)(c - p * (uint32_t)kInfoHalfF4);
    const uint32_t* po = pre + kPreWords * o;
    const uint32_t meta = po[4];
    const uint32_t len = meta >> 16;
    v4f w = {0.0f, 0.0f, 0.0f, 0.0f};
    if (f0 < 62 + 18 * (int)len) {
      const uint64_t prefix = (uint64_t)po[2u * p] | ((uint64_t)po[2u * p + 1u] << 32);  // 32-bit loads
      // history rows touched by elements f0..f0+3 (t = f - 62; two rows at most)
      const int t0 = f0 - 62;
      const uint32_t r0 = t0 < 0 ? 0u : (uint32_t)t0 / 18u;
      const int col0 = t0 - 18 * (int)r0;
      uint32_t va[2];
#pragma unroll
      for (uint32_t k = 0; k < 2; ++k) {
        const uint32_t r = r0 + k;
        const uint32_t e = hist[kHist * o + (r < (uint32_t)kHist ? r : 0u)];
        const bool seen = (e & 0x20u) == 0u || ((e >> 6) & 1u) == p;  // deals: observer's only
        va[k] = (r < len && seen) ? (e & 0x1Fu) : 31u;
      }
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int f = f0 + e;
        const int col = col0 + e;
        const uint32_t row_act = col >= 18 ? va[1] : va[0];
        const float h = (row_act == (uint32_t)(col >= 18 ? col - 18 : col)) ? 1.0f : 0.0f;
        const float pb = (float)((uint32_t)(prefix >> (f & 63)) & 1u);
        const float coin = (float)(f == 60 ? (meta & 0xFFu) : ((meta >> 8) & 0xFFu));
        v[e] = f < 60 ? pb : (f < 62 ? coin : h);
      }
      w = v4f{v[0], v[1], v[2], v[3]};
    }
    if (POL == 2)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, w), rsrc, (int)(16u * (64u * j + lane)), 0, 16);
    else if (o < n_valid)
      __builtin_nontemporal_store(w, dst + 64u * j);
    c += 64u;
    const bool wrap = c >= (uint32_t)kInfoF4;
    c = wrap ? c - (uint32_t)kInfoF4 : c;
    o += wrap ? 1u : 0u;
  }
}

// Cooperative copy of a wave's 64 x 96 history bytes between global memory
// and LDS (6 x 1 KiB per direction; bytes past the last lane are skipped).
template <bool TO_LDS>
__device__ __forceinline__ void wave_hist_copy(uint8_t* __restrict__ global_wave, uint8_t* __restrict__ lds_wave,
                                               uint32_t n_valid) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t limit = n_valid * (uint32_t)kHist;
#pragma unroll
  for (uint32_t j = 0; j < 6u; ++j) {
    const uint32_t off = 1024u * j + 16u * lane;
    if (off < limit) {
      if (TO_LDS)
        *reinterpret_cast<uint4*>(lds_wave + off) = *reinterpret_cast<const uint4*>(global_wave + off);
      else
        *reinterpret_cast<uint4*>(global_wave + off) = *reinterpret_cast<const uint4*>(lds_wave + off);
    }
  }
}

// Fill the block's LDS copy of the 196-entry descriptor table (as 49 uint4).
__device__ __forceinline__ void load_obs_desc(uint32_t* desc_lds) {
  for (int g = threadIdx.x; g < 2 * kObsSize; g += blockDim.x) desc_lds[g] = obs_desc(g);
  __syncthreads();
}

__device__ __forceinline__ void count_error(uint32_t* err_count) { atomicAdd(err_count, 1u); }

// ------------------------------------------------------------------ kernels

struct StepArgs {
  uint4* state;
  int64_t n;
  uint32_t seed_lo, seed_hi, env_id_base;
  int auto_reset;
  const int8_t* actions_in;
  int8_t* actions;
  int8_t* rewards;
  uint8_t* step_type;
  uint32_t* legal;
  int8_t* cur_player;
  float* obs;
  uint8_t* hist;   // [B][96] history bytes (INFO != kInfoNone)
  float* info;     // [B][2][2492] (INFO == kInfoWrite)
  EpAcc ep;        // per-episode accumulators (coup_step_outputs.episodes / return_sum or episode_word)
  uint32_t* err_count;
  int xcd_remap;   // block -> lane group mapping (xcd_group)
  int unchecked;   // caller actions outside LegalActions go through the reference's unchecked ApplyAction
                   // (COUP_FLAG_UNCHECKED; in-place kernels with caller actions only)
#ifdef COUP_WAVE_TRACE
  // measurement builds only (tools/wave_trace.py): per wave, 100 MHz
  // timestamps at entry, end of the step, end of store issue, stores
  // drained, then HW_ID << 32 | XCC_ID, then the state load's return, then
  // (first active lane) action drawn, decision applied, deals done, step done
  uint64_t* trace;
#endif
};



#ifdef COUP_WAVE_TRACE
#define COUP_TRACE(a, k)                                                                           \
  do {                                                                                             \
    if ((a).trace && (threadIdx.x & 63u) == 0u)                                                    \
      (a).trace[((size_t)blockIdx.x * (blockDim.x / 64u) + threadIdx.x / 64u) * 10u + (k)] =      \
          __builtin_amdgcn_s_memrealtime();                                                        \
  } while (0)
// stamp by the first active lane (inside code some lanes have left)
#define COUP_TRACE_ANY(a, k)                                                                        \
  do {                                                                                              \
    if ((a).trace && (threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(__builtin_amdgcn_read_exec()))  \
      (a).trace[((size_t)blockIdx.x * (blockDim.x / 64u) + threadIdx.x / 64u) * 10u + (k)] =        \
          __builtin_amdgcn_s_memrealtime();                                                         \
  } while (0)
#else
#define COUP_TRACE(a, k) \
  do {                   \
  } while (0)
#define COUP_TRACE_ANY(a, k) \
  do {                       \
  } while (0)
#endif

// Lane group of block b in a grid of G.  Blocks are dealt round-robin over
// the 8 XCDs (MI355X_MICROARCH.md, workgroup dispatch), so without a remap
// neighbouring groups -- and their neighbouring obs rows -- land on
// different XCDs.  The remap gives XCD x the contiguous run of groups
// [x G/8, (x+1) G/8) in dispatch order; blocks past the last full round of 8
// keep their own index.  A bijection on [0, G).  Measured on the obs store
// stream alone: 157 -> 143 us (tools/store_probe.hip).
__device__ __forceinline__ uint32_t xcd_group(uint32_t b, uint32_t G) {
  const uint32_t full = G & ~7u;
  if (b >= full) return b;
  return (b & 7u) * (full >> 3) + (b >> 3);
}

// Observation write-out variants (COUP_OBS_MODE selects one at run time for
// A/B measurements; kObsWaveBitsSc1 is the default):
//   1 per-lane rows (each lane stores its own 784 B; uncoalesced)
//   2/3 wave-cooperative, ds_bpermute keys + descriptor table (plain / nt)
//   4 wave-cooperative from the LDS bitmap, nt stores
//   5/6 block-cooperative from the LDS bitmap, 256 / 1024 threads, plain stores
//   7 block-cooperative, 1024 threads, nt stores
//   8/9 as 4 with plain / sc1 (write-through) stores
enum ObsMode : int {
  kObsNone = 0, kObsLaneRows = 1, kObsWave = 2, kObsWaveNT = 3, kObsWaveBits = 4,
  kObsBlockBits = 5, kObsBlockBitsNT = 7, kObsWaveBitsPlain = 8, kObsWaveBitsSc1 = 9
};
constexpr bool is_wave_bits(int m) { return m == kObsWaveBits || m == kObsWaveBitsPlain || m == kObsWaveBitsSc1; }
constexpr int wave_bits_policy(int m) { return m == kObsWaveBitsPlain ? 0 : (m == kObsWaveBitsSc1 ? 2 : 1); }

// A caller action under COUP_FLAG_UNCHECKED: the reference's unchecked
// ApplyAction (apply_action_unchecked, coup_lane.h) on record w into *out;
// returns whether it was applied (false: the reference raises, *out not
// written).  Every caller action of such an env takes it, legal or not --
// LegalActions can offer an action DoApplyAction then refuses once
// unchecked play has left legal play's states (a Challenge of a Block of a
// Tax: coup.cc:930-933 offers it, :691-692 raises).  Out of line, so the
// caller-action kernels keep one transition's registers.
__device__ __noinline__ uint32_t unchecked_decision(uint4 w, uint32_t x, uint4* out) {
  Lane L = unpack(w);
  NoHistory none;
  if (!apply_action_unchecked(L, x, none)) return 0u;
  *out = pack(L);
  return 1u;
}

// The per-lane part of one env step: returns the decision applied (-1 if
// none), the step type, player 0's reward and, at LAST, player 0's return of
// the finished game; L is updated in place and every applied action is
// recorded in `hist`.  FLOW: the decision through apply_decision_v1 (the
// reference's branches) instead of the effect form -- the kernels that write
// observations are bound by their stores, and there the effect form's extra
// VALU work and registers cost more than its shorter divergent paths save
// (same-process A/B, profiles/r02/ab/ab_rules_c3.txt: 160.6 vs 165.6 us per
// 2^20-lane step); the rules-bound kernels take the effect form (c2 8.4 ->
// 7.7 us, c2r 3.61 -> 3.20 us per step, profiles/r02/ab/ab_rules_c2*.txt).
//
// UNCHECKED (COUP_FLAG_UNCHECKED, caller actions only): the decision goes
// through unchecked_decision instead, legal or not.  A compile-time switch:
// the checked kernels' code is exactly what it is without it -- with the
// two paths as a run-time branch in one kernel, ROCm 7.2 produced the
// DESIGN.md section 12 defect in the checked branch (record word 3 after a
// Tax announcement, k_step<false, 0, 256, 1>; tests/test_gpu_server.py).
template <bool UNIFORM, bool FLOW, bool UNCHECKED, class H, class R>
__device__ __forceinline__ void step_lane_rng(const StepArgs& a, int64_t i, Lane& L, int& act, uint32_t& st,
                                              int32_t& rew, int32_t& ret, H& hist, R& rng,
                                              bool count = true) {
  act = -1;
  rew = 0;
  if (!UNIFORM && (int8_t)a.actions_in[i] < 0) {
    // a negative action skips the lane: untouched, no error (SyncVectorEnv
    // stepping a subset of its envs in one launch)
    st = COUP_STEP_SKIPPED;
    return;
  }
  if (is_terminal(L)) {
    // step() after LAST starts a new episode (rl_environment.py:310-311)
    L = new_episode(L.episode + 1u, rng, hist);
    st = COUP_STEP_FIRST;
    return;
  }
  resolve_chance(L, rng, hist);  // no-op unless the lane was left at a chance node
  const uint32_t m = decision_mask(L);
  uint32_t x;
  if (UNIFORM) {
    // in place, the rules-bound kernels mix every draw in a wave: no loop
    x = m ? (FLOW ? sample_action(m, rng.draw(L.episode, L.move)) : sample_action_select(m, rng.draw(L.episode, L.move)))
          : 32u;
  } else {
    x = (uint32_t)(uint8_t)a.actions_in[i];
  }
  COUP_TRACE_ANY(a, 6);
  st = COUP_STEP_MID;
  uint32_t err_before;
  if constexpr (UNCHECKED) {
    err_before = L.err;
    uint4 w;
    if (!unchecked_decision(pack(L), x, &w)) {
      if (count) count_error(a.err_count);
      return;
    }
    hist.record(L.move, hist_decision(x, L.M));
    L = unpack(w);
  } else {
    if (x > 17u || ((m >> x) & 1u) == 0u || is_terminal(L)) {
      if (count) count_error(a.err_count);
      return;
    }
    err_before = L.err;
    hist.record(L.move, hist_decision(x, L.M));
    if (FLOW)
      apply_decision_v1(L, x);
    else
      apply_decision(L, x);
    L.move += 1u;
  }
  COUP_TRACE_ANY(a, 7);
  resolve_chance(L, rng, hist);
  COUP_TRACE_ANY(a, 8);
  if (count && L.err && !err_before) count_error(a.err_count);
  act = (int)x;
  rew = L.r0;
  if (is_terminal(L)) {
    st = COUP_STEP_LAST;
    ret = return0(L);
    if (a.auto_reset) {
      // SyncVectorEnv.step(reset_if_done=True) (vector_env.py:62-65)
      L = new_episode(L.episode + 1u, rng, hist);
    }
  }
  COUP_TRACE_ANY(a, 9);
}

template <bool UNIFORM, bool FLOW, bool UNCHECKED, class H>
__device__ __forceinline__ void step_lane(const StepArgs& a, int64_t i, Lane& L, int& act, uint32_t& st,
                                          int32_t& rew, int32_t& ret, H& hist) {
  Rng rng{a.seed_lo, a.seed_hi, lane_stream_id(a.env_id_base, i), 0u, make_uint4(0, 0, 0, 0)};
  step_lane_rng<UNIFORM, FLOW, UNCHECKED>(a, i, L, act, st, rew, ret, hist, rng);
}

// The per-episode accumulators (coup_episodes.h): the lane's word(s) are
// loaded with its record, before the rules, and every lane stores them back
// (coalesced; unchanged where no episode ended).  Same-process A/B on the c3
// step with the int32 pair (2^20 lanes, obs x2; profiles/r02/ab/
// ab_epstats.jsonl): no accumulators 148.8 us, this form 153.0, stores only
// where an episode ended 163.3, load-add-store after the rules at those lanes
// 163.9 -- the ~7% of lanes that finish scatter their stores over most lines,
// and those partial-line writes cost more than full-line ones.  The packed
// int16 word (round 4) moves 2 bytes per lane each way instead of 8.
__device__ __forceinline__ EpVal ep_prefetch(const StepArgs& a, int64_t i, bool active) {
  return active ? a.ep.load(i) : EpVal{0, 0};
}

__device__ __forceinline__ void ep_update(const StepArgs& a, int64_t i, EpVal e, uint32_t st, int32_t ret) {
  const bool last = st == COUP_STEP_LAST;
  a.ep.store(i, e, last ? 1 : 0, last ? ret : 0);
}

// Wave-scope hand-off of LDS data between lanes of one wave.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// History handling of the step kernel.
enum InfoMode : int { kInfoNone = 0, kInfoHistory = 1, kInfoWrite = 2 };

template <int OBS, int T, int INFO>
struct StepLds {
  static constexpr bool kDesc = OBS == kObsWave || OBS == kObsWaveNT;
  static constexpr bool kBits = is_wave_bits(OBS) || OBS == kObsBlockBits || OBS == kObsBlockBitsNT;
  uint4 desc[kDesc ? kRowF4 : 1];
  uint32_t bits[kBits ? T * 8 : 1];
  uint8_t hist[INFO != kInfoNone ? T * kHist : 16];
  uint32_t pre[INFO == kInfoWrite ? T * kPreWords : 1];
};

template <bool UNIFORM, int OBS, int T, int INFO, bool UNCHECKED>
__device__ __forceinline__ void step_group(const StepArgs& a, int64_t grp, StepLds<OBS, T, INFO>& lds, uint4 rec);

// This thread's lane record of group grp (zeros past the batch).
template <int T>
__device__ __forceinline__ uint4 load_record(const StepArgs& a, int64_t grp) {
  const int64_t i = grp * T + threadIdx.x;
  return i < a.n ? a.state[i] : make_uint4(0u, 0u, 0u, 0u);
}

// One rl_environment step per lane (rl_environment.py:282-322), optionally
// with SyncVectorEnv auto-reset (vector_env.py:40-67).  T threads per block.
// No early exit: the cooperative writers need every lane of the wave /
// block.  INFO: maintain the per-lane history, and write the
// InformationStateTensor of both players.
template <bool UNIFORM, int OBS, int T, int INFO, bool UNCHECKED = false>
__global__ __launch_bounds__(T, INFO == kInfoNone ? 8 : 4) void k_step(StepArgs a) {
  __shared__ StepLds<OBS, T, INFO> lds;
  if (StepLds<OBS, T, INFO>::kDesc) load_obs_desc(reinterpret_cast<uint32_t*>(lds.desc));
  // One group of T lanes per block.  (A persistent variant -- a resident
  // grid looping over groups, loading the next group's records one group
  // ahead -- measured no faster: DESIGN.md section 5.)
  COUP_TRACE(a, 0);
  const uint32_t grp = a.xcd_remap ? xcd_group(blockIdx.x, gridDim.x) : blockIdx.x;
  step_group<UNIFORM, OBS, T, INFO, UNCHECKED>(a, grp, lds, load_record<T>(a, grp));
#ifdef COUP_WAVE_TRACE
  COUP_TRACE(a, 2);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  COUP_TRACE(a, 3);
  if (a.trace && (threadIdx.x & 63u) == 0u)
    a.trace[((size_t)blockIdx.x * (blockDim.x / 64u) + threadIdx.x / 64u) * 10u + 4u] =
        ((uint64_t)__builtin_amdgcn_s_getreg(4 | (31 << 11)) << 32) | (uint32_t)__builtin_amdgcn_s_getreg(20 | (31 << 11));
#endif
}

// Obs store loop of a wave-bitmap group whose words are in LDS.
template <int OBS, int T, int INFO>
__device__ __forceinline__ void step_group_store(const StepArgs& a, int64_t grp, StepLds<OBS, T, INFO>& lds) {
  const uint32_t wl = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x & ~63u));
  const int64_t wave0 = grp * T + wl;
  const int64_t wleft = a.n - wave0;
  const uint32_t wave_valid = wleft >= 64 ? 64u : (wleft > 0 ? (uint32_t)wleft : 0u);  // wave-uniform
  float* wave_obs = a.obs + wave0 * (2 * kObsSize);
  if (wave_valid == 64u)
    write_obs_wave_bits<wave_bits_policy(OBS), true>(wave_obs, lds.bits + wl * 8u, 64u);
  else if (wave_valid > 0u)
    write_obs_wave_bits<wave_bits_policy(OBS), false>(wave_obs, lds.bits + wl * 8u, wave_valid);
  wave_sync();  // words read before the next group overwrites them
}

// Step of group grp up to (for the wave-bitmap writers) the words in LDS.
template <bool UNIFORM, int OBS, int T, int INFO, bool UNCHECKED>
__device__ __forceinline__ void step_group_compute(const StepArgs& a, int64_t grp, StepLds<OBS, T, INFO>& lds,
                                                   uint4 rec);

template <bool UNIFORM, int OBS, int T, int INFO, bool UNCHECKED>
__device__ __forceinline__ void step_group(const StepArgs& a, int64_t grp, StepLds<OBS, T, INFO>& lds, uint4 rec) {
  step_group_compute<UNIFORM, OBS, T, INFO, UNCHECKED>(a, grp, lds, rec);
  if (is_wave_bits(OBS)) step_group_store<OBS, T, INFO>(a, grp, lds);
}

template <bool UNIFORM, int OBS, int T, int INFO, bool UNCHECKED>
__device__ __forceinline__ void step_group_compute(const StepArgs& a, int64_t grp, StepLds<OBS, T, INFO>& lds,
                                                   uint4 rec) {
  constexpr bool kDesc = StepLds<OBS, T, INFO>::kDesc;
  constexpr bool kBits = StepLds<OBS, T, INFO>::kBits;
  const int64_t i = grp * T + threadIdx.x;
  const bool active = i < a.n;
  // first thread of this wave; readfirstlane keeps the wave-uniform values
  // below in SGPRs across the step
  const uint32_t wl = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x & ~63u));
  const int64_t wave0 = grp * T + wl;
  const int64_t wleft = a.n - wave0;
  const uint32_t wave_valid = wleft >= 64 ? 64u : (wleft > 0 ? (uint32_t)wleft : 0u);  // wave-uniform
  uint8_t* hist_wave = lds.hist + wl * kHist;
  const EpVal eps = ep_prefetch(a, i, active);
  if (INFO != kInfoNone) {
    if (wave_valid) wave_hist_copy<true>(a.hist + wave0 * kHist, hist_wave, wave_valid);
    wave_sync();
  }
  Lane L = initial_lane(0);
  if (active) {
    L = unpack(rec);
#ifdef COUP_WAVE_TRACE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    COUP_TRACE(a, 5);
#endif
    int act;
    uint32_t st;
    int32_t rew, ret = 0;
    constexpr bool kFlow = OBS != kObsNone || INFO != kInfoNone;  // store-bound kernels (step_lane)
    if (INFO != kInfoNone) {
      RegHistory rec;
      step_lane<UNIFORM, kFlow, UNCHECKED>(a, i, L, act, st, rew, ret, rec);
      rec.flush(lds.hist + threadIdx.x * kHist);
    } else {
      NoHistory none;
      step_lane<UNIFORM, kFlow, UNCHECKED>(a, i, L, act, st, rew, ret, none);
    }
    a.state[i] = pack(L);
    ep_update(a, i, eps, st, ret);
    if (a.actions) a.actions[i] = (int8_t)act;
    if (a.rewards) {
      a.rewards[2 * i] = (int8_t)rew;
      a.rewards[2 * i + 1] = (int8_t)(-rew);
    }
    if (a.step_type) a.step_type[i] = (uint8_t)st;
    if (a.legal) a.legal[i] = legal_mask(L);
    if (a.cur_player) a.cur_player[i] = (int8_t)current_player(L);
    if (OBS == kObsLaneRows) write_obs_pair(a.obs + i * (2 * kObsSize), L);
  }
  if (INFO != kInfoNone) {
    if (INFO == kInfoWrite) info_prefix_to_lds(L, lds.pre + threadIdx.x * kPreWords);
    wave_sync();
    if (wave_valid) wave_hist_copy<false>(a.hist + wave0 * kHist, hist_wave, wave_valid);
    if (INFO == kInfoWrite && wave_valid)
      write_info_wave<kInfoStorePolicy>(a.info + wave0 * (2 * kInfoSize), hist_wave, lds.pre + wl * kPreWords,
                                        wave_valid);
    wave_sync();  // this group's LDS words read before the next group reuses them
  }
  COUP_TRACE(a, 1);
  if (is_wave_bits(OBS)) {
    // each wave reads only its own lanes' words: a wave-scope hand-off
    obs_bits_to_lds(L, lds.bits + threadIdx.x * 8u);
    wave_sync();
  } else if (kBits) {
    __syncthreads();  // previous group's words fully read by every wave
    obs_bits_to_lds(L, lds.bits + threadIdx.x * 8u);
    __syncthreads();
  }
  if (OBS == kObsBlockBits || OBS == kObsBlockBitsNT) {
    const int64_t block0 = grp * T;
    const int64_t left = a.n - block0;
    const uint32_t n_valid = left >= T ? (uint32_t)T : (uint32_t)left;  // block-uniform, > 0
    write_obs_block_bits<T, OBS == kObsBlockBitsNT>(a.obs + block0 * (2 * kObsSize), lds.bits, n_valid);
  } else if (kDesc && wave_valid > 0) {
    write_obs_wave<OBS == kObsWaveNT>(a.obs + wave0 * (2 * kObsSize), obs_key(L), wave_valid, lds.desc);
  }
}

// Lane k (0..3) of this thread's quad, by DPP quad_perm (a VALU operand
// modifier: no LDS round trip, unlike __shfl's ds_bpermute).
template <int K>
__device__ __forceinline__ uint32_t quad_bcast(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, K * 0x55, 0xF, 0xF, true);
}
template <int K>
__device__ __forceinline__ uint4 quad_bcast4(uint4 v) {
  return make_uint4(quad_bcast<K>(v.x), quad_bcast<K>(v.y), quad_bcast<K>(v.z), quad_bcast<K>(v.w));
}

// The rules-bound step (no observation, no history; c2's kernel at 65,536
// lanes, where 256-lane blocks give ONE wave per SIMD and a lane's dependent
// chain -- record load, Philox, rules, deals, reset -- is exposed).  TPL
// threads play each lane: the Philox blocks the step can need (PrefRng) are
// computed ahead by the group's threads in parallel (TPL = 4: thread q
// computes block q of {current, next, next episode's first}; TPL = 2: two
// each; TPL = 1: all three, interleaved) and traded by DPP within the quad;
// then every thread of the group runs the same rules (branch-free for the
// group, so a wave diverges over 64 / TPL lanes instead of 64), and thread 0
// stores.  TPL > 1 puts TPL waves on each SIMD to hide each other's latency.
// Same draws as k_step (PrefRng::draw == Rng::draw), so the same games.
template <int TPL, bool UNIFORM>
__global__ __launch_bounds__(256) void k_step_group(StepArgs a) {
  static_assert(TPL == 1 || TPL == 2 || TPL == 4, "threads per lane");
  constexpr int kLanes = 256 / TPL;
  const uint32_t q = threadIdx.x % TPL;
  const int64_t i = (int64_t)blockIdx.x * kLanes + threadIdx.x / TPL;
  const bool active = i < a.n;
  const uint4 rec = active ? a.state[i] : pack(initial_lane(0u));
  const EpVal eps = ep_prefetch(a, i, active && q == 0u);
  Lane L = unpack(rec);
  const uint32_t id = lane_stream_id(a.env_id_base, i);
  const uint32_t b = L.move >> 2, ep = L.episode, ep1 = (L.episode + 1u) & kEpisodeMask;
  uint4 c0, c1, r0;
  if (TPL == 4) {
    const uint32_t e = q < 2u ? ep : ep1, bb = q == 0u ? b : (q == 1u ? b + 1u : 0u);
    const uint4 mine = PrefRng::block(a.seed_lo, a.seed_hi, id, e, bb);
    c0 = quad_bcast4<0>(mine);
    c1 = quad_bcast4<1>(mine);
    r0 = quad_bcast4<2>(mine);
  } else if (TPL == 2) {
    // thread 0 of the pair: current + next block; thread 1: next episode's
    // first + next block (the same number of evaluations on both)
    const uint4 m0 = PrefRng::block(a.seed_lo, a.seed_hi, id, q == 0u ? ep : ep1, q == 0u ? b : 0u);
    const uint4 m1 = PrefRng::block(a.seed_lo, a.seed_hi, id, ep, b + 1u);
    c1 = m1;
    const uint4 o = make_uint4(
        (uint32_t)__builtin_amdgcn_mov_dpp((int)m0.x, 0xB1, 0xF, 0xF, true),  // quad_perm [1,0,3,2]: the pair's other
        (uint32_t)__builtin_amdgcn_mov_dpp((int)m0.y, 0xB1, 0xF, 0xF, true),
        (uint32_t)__builtin_amdgcn_mov_dpp((int)m0.z, 0xB1, 0xF, 0xF, true),
        (uint32_t)__builtin_amdgcn_mov_dpp((int)m0.w, 0xB1, 0xF, 0xF, true));
    c0 = q == 0u ? m0 : o;
    r0 = q == 0u ? o : m0;
  } else {
    c0 = PrefRng::block(a.seed_lo, a.seed_hi, id, ep, b);
    c1 = PrefRng::block(a.seed_lo, a.seed_hi, id, ep, b + 1u);
    r0 = PrefRng::block(a.seed_lo, a.seed_hi, id, ep1, 0u);
  }
  if (!active) return;  // after the trades: every quad lane took part
  PrefRng rng{a.seed_lo, a.seed_hi, id, ep, b, c0, c1, r0};
  int act;
  uint32_t st;
  int32_t rew, ret = 0;
  NoHistory none;
  step_lane_rng<UNIFORM, false, false>(a, i, L, act, st, rew, ret, none, rng, q == 0u);  // one count per lane
  if (q != 0u) return;
  a.state[i] = pack(L);
  ep_update(a, i, eps, st, ret);
  if (a.actions) a.actions[i] = (int8_t)act;
  if (a.rewards) {
    a.rewards[2 * i] = (int8_t)rew;
    a.rewards[2 * i + 1] = (int8_t)(-rew);
  }
  if (a.step_type) a.step_type[i] = (uint8_t)st;
  if (a.legal) a.legal[i] = legal_mask(L);
  if (a.cur_player) a.cur_player[i] = (int8_t)current_player(L);
}

// The split observation step (COUP_OBS_SPLIT; coup_step): the rules step
// runs without tensors, then this kernel writes every lane's
// ObservationTensor pair (coup.cc:1051-1056, both players) from the
// post-step records.  One block per 4 KiB of the [B][2][98] buffer, in
// address order: the blocks in flight write one contiguous, moving window,
// the grid-stride sweep's pattern, which the lane-owned stores of the fused
// step cannot follow (a wave owns its 64 lanes' 50 KiB; DESIGN.md section
// 5).  The <= 7 lanes a chunk touches are decoded by the block's first
// threads into LDS (obs_bits_to_lds, the fused writer's 8 words per lane)
// and every thread expands one float4 exactly as write_obs_wave_bits does.
// POL 1: non-temporal stores (the fastest policy for this order), 0 plain.
template <int POL>
__global__ __launch_bounds__(256) void k_obs_sweep(const uint4* __restrict__ state, float* __restrict__ obs, int64_t n) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  constexpr uint32_t kLanes = (256u + (uint32_t)kRowF4 - 1u) / (uint32_t)kRowF4 + 1u;  // 7
  __shared__ uint32_t bits[8 * kLanes];
  const uint32_t t = threadIdx.x;
  const int64_t x0 = (int64_t)blockIdx.x * 256;
  const int64_t o0 = x0 / kRowF4;
  if (t < kLanes && o0 + t < n) obs_bits_to_lds(unpack(state[o0 + t]), bits + 8u * t);
  __syncthreads();
  const int64_t x = x0 + t;
  if (x >= n * kRowF4) return;
  const uint32_t rel = (uint32_t)(x0 - o0 * kRowF4) + t;  // float4 offset from lane o0's row start
  const uint32_t o = rel / (uint32_t)kRowF4, c = rel - o * (uint32_t)kRowF4;
  const uint32_t word = bits[8u * o + (c >> 3)], coins = bits[8u * o + 7u];
  const uint32_t nb = word >> (4u * (c & 7u));
  v4f v;
  v.x = (float)(nb & 1u);
  v.y = (float)((nb >> 1) & 1u);
  v.z = (float)((nb >> 2) & 1u);
  v.w = (float)((nb >> 3) & 1u);
  const float c0 = (float)(coins & 0xFFu), c1 = (float)(coins >> 8);
  v.x = c == 15u ? c0 : v.x;
  v.y = c == 15u ? c1 : v.y;
  v.z = c == 39u ? c0 : v.z;
  v.w = c == 39u ? c1 : v.w;
  v4f* dst = reinterpret_cast<v4f*>(obs) + x;
  if (POL == 1)
    __builtin_nontemporal_store(v, dst);
  else
    *dst = v;
}

// k_obs_sweep's shape variants (COUP_OBS_SPLIT = 3..7, A/B): T threads per
// block writing T x S float4 contiguous (S passes of T float4), every lane
// decoded on two threads (one observer row each, obs_row_bits_rt) into LDS
// as 4 words per row, each float then picked by row and bit.
// The split writers' float4 stores, by policy: 0 non-temporal global stores
// (shipped), 1 plain, 2 sc1 (write-through) buffer stores through the
// block's own resource -- base at the block's first float4, range its float4s
// -- 3 the same nt (measurement builds: COUP_WRITER_POL).
struct SweepDst {
  float* base;                  // the block's first float4
  __amdgpu_buffer_rsrc_t rsrc;  // POL >= 2
};
template <int POL>
__device__ __forceinline__ SweepDst sweep_dst(float* buf, int64_t x0, int64_t nf4, int64_t block_f4) {
  SweepDst d;
  d.base = buf + 4 * x0;
  if (POL >= 2) {
    const int64_t left = nf4 - x0 < block_f4 ? nf4 - x0 : block_f4;
    d.rsrc = __builtin_amdgcn_make_buffer_rsrc(d.base, (short)0, (int)(16 * left), 0x00020000);
  }
  return d;
}
template <int POL, class V>
__device__ __forceinline__ void sweep_put(const SweepDst& d, uint32_t rel_f4, const V& v) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  if constexpr (POL == 0) {
    __builtin_nontemporal_store(v, reinterpret_cast<V*>(d.base) + rel_f4);
  } else if constexpr (POL == 1) {
    reinterpret_cast<V*>(d.base)[rel_f4] = v;
  } else {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), d.rsrc, (int)(16u * rel_f4), 0,
                                           POL == 2 ? 16 : 18);
  }
}

template <int T, int S>
struct ObsSweepLds {
  static constexpr uint32_t kLanes = ((uint32_t)(T * S) + (uint32_t)kRowF4 - 1u) / (uint32_t)kRowF4 + 1u;
  alignas(16) uint32_t rows[kLanes * 8];  // lane, row: lo.x lo.y hi.x hi.y
  uint32_t coins[kLanes];
};

// Block `blk` of the writer (T threads): float4s [blk T S, (blk + 1) T S) of
// the [n][2][98] buffer from the records `state`.
template <int T, int S, int POL = 0>
__device__ __forceinline__ void obs_sweep_rows_block(const uint4* __restrict__ state, float* __restrict__ obs,
                                                     int64_t n, uint32_t blk, ObsSweepLds<T, S>& lds) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  constexpr uint32_t kLanes = ObsSweepLds<T, S>::kLanes;
  static_assert(2 * kLanes <= T, "two decoding threads per lane");
  uint32_t* rows = lds.rows;
  uint32_t* coins = lds.coins;
  const uint32_t t = threadIdx.x;
  const int64_t x0 = (int64_t)blk * (T * S);
  const int64_t o0 = x0 / kRowF4;
  if (t < 2u * kLanes && o0 + (t >> 1) < n) {
    const Lane L = unpack(state[o0 + (t >> 1)]);
    uint64_t lo, hi;
    obs_row_bits_rt(L, is_terminal(L), t & 1u, lo, hi);
    reinterpret_cast<uint4*>(rows)[t] = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi,
                                                   (uint32_t)(hi >> 32));
    if ((t & 1u) == 0u) coins[t >> 1] = L.c0 | (L.c1 << 8);
  }
  __syncthreads();
  const int64_t nf4 = n * kRowF4;
  const uint32_t rel0 = (uint32_t)(x0 - o0 * kRowF4);
  SweepDst dst{};
  if constexpr (POL != 0) dst = sweep_dst<POL>(obs, x0, nf4, T * S);
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const int64_t x = x0 + j * T + t;
    if (x >= nf4) break;
    const uint32_t rel = rel0 + (uint32_t)(j * T) + t;
    const uint32_t o = rel / (uint32_t)kRowF4, c = rel - o * (uint32_t)kRowF4;
    const uint32_t cn = coins[o];
    float f[4];
#pragma unroll
    for (uint32_t e = 0; e < 4; ++e) {
      const uint32_t k = 4u * c + e, p = k >= (uint32_t)kObsSize ? 1u : 0u, b = k - p * (uint32_t)kObsSize;
      const uint32_t w = rows[8u * o + 4u * p + (b >> 5)];
      const float bit = (float)((w >> (b & 31u)) & 1u);
      f[e] = b == 60u ? (float)(cn & 0xFFu) : (b == 61u ? (float)(cn >> 8) : bit);
    }
    v4f v;
    v.x = f[0];
    v.y = f[1];
    v.z = f[2];
    v.w = f[3];
    if constexpr (POL == 0)
      __builtin_nontemporal_store(v, reinterpret_cast<v4f*>(obs) + x);
    else
      sweep_put<POL>(dst, (uint32_t)(j * T) + t, v);
  }
}

// The nibble form of the split observation writer (round 6).  The profile
// of the rows form above (profiles/r05/c3: 176 VALU instructions per wave,
// ~88 per thread for its two float4, VALU busy ~81% over the step) says its
// store loop is VALU-heavy: four LDS word lookups, shifts, conversions and
// coin selects per float4.  Here a lane's two 98-float rows are ONE 196-bit
// string in LDS (row P1 at bits 0..97, row P2 at 98..195, as
// obs_bits_to_lds lays it out), so float4 c of the lane is nibble c of the
// string, and a 16-entry float4 table in LDS turns the nibble into the four
// floats with one ds_read_b128 (entry e of 16 covers banks 4e..4e+3: no
// conflicts).  The coins (elements 60, 61 of each row: float4 15 .x .y and
// float4 39 .z .w) are patched in from two floats per lane.  The two
// decoding threads of a lane split the string: P1's thread words 0..2 and
// the coins, P2's thread words 3..6 (word 3 also holds P1's bits 96, 97,
// which are the same in both rows: the last actions are public).
template <int T, int S>
struct ObsNibLds {
  static constexpr uint32_t kLanes = ((uint32_t)(T * S) + (uint32_t)kRowF4 - 1u) / (uint32_t)kRowF4 + 1u;
  alignas(16) float lut[16 * 4];
  alignas(16) uint32_t bits[kLanes * 8];  // words 0..6 of the lane's 196-bit string
  alignas(8) float coins[kLanes * 2];     // P1, P2 coins as floats
};

template <int T, int S>
__device__ __forceinline__ void obs_sweep_nib_block(const uint4* __restrict__ state, float* __restrict__ obs, int64_t n,
                                                    uint32_t blk, ObsNibLds<T, S>& lds) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  typedef float v2f __attribute__((ext_vector_type(2)));
  constexpr uint32_t kLanes = ObsNibLds<T, S>::kLanes;
  static_assert(2 * kLanes + 16 <= T, "two decoding threads per lane and the table's 16 threads");
  const uint32_t t = threadIdx.x;
  const int64_t x0 = (int64_t)blk * (T * S);
  const int64_t o0 = x0 / kRowF4;
  if (t < 2u * kLanes) {
    if (o0 + (t >> 1) < n) {
      const Lane L = unpack(state[o0 + (t >> 1)]);
      const uint32_t p = t & 1u;
      uint64_t lo, hi;
      obs_row_bits_rt(L, is_terminal(L), p, lo, hi);
      uint32_t* w = lds.bits + 8u * (t >> 1);
      if (p == 0u) {
        w[0] = (uint32_t)lo;
        w[1] = (uint32_t)(lo >> 32);
        w[2] = (uint32_t)hi;
        lds.coins[t] = (float)L.c0;
        lds.coins[t + 1u] = (float)L.c1;
      } else {
        w[3] = ((uint32_t)(hi >> 32) & 3u) | ((uint32_t)lo << 2);
        w[4] = (uint32_t)(lo >> 30);
        w[5] = (uint32_t)(lo >> 62) | ((uint32_t)hi << 2);
        w[6] = (uint32_t)(hi >> 30) & 0xFu;
      }
    }
  } else if (t < 2u * kLanes + 16u) {
    const uint32_t e = t - 2u * kLanes;
    reinterpret_cast<v4f*>(lds.lut)[e] = v4f{(float)(e & 1u), (float)((e >> 1) & 1u), (float)((e >> 2) & 1u),
                                             (float)(e >> 3)};
  }
  __syncthreads();
  const int64_t nf4 = n * kRowF4;
  const uint32_t rel0 = (uint32_t)(x0 - o0 * kRowF4);
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const int64_t x = x0 + j * T + t;
    if (x >= nf4) break;
    const uint32_t rel = rel0 + (uint32_t)(j * T) + t;
    const uint32_t o = rel / (uint32_t)kRowF4, c = rel - o * (uint32_t)kRowF4;
    const uint32_t nb = (lds.bits[8u * o + (c >> 3)] >> (4u * (c & 7u))) & 0xFu;
    v4f v = reinterpret_cast<const v4f*>(lds.lut)[nb];
    const v2f cn = reinterpret_cast<const v2f*>(lds.coins)[o];
    v.x = c == 15u ? cn.x : v.x;
    v.y = c == 15u ? cn.y : v.y;
    v.z = c == 39u ? cn.x : v.z;
    v.w = c == 39u ? cn.y : v.w;
    __builtin_nontemporal_store(v, reinterpret_cast<v4f*>(obs) + x);
  }
}

template <int T, int S>
__global__ __launch_bounds__(T) void k_obs_sweep_nib(const uint4* __restrict__ state, float* __restrict__ obs,
                                                     int64_t n) {
  __shared__ ObsNibLds<T, S> lds;
  obs_sweep_nib_block<T, S>(state, obs, n, blockIdx.x, lds);
}

// PRIO (measurement builds, COUP_WRITER_PRIO): the writer's waves raise
// their issue priority (s_setprio) over the rules waves beside them
template <int T, int S, int POL = 0, int PRIO = 0>
__global__ __launch_bounds__(T) void k_obs_sweep_rows(const uint4* __restrict__ state, float* __restrict__ obs,
                                                      int64_t n) {
  if constexpr (PRIO > 0) __builtin_amdgcn_s_setprio(PRIO);
  __shared__ ObsSweepLds<T, S> lds;
  obs_sweep_rows_block<T, S, POL>(state, obs, n, blockIdx.x, lds);
}

// coup_measure_step_traffic: the bytes of k_step<*, kObsWaveBitsSc1, 256,
// kInfoNone> with no rules in between -- the record loaded and stored back,
// the small outputs stored, the lane's 8 LDS words taken from its record
// instead of built by obs_bits_to_lds, then the same wave-cooperative sc1
// store loop over the same XCD-remapped lane groups.  Its duration is the
// step's store-pattern ceiling on the box that runs it.
__global__ __launch_bounds__(kThreads, 8) void k_measure_traffic(StepArgs a) {
  __shared__ uint32_t bits[kThreads * 8];
  const uint32_t grp = a.xcd_remap ? xcd_group(blockIdx.x, gridDim.x) : blockIdx.x;
  const int64_t i = (int64_t)grp * kThreads + threadIdx.x;
  const uint4 rec = i < a.n ? a.state[i] : make_uint4(0u, 0u, 0u, 0u);
  if (i < a.n) {
    a.state[i] = rec;
    if (a.actions) a.actions[i] = (int8_t)(rec.x & 15u);
    if (a.rewards) {
      a.rewards[2 * i] = (int8_t)(rec.y & 1u);
      a.rewards[2 * i + 1] = (int8_t)(rec.y & 2u);
    }
    if (a.step_type) a.step_type[i] = (uint8_t)(rec.z & 3u);
    if (a.legal) a.legal[i] = rec.w;
    if (a.cur_player) a.cur_player[i] = (int8_t)(rec.x >> 28);
  }
  reinterpret_cast<uint4*>(bits + threadIdx.x * 8u)[0] = rec;
  reinterpret_cast<uint4*>(bits + threadIdx.x * 8u)[1] = make_uint4(rec.w, rec.z, rec.y, rec.x & 0x0F0Fu);
  wave_sync();
  if (a.obs) {
    const uint32_t wl = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x & ~63u));
    const int64_t wave0 = (int64_t)grp * kThreads + wl;
    const int64_t wleft = a.n - wave0;
    const uint32_t wave_valid = wleft >= 64 ? 64u : (wleft > 0 ? (uint32_t)wleft : 0u);
    float* wave_obs = a.obs + wave0 * (2 * kObsSize);
    if (wave_valid == 64u)
      write_obs_wave_bits<2, true>(wave_obs, bits + wl * 8u, 64u);
    else if (wave_valid > 0u)
      write_obs_wave_bits<2, false>(wave_obs, bits + wl * 8u, wave_valid);
  }
}

// coup_measure_store_sweep: the split writers' store pattern with no
// decode -- block b writes float4s [b T S, (b + 1) T S) of a buffer of
// nf4 float4 in S passes of T (the grid shape of k_obs_sweep_rows<T, S> /
// k_info_sweep<T, S>), non-temporal, as they do.  Its duration is the
// writers' store ceiling on the box at hand (bench.py: roofline.
// store_ceiling_ms of the split steps).  The values stored: like the
// tensors' (0.0 with a 1.0 in one float of 32: one-hot ObservationTensor /
// InformationStateTensor fields), or with `bits` the float4's index bits in
// every float (no all-zero lines; round 5a's form, measured 3-12 % slower
// than the tensor-like data on the same buffer: HBM store time depends on
// the data, profiles/r05/sweep).
__device__ inline void sweep_store(float* dst, int64_t x, bool bits) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  v4f v;
  if (bits) {
    const float f = __int_as_float((int)(x & 0x3FFFFF));  // small denormals: a pattern, never read
    v = v4f{f, f, f, f};
  } else {
    v = v4f{(x & 7) == 0 ? 1.0f : 0.0f, 0.0f, 0.0f, 0.0f};
  }
  __builtin_nontemporal_store(v, reinterpret_cast<v4f*>(dst) + x);
}

template <int T, int S>
__global__ __launch_bounds__(T) void k_store_sweep(float* __restrict__ dst, int64_t nf4, int bits) {
  const int64_t x0 = (int64_t)blockIdx.x * (T * S) + threadIdx.x;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const int64_t x = x0 + j * T;
    if (x >= nf4) break;
    sweep_store(dst, x, bits != 0);
  }
}

#ifdef COUP_AB_VARIANTS
// measurement builds: the same stores, each float4's value the end of a
// dependent chain of `pad` integer operations (the writers' decode work
// stands between their stores; is the sweep's store rate a pacing effect?)
template <int T, int S>
__global__ __launch_bounds__(T) void k_store_sweep_paced(float* __restrict__ dst, int64_t nf4, int pad) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  const int64_t x0 = (int64_t)blockIdx.x * (T * S) + threadIdx.x;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const int64_t x = x0 + j * T;
    if (x >= nf4) break;
    uint32_t h = (uint32_t)x;
    for (int k = 0; k < pad; ++k) h = (h ^ (h >> 7)) * 0x9E3779B1u + (uint32_t)k;
    v4f v = v4f{(h & 31u) == 0u ? 1.0f : 0.0f, 0.0f, 0.0f, 0.0f};
    __builtin_nontemporal_store(v, reinterpret_cast<v4f*>(dst) + x);
  }
}

// measurement builds: the writer's structure without its decode -- the
// block's first threads load one record-sized uint4 per lane it touches (from
// `src`, 16 B per 49 float4 stored, as the observation writer reads its
// records), park them in LDS, a barrier, then the stores, each float4's value
// taken from its lane's parked word (is the writer's store rate its
// load -> LDS -> barrier -> store shape?)
template <int T, int S>
__global__ __launch_bounds__(T) void k_store_sweep_writerlike(float* __restrict__ dst, const uint4* __restrict__ src,
                                                              int64_t nf4) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  constexpr uint32_t kLanes = ((uint32_t)(T * S) + (uint32_t)kRowF4 - 1u) / (uint32_t)kRowF4 + 1u;
  __shared__ uint32_t w[kLanes];
  const uint32_t t = threadIdx.x;
  const int64_t x0 = (int64_t)blockIdx.x * (T * S);
  const int64_t o0 = x0 / kRowF4;
  if (t < kLanes && (o0 + t) * kRowF4 < nf4) w[t] = src[o0 + t].x;
  __syncthreads();
  const uint32_t rel0 = (uint32_t)(x0 - o0 * kRowF4);
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const int64_t x = x0 + j * T + t;
    if (x >= nf4) break;
    const uint32_t rel = rel0 + (uint32_t)(j * T) + t;
    const uint32_t o = rel / (uint32_t)kRowF4, c = rel - o * (uint32_t)kRowF4;
    const uint32_t b = (w[o] >> (c & 31u)) & 1u;
    v4f v = v4f{(float)b, 0.0f, 0.0f, 0.0f};
    __builtin_nontemporal_store(v, reinterpret_cast<v4f*>(dst) + x);
  }
}

// measurement builds: the same stores with a chosen share of all-zero lines:
// a 1.0 in the float4s x with x % 2^(dens - 1) == 0 (dens 1: every float4;
// 4: the tensor-like data; 6: one per 512 B), none at dens 31 (all zeros).
// The observation rows are mostly zero lines; is the HBM store rate a
// function of the share of zero lines?
template <int T, int S>
__global__ __launch_bounds__(T) void k_store_sweep_density(float* __restrict__ dst, int64_t nf4, int dens) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  const int64_t x0 = (int64_t)blockIdx.x * (T * S) + threadIdx.x;
  const int64_t mask = dens >= 31 ? -1 : ((int64_t)1 << (dens - 1)) - 1;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const int64_t x = x0 + j * T;
    if (x >= nf4) break;
    v4f v = v4f{dens < 31 && (x & mask) == 0 ? 1.0f : 0.0f, 0.0f, 0.0f, 0.0f};
    __builtin_nontemporal_store(v, reinterpret_cast<v4f*>(dst) + x);
  }
}

// measurement builds: the same stores from a resident grid, each block
// looping over chunks of T S float4 (grid-stride), without a wave launch
// per chunk
template <int T, int S>
__global__ __launch_bounds__(T) void k_store_sweep_resident(float* __restrict__ dst, int64_t nf4, int bits) {
  for (int64_t c = blockIdx.x; c * (T * S) < nf4; c += gridDim.x) {
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const int64_t x = c * (T * S) + j * T + threadIdx.x;
      if (x >= nf4) break;
      sweep_store(dst, x, bits != 0);
    }
  }
}
#endif

struct RolloutArgs {
  uint4* state;
  int64_t n;
  uint32_t seed_lo, seed_hi, env_id_base;
  int64_t steps;
  EpAcc ep;  // coup_rollout_stats: episodes / return_sum or episode_word
  int32_t* length_sum;
  uint32_t* err_count;
};

// `steps` uniform-random env steps per lane with auto-reset, state held in
// registers for the whole launch.
__global__ __launch_bounds__(kThreads) void k_rollout(RolloutArgs a) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= a.n) return;
  Lane L = unpack(a.state[i]);
  Rng rng{a.seed_lo, a.seed_hi, lane_stream_id(a.env_id_base, i), 0u, make_uint4(0, 0, 0, 0)};
  NoHistory none;
  int32_t eps = 0, ret = 0, len = 0, cur = 0;
  uint32_t errs = 0;
  for (int64_t s = 0; s < a.steps; ++s) {
    if (is_terminal(L)) L = new_episode(L.episode + 1u, rng, none);  // a terminal starting record
    resolve_chance(L, rng);  // a lane left at a chance node
    const uint32_t m = decision_mask(L);
    if (m == 0u) {
      errs += 1u;
      break;
    }
    const uint32_t err_before = L.err;
    apply_decision(L, sample_action_select(m, rng.draw(L.episode, L.move)));
    L.move += 1u;
    resolve_chance(L, rng);
    errs += (L.err && !err_before) ? 1u : 0u;
    cur += 1;
    if (is_terminal(L)) {
      eps += 1;
      ret += return0(L);
      len += cur;
      cur = 0;
      L = new_episode(L.episode + 1u, rng, none);
    }
  }
  a.state[i] = pack(L);
  a.ep.add(i, eps, ret);
  if (a.length_sum) a.length_sum[i] += len;
  if (errs) atomicAdd(a.err_count, errs);
}

// coup_step_trajectory: `steps` uniform-policy env steps per lane in ONE
// launch, the state held in registers, step t's outputs stored to slice t
// of the caller's [steps][B] buffers (stride B; coup_step_many: stride 0,
// every step overwriting the [B] outputs).  The step is k_step's own step_lane
// (effect form, no history), so the outputs, records and accumulators equal
// those of `steps` coup_step launches; what goes is the per-step record
// round trip and launch.
__global__ __launch_bounds__(kThreads) void k_step_trajectory(StepArgs a, int64_t steps, int64_t stride) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= a.n) return;
  Lane L = unpack(a.state[i]);
  NoHistory none;
  int32_t eps = 0, ret_sum = 0;
  for (int64_t t = 0; t < steps; ++t) {
    int act;
    uint32_t st;
    int32_t rew, ret = 0;
    step_lane<true, false, false>(a, i, L, act, st, rew, ret, none);
    const int64_t o = t * stride + i;
    if (a.actions) a.actions[o] = (int8_t)act;
    if (a.rewards) {
      a.rewards[2 * o] = (int8_t)rew;
      a.rewards[2 * o + 1] = (int8_t)(-rew);
    }
    if (a.step_type) a.step_type[o] = (uint8_t)st;
    if (a.legal) a.legal[o] = legal_mask(L);
    if (a.cur_player) a.cur_player[o] = (int8_t)current_player(L);
    if (st == COUP_STEP_LAST) {
      eps += 1;
      ret_sum += ret;
    }
  }
  a.state[i] = pack(L);
  a.ep.add(i, eps, ret_sum);
}

// The regrouping key of decision x at L: x itself, or refine_key
// (coup_lane.h) in -DCOUP_REFINE_KEYS builds.  Unlike the 6-player kernels,
// the 2-player ones lose with refined keys (step 27.9 -> 30.9 us, rollout
// 15.9 -> 16.4 us per 2^20-lane step, profiles/r02/ab/refined_keys_2p.log):
// the step computes them in the unsorted phase 1, and a 2-player Pass has
// no next responder to tell apart.
__device__ __forceinline__ uint32_t regroup_key(const Lane& L, uint32_t x) {
#ifdef COUP_REFINE_KEYS
  return refine_key(L, x);
#else
  (void)L;
  return x;
#endif
}

// The bare step (no observations, no history) with the block's lanes
// regrouped by decision (batches of 2^18 lanes and more: coup_regroup.h),
// the 2-player form of np::k_step_sorted.  Phase 1: each thread takes its
// lane up to the decision (step_lane's first half); the block counting-sorts
// the lanes by decision through LDS.  Phase 2: thread t applies slot t's
// decision and resolves the deals; finished lanes are listed and dealt their
// next episode by the block's first threads.  Phase 3: each thread stores
// its own lane's record and outputs, coalesced.  Same results as k_step.
template <int T>
struct SortStepLds {
  uint4 rec[T];
  uint32_t meta[T];   // slot -> owner thread | key << kO | st << kO + 5
  uint32_t out[T];    // slot -> act + 1 | st << 5 | (rew + 2) << 7 | (ret + 2) << 10 | cp << 24
  uint32_t legal[T];  // slot -> post-step legal mask
  uint32_t reset[T];  // slots whose lane auto-resets
  alignas(16) uint32_t bin[32];  // read as uint4 by bins_below
  uint32_t nreset;
};

// Block `blk` of the regrouped step: lanes [blk T, (blk + 1) T) read from
// a.state and written to rec_out (a.state itself, or the other record buffer
// of the pipelined step, coup_step_many).
template <bool UNIFORM, int T>
__device__ __forceinline__ void step_sorted_block(const StepArgs& a, uint32_t blk, uint4* rec_out,
                                                  SortStepLds<T>& lds) {
  static_assert((T & (T - 1)) == 0 && T >= 64 && T <= 1024, "power-of-two block of whole waves");
  constexpr uint32_t kO = T <= 256 ? 8u : 10u;  // owner-thread bits of s_meta
  uint4* s_rec = lds.rec;
  uint32_t* s_meta = lds.meta;
  uint32_t* s_out = lds.out;
  uint32_t* s_legal = lds.legal;
  uint32_t* s_reset = lds.reset;
  uint32_t* s_bin = lds.bin;
  uint32_t& s_nreset = lds.nreset;
  const uint32_t t = threadIdx.x;
  const int64_t base = (int64_t)blk * T;
  const int64_t i = base + t;
  const bool live = i < a.n;
  if (t < 32u) s_bin[t] = 0u;
  if (t == 0u) s_nreset = 0u;
  NoHistory none;

  // phase 1: up to the decision (step_lane)
  Lane L = initial_lane(0u);
  uint32_t key = kKeyDead, st = COUP_STEP_MID;
  const EpVal eps = ep_prefetch(a, i, live);
  if (live) {
    L = unpack(a.state[i]);
    Rng rng{a.seed_lo, a.seed_hi, lane_stream_id(a.env_id_base, i), 0u, make_uint4(0, 0, 0, 0)};
    if (!UNIFORM && (int8_t)a.actions_in[i] < 0) {
      st = COUP_STEP_SKIPPED;  // a negative action skips the lane (coup_step)
      key = kKeyReset;         // nothing to apply
    } else if (is_terminal(L)) {
      L = new_episode(L.episode + 1u, rng, none);  // step() after LAST (rl_environment.py:310-311)
      st = COUP_STEP_FIRST;
      key = kKeyReset;  // nothing left to apply
    } else {
      resolve_chance(L, rng);
      const uint32_t m = decision_mask(L);
      const uint32_t x = UNIFORM ? (m ? sample_action_select(m, rng.draw(L.episode, L.move)) : 32u)  // unsorted lanes
                                 : (uint32_t)(uint8_t)a.actions_in[i];
      if (x > 17u || ((m >> x) & 1u) == 0u || is_terminal(L)) {
        count_error(a.err_count);
        key = kKeyReset;  // rejected: nothing to apply either
      } else {
        key = regroup_key(L, x);
      }
    }
  }
  __syncthreads();
  const uint32_t rank = atomicAdd(&s_bin[key], 1u);
  __syncthreads();
  const uint32_t pos = COUP_BINS_BELOW(s_bin, key) + rank;  // keys up to kKeyChallengeLost = 25
  s_rec[pos] = pack(L);
  s_meta[pos] = t | (key << kO) | (st << (kO + 5));
  __syncthreads();

  // phase 2: thread t runs slot t's decision
  {
    const uint32_t m = s_meta[t], k = (m >> kO) & 31u;
    if (k != kKeyDead) {
      L = unpack(s_rec[t]);
      uint32_t out = ((m >> (kO + 5)) & 3u) << 5 | (2u << 7), legal = 0u;  // no action, reward 0
      bool pending = false;
      if (is_decision_key(k)) {
        Rng rng{a.seed_lo, a.seed_hi, lane_stream_id(a.env_id_base, base + (m & (T - 1u))), 0u, make_uint4(0, 0, 0, 0)};
        const uint32_t x = key_action(k);
        const uint32_t err_before = L.err;
        apply_decision_v1(L, x);  // regrouped lanes diverge little: the branch form (coup_lane.h)
        L.move += 1u;
        resolve_chance(L, rng);
        if (L.err && !err_before) count_error(a.err_count);
        const bool term = is_terminal(L);
        out = (x + 1u) | ((term ? COUP_STEP_LAST : COUP_STEP_MID) << 5) | ((uint32_t)(L.r0 + 2) << 7);
        if (a.ep.on() && term) out |= (uint32_t)(return0(L) + 2) << 10;
        pending = term && a.auto_reset != 0;
        if (pending) s_reset[atomicAdd(&s_nreset, 1u)] = t;
        s_rec[t] = pack(L);
      }
      if (!pending) {
        legal = legal_mask(L);
        out |= ((uint32_t)current_player(L) & 0xFFu) << 24;
      }
      s_out[t] = out;
      s_legal[t] = legal;
    }
  }
  __syncthreads();

  // the auto-resets (vector_env.py:62-65), packed onto the first threads
  const uint32_t nreset = s_nreset;
  for (uint32_t j = t; j < nreset; j += T) {
    const uint32_t slot = s_reset[j];
    Rng rng{a.seed_lo, a.seed_hi, lane_stream_id(a.env_id_base, base + (s_meta[slot] & (T - 1u))), 0u,
            make_uint4(0, 0, 0, 0)};
    const Lane R = new_episode(unpack(s_rec[slot]).episode + 1u, rng, none);
    s_rec[slot] = pack(R);
    s_legal[slot] = legal_mask(R);
    s_out[slot] = (s_out[slot] & 0x00FFFFFFu) | (((uint32_t)current_player(R) & 0xFFu) << 24);
  }
  __syncthreads();

  // phase 3: each thread stores its own lane
  if (!live) return;
  rec_out[i] = s_rec[pos];
  const uint32_t o = s_out[pos];
  const int32_t rew = (int32_t)((o >> 7) & 7u) - 2;
  if (a.actions) a.actions[i] = (int8_t)((int32_t)(o & 31u) - 1);
  if (a.rewards) {
    a.rewards[2 * i] = (int8_t)rew;
    a.rewards[2 * i + 1] = (int8_t)(-rew);
  }
  if (a.step_type) a.step_type[i] = (uint8_t)((o >> 5) & 3u);
  if (a.legal) a.legal[i] = s_legal[pos];
  if (a.cur_player) a.cur_player[i] = (int8_t)(o >> 24);
  ep_update(a, i, eps, (o >> 5) & 3u, (int32_t)((o >> 10) & 7u) - 2);
}

template <bool UNIFORM, int T = kThreads>
__global__ __launch_bounds__(T, 8) void k_step_sorted(StepArgs a) {
  __shared__ SortStepLds<T> lds;
  step_sorted_block<UNIFORM, T>(a, blockIdx.x, a.state, lds);
}

// The pipelined split observation step (coup_step_many; DESIGN.md section
// 5): ONE launch holds the rules blocks of step t+1 (step_sorted_block,
// uniform policy: records rules_in -> rules_out) and the observation-writer
// blocks of step t (obs_sweep_rows_block over the records rules_in, the
// post-step records of step t).  The two read the same records and write
// disjoint buffers, so no block waits for another; the rules no longer sit
// on the path between two writers.  Rules block k sits at block position
// k * stride (stride >= 1, k < rules_blocks), every other position is the
// next writer block in address order, so the rules spread over the first
// positions of the launch while the writer sweeps the buffer.  With
// rules_blocks == 0 or writer_blocks == 0 the launch is one role only (the
// pipeline's first and last launches).
struct PipeArgs {
  StepArgs a;               // the rules step; a.state = its input records (rules_in)
  uint4* rules_out;         // its output records: a.state (in place) or the other buffer
  const uint4* obs_state;   // the writer's records
  float* obs;               // [n][2][98]
  uint32_t rules_blocks, writer_blocks, stride;
};

template <int T, int S>
__global__ __launch_bounds__(T, 8) void k_step_obs_pipe(PipeArgs p) {
  __shared__ union PipeLds {
    SortStepLds<T> rules;
    ObsSweepLds<T, S> writer;
  } lds;
  const uint32_t b = blockIdx.x;
  uint32_t role_rules, idx;
  if (p.writer_blocks == 0u) {
    role_rules = 1u, idx = b;
  } else if (p.rules_blocks == 0u) {
    role_rules = 0u, idx = b;
  } else {
    const uint32_t k = b / p.stride;
    role_rules = (b == k * p.stride && k < p.rules_blocks) ? 1u : 0u;
    idx = role_rules ? k : b - min(k + 1u, p.rules_blocks);
  }
  if (role_rules)
    step_sorted_block<true, T>(p.a, idx, p.rules_out, lds.rules);
  else
    obs_sweep_rows_block<T, S>(p.obs_state, p.obs, p.a.n, idx, lds.writer);
}

// The decision key of a lane at a decision node: the uniform policy's draw,
// or kKeyDead (counted as an error) if the node has no legal decision.
__device__ __forceinline__ uint32_t draw_key(const Lane& L, Rng& rng, uint32_t& errs) {
  const uint32_t m = decision_mask(L);
  if (m == 0u) {
    errs += 1u;
    return kKeyDead;
  }
  return regroup_key(L, sample_action(m, rng.draw(L.episode, L.move)));
}

// k_rollout with the block's lanes regrouped by decision every step
// (batches of 2^18 lanes and more: coup_regroup.h).  A lane's
// next decision is drawn at the end of the step before; the block sorts its
// lanes by it through LDS and thread t plays the lane in slot t.  Finished
// lanes get kKeyReset and are dealt their next episode together, in one
// wave.  Per-lane statistics live in LDS by lane; the lanes go home at the
// end.  Same results as k_rollout.
template <int T = kThreads>
__global__ __launch_bounds__(T, 8) void k_rollout_sorted(RolloutArgs a) {
  static_assert((T & (T - 1)) == 0 && T >= 64 && T <= 1024, "power-of-two block of whole waves");
  constexpr uint32_t kO = T <= 256 ? 8u : 10u;  // lane bits of s_meta
  __shared__ uint4 s_rec[T];
  __shared__ uint32_t s_meta[T];  // slot -> lane | key << kO | decisions this episode << kO + 5
  __shared__ int32_t s_eps[T], s_ret[T], s_len[T];  // by lane
  __shared__ __attribute__((aligned(16))) uint32_t s_bin[2][32];
  const uint32_t t = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * T;
  const bool live = base + t < a.n;
  if (t < 64u) s_bin[t >> 5][t & 31u] = 0u;
  s_eps[t] = 0;
  s_ret[t] = 0;
  s_len[t] = 0;
  Rng rng{a.seed_lo, a.seed_hi, lane_stream_id(a.env_id_base, base + t), 0u, make_uint4(0, 0, 0, 0)};
  NoHistory none;
  Lane L = initial_lane(0u);
  uint32_t lane = t, cur = 0u, key = kKeyDead, errs = 0u;
  if (live) {
    L = unpack(a.state[base + t]);
    if (is_terminal(L)) L = new_episode(L.episode + 1u, rng, none);  // a terminal starting record
    resolve_chance(L, rng);  // a lane left at a chance node
    key = draw_key(L, rng, errs);
  }
  // two barriers per step, as k_trajectory_sorted (its comment)
  __syncthreads();  // the bins and by-lane counters above are initialised
  for (int64_t s = 0; s < a.steps; ++s) {
    uint32_t* bin = s_bin[s & 1];
#ifdef COUP_TRAJ_TOP_BARRIER
    __syncthreads();  // measurement builds: the third barrier of rounds 2-5
#endif
    const uint32_t rank = atomicAdd(&bin[key], 1u);
    __syncthreads();
    const uint32_t pos = COUP_BINS_BELOW(bin, key) + rank;  // keys up to kKeyChallengeLost = 25
    if (t < 32u) s_bin[(s + 1) & 1][t] = 0u;  // read for the last time in step s - 1
    s_rec[pos] = pack(L);
    s_meta[pos] = lane | (key << kO) | (cur << (kO + 5));
    __syncthreads();
    const uint32_t m = s_meta[t];
    lane = m & (T - 1u);
    key = (m >> kO) & 31u;
    cur = m >> (kO + 5);
    L = unpack(s_rec[t]);
    if (key == kKeyDead) continue;
    rng.env_id = lane_stream_id(a.env_id_base, base + lane);
    rng.blk_tag = 0u;
    if (key == kKeyReset) {
      L = new_episode(L.episode + 1u, rng, none);
      key = draw_key(L, rng, errs);
      if (key == kKeyDead) continue;
    }
    const uint32_t err_before = L.err;
    apply_decision_v1(L, key_action(key));  // regrouped: the branch form (2^20 lanes: 18.4 vs 19.4 us, profiles/r02/ab)
    L.move += 1u;
    resolve_chance(L, rng);
    errs += (L.err && !err_before) ? 1u : 0u;
    cur += 1u;
    if (is_terminal(L)) {
      s_eps[lane] += 1;
      s_ret[lane] += return0(L);
      s_len[lane] += (int32_t)cur;
      cur = 0u;
      key = kKeyReset;
    } else if (s + 1 < a.steps) {
      key = draw_key(L, rng, errs);
    }
  }
  if (key == kKeyReset) L = new_episode(L.episode + 1u, rng, none);  // finished on the last step
  __syncthreads();
  s_rec[lane] = pack(L);
  __syncthreads();
  if (live) {
    const int64_t i = base + t;
    a.state[i] = s_rec[t];
    a.ep.add(i, s_eps[t], s_ret[t]);
    if (a.length_sum) a.length_sum[i] += s_len[t];
  }
  if (errs) atomicAdd(a.err_count, errs);
}

// coup_step_trajectory for 2 players with the block's lanes regrouped by
// decision every step (batches of 2^18 lanes and more): k_rollout_sorted's
// schedule with coup_step's outputs, the 2-player form of
// np::k_trajectory_sorted (coup_nplayer.hip has the key protocol: a lane
// that finished with auto-reset keeps kKeyReset, and the next step's reset
// group deals its new episode and completes the finished step's legal mask
// and player; kKeyFirst restarts a lane that is terminal as a step starts).
// Results equal coup_step's, step for step.  Step s's outputs go to offset
// s * x.stride of the output buffers (x.stride = B: [steps][B] slices; 0:
// every step overwrites them, the last step's stay).  REC: also every
// step's post-step record (after an auto-reset) to x.rec[s * B + lane] --
// the records the observation writer of step s reads (coup_step_many's
// rules-trajectory form).  OBS: every step's
// ObservationTensor [B][2][98] written by the block itself, in address
// order, at a.obs + s * x.obs_stride floats: each thread decodes its lane's
// two rows into LDS after the step, then the block's threads store the
// block's contiguous 1024 x 784 B as float4s (k_obs_sweep_rows' decode); a
// finished lane is dealt its next episode in the same step (the post-reset
// record is the observed one), not at the next.
struct TrajOut {
  uint4* rec;          // REC: [steps][B] post-step records
  int64_t stride;      // output offset per step: B or 0
  int64_t obs_stride;  // OBS: floats per step (B * 196) or 0
};

template <int T>
struct TrajObsLds {
  alignas(16) uint32_t rows[T * 8];  // lane, row: lo.x lo.y hi.x hi.y
  uint32_t coins[T];
};
template <int T>
struct TrajNoLds {};
// STAGE: a step's outputs by lane, stored by each lane's home thread
// The output staging the shipped rules trajectories use (STAGE above): 0,
// the playing thread stores.  -DCOUP_TRAJ_OUT_STAGE=2 measurement builds
// stage by lane: equal within noise (c3 132.5 against 132.4 us per step, the
// bare trajectory at 2^20 lanes 17.54 against 17.34, call r06l), so the
// simpler form ships.
#ifndef COUP_TRAJ_OUT_STAGE
#define COUP_TRAJ_OUT_STAGE 0
#endif
constexpr int kTrajStage = COUP_TRAJ_OUT_STAGE;
constexpr int8_t kCpDeferred = -128;  // STAGE 2: legal mask, player and record stored by the reset group
template <int T>
struct TrajStageLds {
  uint4 rec[T];
  uint32_t legal[T];
  uint16_t rew[T];
  int8_t act[T];
  uint8_t st[T];
  int8_t cp[T];
};

// W: the minimum waves per SIMD the register budget is sized for (8: 64
// VGPRs; the OBS form spills at 64, W = 4 gives it 128).  STAGE: each
// step's outputs (and REC records) staged by lane in LDS and stored by the
// lanes' home threads, coalesced, instead of from the thread that played
// the lane (a wave of regrouped lanes scatters its stores over the
// block's window, one cache line per lane or so): 1 (round 5) behind a
// barrier of their own in the same step, finished lanes dealt in the same
// step as with OBS; 2 behind the next step's count barrier (the block has
// it anyway), finished lanes dealt in the reset group of the next step,
// whose direct stores of the finished step's legal mask, player and record
// follow the staged ones (the slot barrier orders them).
// FULL: every per-step output buffer (actions, rewards, step types, legal
// masks, players) is present, so no store tests its pointer.
template <int T, bool REC = false, bool OBS = false, int W = 8, int STAGE = 0, bool FULL = false>
__global__ __launch_bounds__(T, W) void k_trajectory_sorted(StepArgs a, int64_t steps, TrajOut x) {
  static_assert((T & (T - 1)) == 0 && T >= 64 && T <= 1024, "power-of-two block of whole waves");
  constexpr uint32_t kO = T <= 256 ? 8u : 10u;  // lane bits of s_meta
  __shared__ uint4 s_rec[T];
  __shared__ uint32_t s_meta[T];          // slot -> lane | key << kO
  __shared__ int32_t s_eps[T], s_ret[T];  // by lane
  __shared__ __attribute__((aligned(16))) uint32_t s_bin[2][32];
  __shared__ uint32_t s_fin;  // lanes that finished on the last step (gathered after the loop)
  __shared__ typename std::conditional<OBS, TrajObsLds<T>, TrajNoLds<T>>::type s_obs;
  __shared__ typename std::conditional<STAGE != 0, TrajStageLds<T>, TrajNoLds<T>>::type s_st;
  constexpr bool kNow = OBS || STAGE == 1;  // a finished lane's next episode dealt in the same step
  const uint32_t t = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * T;
  const bool ar = a.auto_reset != 0;
  if (t < 64u) s_bin[t >> 5][t & 31u] = 0u;
  if (t == 0u) s_fin = 0u;
  s_eps[t] = 0;
  s_ret[t] = 0;
  Rng rng{a.seed_lo, a.seed_hi, lane_stream_id(a.env_id_base, base + t), 0u, make_uint4(0, 0, 0, 0)};
  NoHistory none;
  Lane L = initial_lane(0u);
  // rw: the lane's packed record, the one value that crosses the step loop's
  // back edge (the regroup moves it through LDS).  Every path of the step
  // ends by packing its Lane into rw -- the same value its record store
  // needs -- so the unpacked Lane's ~20 fields die inside the step, and the
  // join of the step's exits copies 4 registers instead of ~23 (and packs
  // once, not again at the next step's top).
  uint4 rw = make_uint4(0u, 0u, 0u, 0u);
  uint32_t lane = t, key = kKeyDead, errs = 0u;
  // a drawn decision's sort key (-DCOUP_TRAJ_SELECT_DRAW measurement builds:
  // the loop-free policy draw)
  auto draw_decision = [&](uint32_t legal) {
#ifdef COUP_TRAJ_SELECT_DRAW
    return regroup_key(L, sample_action_select(legal, rng.draw(L.episode, L.move)));
#else
    return regroup_key(L, sample_action(legal, rng.draw(L.episode, L.move)));
#endif
  };
  // STAGE 2: step sp's staged outputs of lane base + t, from its home thread
  auto store_staged = [&](int64_t sp) {
    if constexpr (STAGE == 2) {
      const int64_t i = base + t;
      if (i < a.n) {
        const int64_t oh = sp * x.stride + i;
        if (FULL || a.actions) a.actions[oh] = s_st.act[t];
        if (FULL || a.rewards) reinterpret_cast<uint16_t*>(a.rewards)[oh] = s_st.rew[t];
        if (FULL || a.step_type) a.step_type[oh] = s_st.st[t];
        const int8_t cp = s_st.cp[t];
        if (cp != kCpDeferred) {  // else the next step's reset group stores these three, once
          if (FULL || a.legal) a.legal[oh] = s_st.legal[t];
          if (FULL || a.cur_player) a.cur_player[oh] = cp;
          if (REC) x.rec[sp * a.n + i] = s_st.rec[t];
        }
      }
    }
  };
  if (base + t < a.n) {
    rw = a.state[base + t];
    L = unpack(rw);
    if (is_terminal(L)) {
      key = kKeyFirst;
    } else {
      resolve_chance(L, rng);  // a lane left at a chance node
      const uint32_t m = decision_mask(L);
      key = m ? draw_decision(m) : kKeyDead;
      rw = pack(L);
    }
  }
  // Two barriers per step.  The bins, slots and by-lane LDS need no third at
  // the step's top: this step's bins were zeroed before the last step's
  // slot barrier, and every thread reads its slot (and finishes the last
  // step's LDS work: OBS rows, STAGE outputs) before it reaches this step's
  // count barrier, which any write of this step's slots follows.
  __syncthreads();  // the bins and by-lane counters above are initialised
  COUP_TRAJ_STAMP_DECL
  for (int64_t s = 0; s < steps; ++s) {
    uint32_t* bin = s_bin[s & 1];
#ifdef COUP_TRAJ_TOP_BARRIER
    __syncthreads();  // measurement builds: the third barrier of rounds 2-5
#endif
#ifdef COUP_TRAJ_PRIO
    __builtin_amdgcn_s_setprio(0);  // measurement builds: the step's slow waves raised below
#endif
    const uint32_t rank = atomicAdd(&bin[key], 1u);
    __syncthreads();
    COUP_TRAJ_STAMP(0);
    if constexpr (STAGE == 2)
      if (s > 0) store_staged(s - 1);  // the last step's outputs, complete behind the count barrier
    const uint32_t pos = COUP_BINS_BELOW(bin, key) + rank;  // keys up to kKeyFirst = 26
    if (t < 32u) s_bin[(s + 1) & 1][t] = 0u;  // read for the last time in step s - 1
    s_rec[pos] = rw;
    s_meta[pos] = lane | (key << kO);
    COUP_TRAJ_STAMP(1);
    __syncthreads();
    COUP_TRAJ_STAMP(2);
    const uint32_t m = s_meta[t];
    lane = m & (T - 1u);
    key = (m >> kO) & 31u;
    rw = s_rec[t];
    L = unpack(rw);
    // the step's rules: `continue` ends the lane's step (the do-while), and
    // with OBS every thread then meets the block's observation write below
    do {
    const int64_t li = base + lane;
    if (li >= a.n) continue;  // past the batch
    const int64_t o = s * x.stride + li;
    uint4* const rec_s = REC ? x.rec + s * a.n + li : nullptr;  // step s's record of the lane
    // the lane's step-s outputs: to the buffers, or (STAGE) to LDS by lane
#if defined(COUP_ABLATE_TRAJ_STORES) && COUP_ABLATE_TRAJ_STORES >= 1
    // measurement builds: the small outputs not stored (1), nor the records
    // (2) -- wrong results, the stores' share of the rules trajectory
    constexpr bool kSkipOut = true, kSkipRec = COUP_ABLATE_TRAJ_STORES >= 2;
#else
    constexpr bool kSkipOut = false, kSkipRec = false;
#endif
    auto put_act = [&](int8_t v) {
      if constexpr (kSkipOut) return;
      if constexpr (STAGE != 0) s_st.act[lane] = v;
      else if (FULL || a.actions) a.actions[o] = v;
    };
    auto put_rew = [&](uint16_t v) {
      if constexpr (kSkipOut) return;
      if constexpr (STAGE != 0) s_st.rew[lane] = v;
      else if (FULL || a.rewards) reinterpret_cast<uint16_t*>(a.rewards)[o] = v;
    };
    auto put_st = [&](uint8_t v) {
      if constexpr (kSkipOut) return;
      if constexpr (STAGE != 0) s_st.st[lane] = v;
      else if (FULL || a.step_type) a.step_type[o] = v;
    };
    auto put_legal = [&](uint32_t v) {
      if constexpr (kSkipOut) return;
      if constexpr (STAGE != 0) s_st.legal[lane] = v;
      else if (FULL || a.legal) a.legal[o] = v;
    };
    auto put_cp = [&](int8_t v) {
      if constexpr (kSkipOut) return;
      if constexpr (STAGE != 0) s_st.cp[lane] = v;
      else if (FULL || a.cur_player) a.cur_player[o] = v;
    };
    auto put_rec = [&](const Lane& R) {  // also the lane's rw
      rw = pack(R);
      if constexpr (kSkipRec) return;
      if constexpr (STAGE != 0) s_st.rec[lane] = rw;
      else if (REC) *rec_s = rw;
    };
    rng.env_id = lane_stream_id(a.env_id_base, li);
    rng.blk_tag = 0u;
    // a new episode and a live lane after resolve_chance are at decision
    // nodes: LegalActionsMask is decision_mask, the player L.M
    if (key == kKeyFirst) {  // step() after LAST (rl_environment.py:310-311)
      L = new_episode(L.episode + 1u, rng, none);
      const uint32_t legal = decision_mask(L);
      put_act(-1);
      put_rew(0u);
      put_st((uint8_t)COUP_STEP_FIRST);
      put_legal(legal);
      put_cp((int8_t)L.M);
      put_rec(L);
      key = draw_decision(legal);
      continue;
    }
    if (!kNow && key == kKeyReset) {  // finished in step s - 1 with auto-reset (vector_env.py:62-65)
#ifdef COUP_TRAJ_PRIO
      __builtin_amdgcn_s_setprio(COUP_TRAJ_PRIO);  // a wave of the reset group: the block's slowest
#endif
#ifdef COUP_ABLATE_TRAJ_RESET
      {  // measurement builds: the reset group's cost without its deals (wrong results): four distinct
         // types from the lane's id and episode, no Philox block, then the decision drawn as usual
        Lane R = initial_lane(L.episode + 1u);
        const uint32_t b0 = (uint32_t)(li + L.episode) % 5u, b1 = (b0 + 1u) % 5u, b2 = (b0 + 2u) % 5u,
                       b3 = (b0 + 3u) % 5u;
        R.h0 = (2u * min(b0, b2)) | ((2u * max(b0, b2)) << 4) | 0xFF00u;
        R.h1 = (2u * min(b1, b3)) | ((2u * max(b1, b3)) << 4) | 0xFF00u;
        R.deck -= (1u << (4u * b0)) + (1u << (4u * b1)) + (1u << (4u * b2)) + (1u << (4u * b3));
        R.qlen = 0u;
        R.qids = 0u;
        R.move = 4u;
        L = R;
      }
#else
      L = new_episode(L.episode + 1u, rng, none);
#endif
      const uint32_t legal = decision_mask(L);
      if (FULL || a.legal) a.legal[o - x.stride] = legal;
      if (FULL || a.cur_player) a.cur_player[o - x.stride] = (int8_t)L.M;
      rw = pack(L);
      if (REC) *(rec_s - a.n) = rw;  // step s - 1's record, after its auto-reset
      key = regroup_key(L, sample_action(legal, rng.draw(L.episode, L.move)));
    }
    if (key == kKeyDead) {  // no legal decision: coup_step's rejected step
      errs += 1u;
      put_act(-1);
      put_rew(0u);
      put_st((uint8_t)COUP_STEP_MID);
      put_legal(legal_mask(L));
      put_cp((int8_t)current_player(L));
      put_rec(L);
      continue;
    }
    COUP_TRAJ_STAMP(3);
    const uint32_t act = key_action(key);
    const uint32_t err_before = L.err;
    apply_decision_v1(L, act);  // regrouped: the branch form, as k_rollout_sorted
    L.move += 1u;
#ifdef COUP_TRAJ_PRIO
    if (L.qlen != 0u) __builtin_amdgcn_s_setprio(COUP_TRAJ_PRIO);  // a wave with deals
#endif
    resolve_chance(L, rng);
    errs += (L.err && !err_before) ? 1u : 0u;
    COUP_TRAJ_STAMP(4);
    const bool term = is_terminal(L);
    put_act((int8_t)act);
    put_rew((uint16_t)((uint8_t)L.r0 | ((uint8_t)(-L.r0) << 8)));
    put_st((uint8_t)(term ? COUP_STEP_LAST : COUP_STEP_MID));
    if (term) {
      s_eps[lane] += 1;
      s_ret[lane] += return0(L);
      if (ar && kNow) {  // the next episode now: the observed / staged record is the post-reset one
        L = new_episode(L.episode + 1u, rng, none);
        const uint32_t legal = decision_mask(L);
        put_legal(legal);
        put_cp((int8_t)L.M);
        put_rec(L);
        key = s + 1 < steps ? draw_decision(legal) : kKeyDead;
        continue;
      }
      if (ar) {
        key = kKeyReset;  // legal mask and player once the next episode is dealt
        rw = pack(L);
        if constexpr (STAGE == 2) s_st.cp[lane] = kCpDeferred;
        continue;
      }
      key = kKeyFirst;
      put_legal(0u);  // terminal: no legal actions, kTerminalPlayerId
      put_cp((int8_t)-4);
      put_rec(L);
      continue;
    }
    const uint32_t legal = decision_mask(L);
    put_legal(legal);
    put_cp((int8_t)L.M);
    put_rec(L);
    if (s + 1 < steps) key = draw_decision(legal);
    } while (false);
    COUP_TRAJ_STAMP(5);
    if constexpr (STAGE == 1) {  // the staged outputs from each lane's home thread, coalesced
      __syncthreads();
      const int64_t i = base + t;
      if (i < a.n) {
        const int64_t oh = s * x.stride + i;
        if (a.actions) a.actions[oh] = s_st.act[t];
        if (a.rewards) reinterpret_cast<uint16_t*>(a.rewards)[oh] = s_st.rew[t];
        if (a.step_type) a.step_type[oh] = s_st.st[t];
        if (a.legal) a.legal[oh] = s_st.legal[t];
        if (a.cur_player) a.cur_player[oh] = s_st.cp[t];
        if (REC) x.rec[s * a.n + i] = s_st.rec[t];
      }
    }
    if constexpr (OBS) {
      // the block's lanes' observation rows, by lane, then the block's
      // [lanes][2][98] floats in address order
      const int64_t nl = a.n - base < (int64_t)T ? a.n - base : (int64_t)T;
      if ((int64_t)lane < nl) {
        uint64_t lo, hi;
        const bool term = is_terminal(L);
        obs_row_bits_rt(L, term, 0u, lo, hi);
        reinterpret_cast<uint4*>(s_obs.rows)[2u * lane] =
            make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
        obs_row_bits_rt(L, term, 1u, lo, hi);
        reinterpret_cast<uint4*>(s_obs.rows)[2u * lane + 1u] =
            make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
        s_obs.coins[lane] = L.c0 | (L.c1 << 8);
      }
      __syncthreads();
      typedef float v4f __attribute__((ext_vector_type(4)));
      v4f* const dst = reinterpret_cast<v4f*>(a.obs + s * x.obs_stride + base * (2 * kObsSize));
      const uint32_t nf4 = (uint32_t)nl * (uint32_t)kRowF4;
      for (uint32_t j = t; j < nf4; j += (uint32_t)T) {
        const uint32_t ol = j / (uint32_t)kRowF4, c = j - ol * (uint32_t)kRowF4;
        const uint32_t cn = s_obs.coins[ol];
        float f[4];
#pragma unroll
        for (uint32_t e = 0; e < 4; ++e) {
          const uint32_t k = 4u * c + e, p = k >= (uint32_t)kObsSize ? 1u : 0u, b = k - p * (uint32_t)kObsSize;
          const uint32_t w = s_obs.rows[8u * ol + 4u * p + (b >> 5)];
          const float bit = (float)((w >> (b & 31u)) & 1u);
          f[e] = b == 60u ? (float)(cn & 0xFFu) : (b == 61u ? (float)(cn >> 8) : bit);
        }
        v4f v;
        v.x = f[0];
        v.y = f[1];
        v.z = f[2];
        v.w = f[3];
        __builtin_nontemporal_store(v, dst + j);
      }
    }
  }
  if constexpr (STAGE == 2) {
    __syncthreads();  // the last step's staged outputs are complete
    if (steps > 0) store_staged(steps - 1);
    __syncthreads();  // ... and stored before the finished lanes' direct stores below
  }
  // The lanes that finished on the last step are dealt their next episode
  // here, in place: after the last step's regroup they sit a few to a wave.
  // -DCOUP_TRAJ_FIN_GATHER measurement builds gather them into the block's
  // first slots through LDS so one or two waves deal them: no faster (c3
  // 132.8 against 132.5 us per step, the bare trajectory 17.00 against 16.86,
  // call r06y), the extra barrier costing what the waves save.
  auto deal_finished = [&](uint32_t fl, uint4 w) {  // lane fl finished the last step; returns its record
    const int64_t li = base + fl;
    rng.env_id = lane_stream_id(a.env_id_base, li);
    rng.blk_tag = 0u;
    const Lane R = new_episode(unpack(w).episode + 1u, rng, none);
    const int64_t o = (steps - 1) * x.stride + li;
    if (FULL || a.legal) a.legal[o] = decision_mask(R);
    if (FULL || a.cur_player) a.cur_player[o] = (int8_t)R.M;
    const uint4 rr = pack(R);
    if (REC) x.rec[(steps - 1) * a.n + li] = rr;
    return rr;
  };
#ifdef COUP_TRAJ_FIN_GATHER
  constexpr bool kFinSorted = !kNow;
#else
  constexpr bool kFinSorted = false;
#endif
  const bool fin = !kNow && key == kKeyReset && base + lane < a.n;
  if (!kFinSorted && fin) rw = deal_finished(lane, rw);
  __syncthreads();  // every thread has read its last slot
  s_rec[lane] = rw;
  if constexpr (kFinSorted) {
    if (fin) s_meta[atomicAdd(&s_fin, 1u)] = lane;
    __syncthreads();
    if (t < s_fin) {
      const uint32_t fl = s_meta[t];
      s_rec[fl] = deal_finished(fl, s_rec[fl]);
    }
  }
  __syncthreads();
  if (base + t < a.n) {
    const int64_t i = base + t;
    a.state[i] = s_rec[t];
    a.ep.add(i, s_eps[t], s_ret[t]);
  }
  if (errs) atomicAdd(a.err_count, errs);
  COUP_TRAJ_STAMP_FLUSH(g_traj_phases, steps);
}

// NewInitialState / reset of selected lanes.  mode 0: fresh env (episode 0);
// mode 1: next episode.  deal: resolve the four initial deals.
__global__ __launch_bounds__(kThreads) void k_reset(uint4* state, int64_t n, const uint8_t* mask, int mode, int deal,
                                                  uint32_t seed_lo, uint32_t seed_hi, uint32_t env_id_base,
                                                  uint8_t* hist) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  if (mask && mask[i] == 0) return;
  const uint32_t ep = mode == 0 ? 0u : unpack(state[i]).episode + 1u;
  Lane L = initial_lane(ep);
  L.err = (mode != 0 && L.episode == 0u) ? 1u : 0u;  // counter wrap (coup_lane.h kEpisodeMask)
  if (deal) {
    Rng rng{seed_lo, seed_hi, lane_stream_id(env_id_base, i), 0u, make_uint4(0, 0, 0, 0)};
    if (hist) {
      RegHistory rec;
      resolve_chance(L, rng, rec);
      rec.flush(hist + i * kHist);
    } else {
      resolve_chance(L, rng);
    }
  }
  state[i] = pack(L);
}

// State::ApplyAction per lane (decision or chance outcome); the entry goes
// to the lane's history bytes when the env keeps a history.
// UNCHECKED: COUP_FLAG_UNCHECKED (unchecked_decision); a compile-time
// switch, as step_lane's.
template <bool UNCHECKED>
__global__ __launch_bounds__(kThreads) void k_apply(uint4* state, int64_t n, const int8_t* actions,
                                                  uint8_t* hist, uint32_t* err_count) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const int x = actions[i];
  if (x < 0) return;
  Lane L = unpack(state[i]);
  const uint32_t err_before = L.err;
  // the history entry is formed before and stored after the transition, so
  // the byte store stays out of the inlined rules
  const uint32_t idx = L.move;
  const uint32_t entry = is_chance(L) ? hist_deal((uint32_t)x, L.qids & 1u) : hist_decision((uint32_t)x, L.M);
  if constexpr (UNCHECKED) {  // the reference's unchecked ApplyAction
    uint4 w;
    if (!unchecked_decision(pack(L), (uint32_t)x, &w)) {
      count_error(err_count);
      return;
    }
    L = unpack(w);
  } else {
    NoHistory none;
    if (!apply_action(L, (uint32_t)x, none)) {
      count_error(err_count);
      return;
    }
  }
  if (L.err && !err_before) count_error(err_count);
  state[i] = pack(L);
  if (hist && idx < (uint32_t)kHist) hist[i * kHist + idx] = (uint8_t)entry;
}

struct QueryArgs {
  const uint4* state;
  int64_t n;
  uint32_t* legal;
  int8_t* cur_player;
  uint8_t* terminal;
  int8_t* rewards;
  int8_t* returns;
  float* obs;
  const uint8_t* hist;
  float* info;
};

// Per-lane accessors of the current state (State::LegalActionsMask,
// CurrentPlayer, IsTerminal, Rewards, Returns, ObservationTensor,
// InformationStateTensor).  No early exit: the tensor writers are
// wave-cooperative.
template <bool OBS, bool INFO>
__global__ __launch_bounds__(kThreads) void k_query(QueryArgs a) {
  __shared__ uint32_t bits[OBS ? kThreads * 8 : 1];
  __shared__ uint8_t hist[INFO ? kThreads * kHist : 16];
  __shared__ __attribute__((aligned(16))) uint32_t pre[INFO ? kThreads * kPreWords : 1];
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  const bool active = i < a.n;
  const uint32_t wl = threadIdx.x & ~63u;
  const int64_t wave0 = (int64_t)blockIdx.x * kThreads + wl;
  const int64_t wleft = a.n - wave0;
  const uint32_t wave_valid = wleft >= 64 ? 64u : (wleft > 0 ? (uint32_t)wleft : 0u);
  const Lane L = active ? unpack(a.state[i]) : initial_lane(0);
  if (active) {
    if (a.legal) a.legal[i] = legal_mask(L);
    if (a.cur_player) a.cur_player[i] = (int8_t)current_player(L);
    if (a.terminal) a.terminal[i] = is_terminal(L) ? 1 : 0;
    if (a.rewards) {
      a.rewards[2 * i] = (int8_t)L.r0;
      a.rewards[2 * i + 1] = (int8_t)(-L.r0);
    }
    if (a.returns) {
      const int32_t r = return0(L);
      a.returns[2 * i] = (int8_t)r;
      a.returns[2 * i + 1] = (int8_t)(-r);
    }
  }
  if (OBS) {
    obs_bits_to_lds(L, bits + threadIdx.x * 8u);
    wave_sync();
    if (wave_valid) write_obs_wave_bits<1, false>(a.obs + wave0 * (2 * kObsSize), bits + wl * 8u, wave_valid);
  }
  if (INFO) {
    if (wave_valid)
      wave_hist_copy<true>(const_cast<uint8_t*>(a.hist) + wave0 * kHist, hist + wl * kHist, wave_valid);
    info_prefix_to_lds(L, pre + threadIdx.x * kPreWords);
    wave_sync();
    if (wave_valid)
      write_info_wave<kInfoStorePolicy>(a.info + wave0 * (2 * kInfoSize), hist + wl * kHist, pre + wl * kPreWords,
                                        wave_valid);
  }
}


// InformationStateTensor of a few lanes, one thread per float4 (lane-major
// [n][2][2492] output).  The wave-cooperative writer gives each wave 1246
// store instructions for its 64 lanes; at one lane (the per-game State
// facade, rl_environment) that is one wave storing alone, ~150 us.  Here the
// 1246 float4 of a lane are spread over 1246 threads; each thread decodes its
// lane's record and history bytes itself (L2-resident).
// reqs (coup_slot_ops): output row l is the lane of request l.

__global__ __launch_bounds__(kThreads) void k_info_elems(const uint4* __restrict__ state,
                                                        const uint8_t* __restrict__ hist, int64_t n,
                                                        float* __restrict__ info,
                                                        const coup_slot_req* __restrict__ reqs = nullptr) {
  const int64_t g = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (g >= n * kInfoF4) return;
  const int64_t row = g / kInfoF4;
  const uint32_t c = (uint32_t)(g - row * kInfoF4);
  const int64_t lane = reqs ? reqs[row].lane : row;
  uint32_t pre[kPreWords];
  info_prefix_to_lds(unpack(state[lane]), pre);
  reinterpret_cast<float4*>(info)[g] = info_f4(pre, hist + lane * kHist, c);
}

// The split InformationStateTensor step (COUP_INFO_SPLIT; coup_step): the
// rules step maintaining the history without tensors, then this kernel
// writes [B][2][2492] in address order, T x S float4 per block (S passes of
// T float4).  The <= 2-3 lanes a block touches get their prefix words
// (info_prefix_to_lds) and 96 history bytes into LDS from its first
// threads; every thread then decodes its float4s with info_f4, the fused
// writer's decode (coup_tensor.h), and stores them non-temporally.
template <int T, int S, int POL = 0>
__global__ __launch_bounds__(T) void k_info_sweep(const uint4* __restrict__ state, const uint8_t* __restrict__ hist,
                                                  float* __restrict__ info, int64_t n) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  constexpr uint32_t kLanes = ((uint32_t)(T * S) + (uint32_t)kInfoF4 - 1u) / (uint32_t)kInfoF4 + 1u;
  constexpr uint32_t kHistU4 = (uint32_t)kHist / 16u;  // 6
  static_assert(kLanes * kHistU4 <= (uint32_t)T, "one history uint4 per thread");
  __shared__ __attribute__((aligned(16))) uint32_t pre[kLanes * kPreWords];
  __shared__ uint4 h4[kLanes * kHistU4];
  const uint32_t t = threadIdx.x;
  const int64_t x0 = (int64_t)blockIdx.x * (T * S);
  const int64_t o0 = x0 / kInfoF4;
  if (t < 2u * kLanes && o0 + (t >> 1) < n) {
    // info_prefix_to_lds's words, one observer row per thread, 32-bit
    // values only (its uint2 form gave wrong prefix bits in this kernel)
    const Lane L = unpack(state[o0 + (t >> 1)]);
    const uint32_t p = t & 1u;
    uint64_t lo, hi;
    obs_row_bits_rt(L, is_terminal(L), p, lo, hi);
    const uint64_t m62 = (1ull << 62) - 1ull;  // drop the observation's last_action bits
    uint32_t* w = pre + kPreWords * (t >> 1);
    w[2u * p] = (uint32_t)lo;
    w[2u * p + 1u] = (uint32_t)((lo & m62) >> 32);
    if (p == 0u) {
      w[4] = L.c0 | (L.c1 << 8) | (L.move << 16);
      w[5] = 0u;
    }
  }
  if (t < kLanes * kHistU4 && o0 + t / kHistU4 < n)
    h4[t] = reinterpret_cast<const uint4*>(hist)[o0 * kHistU4 + t];
  __syncthreads();
  const int64_t nf4 = n * kInfoF4;
  const uint32_t rel0 = (uint32_t)(x0 - o0 * kInfoF4);
  const uint8_t* hb = reinterpret_cast<const uint8_t*>(h4);
  SweepDst dst{};
  if constexpr (POL != 0) dst = sweep_dst<POL>(info, x0, nf4, T * S);
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const int64_t x = x0 + j * T + t;
    if (x >= nf4) break;
    const uint32_t rel = rel0 + (uint32_t)(j * T) + t;
    const uint32_t o = rel / (uint32_t)kInfoF4, c = rel - o * (uint32_t)kInfoF4;
    const float4 f = info_f4(pre + kPreWords * o, hb + kHist * o, c);
    v4f v;
    v.x = f.x;
    v.y = f.y;
    v.z = f.z;
    v.w = f.w;
    if constexpr (POL == 0)
      __builtin_nontemporal_store(v, reinterpret_cast<v4f*>(info) + x);
    else
      sweep_put<POL>(dst, (uint32_t)(j * T) + t, v);
  }
}

// ObservationTensor rows of the requests' lanes (coup_step_host with
// COUP_HOST_ACTIVE): row l = lane reqs[l].lane, one thread per row.
__global__ __launch_bounds__(kThreads) void k_obs_lanes(const uint4* __restrict__ state,
                                                       const coup_slot_req* __restrict__ reqs, int64_t m,
                                                       float* __restrict__ obs) {
  const int64_t l = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (l >= m) return;
  write_obs_pair(obs + l * (2 * kObsSize), unpack(state[reqs[l].lane]));
}

// Batches up to this size take k_info_elems for the InformationStateTensor
// of coup_query (and coup_slot_op always does).
constexpr int64_t kInfoElemsMaxBatch = 1024;

// Lane-pool op of the per-game State facade (coup_slot_op): one wave, one
// lane.  Thread 0 runs the transition and the accessors; the history bytes
// go through LDS so the copy, the new entry and the write-back are ordered
// by wave barriers.  The
// observation writer is the batched one with n_valid = 1, so its LDS array
// keeps the 64-lane shape (the writer indexes it before its predicate); the
// InformationStateTensor is left to k_info_elems.
static_assert(sizeof(coup_slot_result) == 128, "coup_slot_result layout");

struct SlotArgs {
  uint4* dst_state;
  uint8_t* dst_hist;
  const uint4* src_state;  // null: no copy
  const uint8_t* src_hist;
  int action;              // < 0: none
  int init;
  int store;               // write the lane back (copy, init or action)
  coup_slot_result* out;   // null: no result
  float* obs;              // [2][98] or null
  uint32_t* done = nullptr;  // k_slot: completion flag in mapped host memory (null: none)
  uint32_t seq = 0;          // the value k_slot stores there once its results are visible
  uint32_t mode = 0;         // kSlotReset | kSlotDeal | kSlotUnchecked (COUP_SLOT_RESET / _DEAL / _UNCHECKED)
  uint32_t seed_lo = 0, seed_hi = 0, env_id = 0;  // the lane's sampling-contract stream (kSlotDeal)
};
constexpr uint32_t kSlotReset = 1u, kSlotDeal = 2u, kSlotUnchecked = 4u;

// -DCOUP_SLOT_INLINE (investigation builds only): the
// two pieces below inlined into the wave-uniform k_slot, the form the ROCm 7.2
// compiler miscompiles at -O2/-O3 (word 3 of the record after a next_move
// transition; reproducer: tools/slot_inline_repro.hip, k_min<0>).  The
// product must never be built this way.
#if defined(COUP_SLOT_INLINE) && !defined(COUP_INVESTIGATION_BUILD)
#error "COUP_SLOT_INLINE reproduces a miscompile (DESIGN.md section 12); only tools/slot_inline_repro.hip may set it"
#endif
#ifdef COUP_SLOT_INLINE
#define COUP_SLOT_FN __forceinline__
#else
#define COUP_SLOT_FN __noinline__
#endif

// Out-of-line pieces of k_slot.  slot_transition applies action x to the
// packed record `w` (State::ApplyAction with its legality check, or without
// it when `unchecked`: apply_action_unchecked, coup_lane.h) into *out and
// returns bit 0 = accepted without a new error, bit 1 = history entry to
// store, bits 8..15 its index, bits 16..23 the entry byte.
// The checked transition (State::ApplyAction with its legality check) on
// record w into *out; false, *out not written, for an illegal action or one
// that raises a new error.  Each transition form lives in a function of its
// own (this one, unchecked_decision): one body combining both behind a
// run-time flag is the shape the section-12 defect strikes (step_lane).
__device__ COUP_SLOT_FN uint32_t checked_transition(uint4 w, uint32_t x, uint4* out) {
  Lane L = unpack(w);
  const uint32_t err_before = L.err;
  NoHistory none;
  if (!apply_action(L, x, none) || (L.err && !err_before)) return 0u;
  *out = pack(L);
  return 1u;
}

// Whether the reference's DoApplyAction accepts decision x on record w while
// its result leaves the packed record's fields (apply_action_unchecked's
// `representable` test, coup_lane.h): for a rejected unchecked action, tells
// a known parity gap from a reference raise (coup_slot_result.
// unrepresentable).  Out of line, on the rejection path only.
__device__ COUP_SLOT_FN uint32_t unrepresentable_decision(uint4 w, uint32_t x) {
  Lane R = unpack(w);
  if (x > 17u || is_terminal(R) || R.err || is_chance(R)) return 0u;
  return (ref_decision(R, x) && !representable(R)) ? 1u : 0u;
}

// Returns bit 2 = rejected but unrepresentable (unrepresentable_decision).
__device__ COUP_SLOT_FN uint32_t slot_transition(uint4 w, uint32_t x, uint32_t unchecked, uint4* out) {
  const Lane L = unpack(w);
  const uint32_t idx = L.move;
  const uint32_t entry = is_chance(L) ? hist_deal(x, L.qids & 1u) : hist_decision(x, L.M);
  uint4 r;
  if (!(unchecked ? unchecked_decision(w, x, &r) : checked_transition(w, x, &r))) {
    // a rejected action (or one the reference's DoApplyAction raises on)
    // leaves the record untouched
    *out = w;
    return (unchecked && unrepresentable_decision(w, x)) ? 4u : 0u;
  }
  *out = r;
  const uint32_t store = idx < (uint32_t)kHist ? 2u : 0u;
  return 1u | store | (idx << 8) | (entry << 16);
}

// The rl_environment ops of a lane (COUP_SLOT_RESET / COUP_SLOT_DEAL):
// kSlotReset starts the lane's next episode (coup_reset's k_reset, mode 1);
// then decision x (< 18; 0xFF: none) is applied with its legality check
// (without it under kSlotUnchecked); then kSlotDeal resolves the pending chance deals under the sampling
// contract, as rl_environment samples chance until a decision node
// (rl_environment.py:369-382).  Every entry goes to the history bytes `hist`
// (LDS).  Returns bit 0 = accepted without a new error, bit 2 = rejected but
// unrepresentable (as slot_transition); an illegal x leaves the record
// untouched.  Out of line, like slot_transition.
__device__ COUP_SLOT_FN uint32_t slot_step(uint4 w, uint32_t x, uint32_t mode, uint32_t seed_lo, uint32_t seed_hi,
                                           uint32_t env_id, uint4* out, uint8_t* hist) {
  Lane L = unpack(w);
  if (mode & kSlotReset) {
    L = initial_lane(L.episode + 1u);
    L.err = L.episode == 0u ? 1u : 0u;  // counter wrap (coup_lane.h kEpisodeMask)
  }
  RegHistory rec;
  if (x != 0xFFu && x >= 18u) {
    // an int8 action id outside 0..17: DoApplyAction raises (coup.cc:493,
    // :806) -- rejected, the lane untouched, the reset included
    *out = w;
    return 0u;
  }
  if (x < 18u) {
    const uint32_t idx = L.move;
    const uint32_t entry = is_chance(L) ? hist_deal(x, L.qids & 1u) : hist_decision(x, L.M);
    uint4 r;
    if (!((mode & kSlotUnchecked) ? unchecked_decision(pack(L), x, &r) : checked_transition(pack(L), x, &r))) {
      *out = w;  // untouched, the reset included
      return ((mode & kSlotUnchecked) && unrepresentable_decision(pack(L), x)) ? 4u : 0u;
    }
    L = unpack(r);
    rec.record(idx, entry);
  }
  if (mode & kSlotDeal) {
    Rng rng{seed_lo, seed_hi, env_id, 0u, make_uint4(0, 0, 0, 0)};
    resolve_chance(L, rng, rec);
  }
  rec.flush(hist);
  *out = pack(L);
  return 1u;
}

// ok: bit 0 accepted, bit 2 rejected but unrepresentable (slot_transition).
__device__ COUP_SLOT_FN void slot_result(uint4 w, uint32_t ok, coup_slot_result* out) {
  const Lane L = unpack(w);
  out->record[0] = w.x;
  out->record[1] = w.y;
  out->record[2] = w.z;
  out->record[3] = w.w;
  out->legal_mask = legal_mask(L);
  out->cur_player = (int8_t)current_player(L);
  out->terminal = is_terminal(L) ? 1 : 0;
  out->ok = (uint8_t)(ok & 1u);
  out->unrepresentable = (uint8_t)((ok >> 2) & 1u);
  out->rewards[0] = (int8_t)L.r0;
  out->rewards[1] = (int8_t)(-L.r0);
  const int32_t r0 = return0(L);
  out->returns[0] = (int8_t)r0;
  out->returns[1] = (int8_t)(-r0);
}

// One State op on one lane by one wave (k_slot: one op per launch;
// k_slot_batch: one op per block).  hist / bits: the wave's LDS.
template <bool OBS>
__device__ __forceinline__ void slot_op(const SlotArgs& a, uint8_t* __restrict__ hist, uint32_t* __restrict__ bits) {
  const uint32_t t = threadIdx.x;
  const uint4* rs = a.src_state ? a.src_state : a.dst_state;
  const uint8_t* hs = a.src_state ? a.src_hist : a.dst_hist;
  // the record's load goes out with the history's, one memory round trip
  // for both (thread 0 used to issue it after the barrier)
  uint4 rec = make_uint4(0u, 0u, 0u, 0u);
  if (t == 0u) rec = a.init ? pack(initial_lane(0u)) : *rs;
  if (t < 6u)
    reinterpret_cast<uint4*>(hist)[t] =
        a.init ? make_uint4(~0u, ~0u, ~0u, ~0u) : reinterpret_cast<const uint4*>(hs)[t];
  wave_sync();
  // Thread 0 runs the rules (the other threads only copy history bytes and
  // store tensors).  The transition and the accessors are out-of-line
  // functions (VGPR arguments), so they compile as the per-lane code of the
  // batched kernels: inlined here on the wave-uniform record, the compiler
  // moved them to scalar code and produced wrong records.
  Lane L = initial_lane(0u);
  if (t == 0u) {
    uint32_t ok = 1u;
    if (a.mode & (kSlotReset | kSlotDeal)) {
      ok = slot_step(rec, a.action >= 0 ? (uint32_t)a.action : 0xFFu, a.mode, a.seed_lo, a.seed_hi, a.env_id, &rec,
                     hist);
    } else if (a.action >= 0) {
      const uint32_t r = slot_transition(rec, (uint32_t)a.action, a.mode & kSlotUnchecked, &rec);
      ok = r & 5u;
      if (r & 2u) hist[(r >> 8) & 0xFFu] = (uint8_t)(r >> 16);
    }
    if (a.store) *a.dst_state = rec;
    if (a.out) slot_result(rec, ok, a.out);
    L = unpack(rec);
  }
  wave_sync();
  if (t < 6u) {
    const uint4 h = reinterpret_cast<const uint4*>(hist)[t];
    if (a.store) reinterpret_cast<uint4*>(a.dst_hist)[t] = h;
    if (a.out) reinterpret_cast<uint4*>(a.out->history)[t] = h;
  }
  if (OBS) {
    if (t == 0u) obs_bits_to_lds(L, bits);
    wave_sync();
    write_obs_wave_bits<0, false>(a.obs, bits, 1u);
  }
}

template <bool OBS>
__global__ __launch_bounds__(64) void k_slot(SlotArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t hist[kHist];
  __shared__ __attribute__((aligned(16))) uint32_t bits[OBS ? 64 * 8 : 1];
  slot_op<OBS>(a, hist, bits);
  if (a.done) {
    // the host polls this flag instead of synchronising the stream: every
    // thread's result / tensor stores reach system scope first
    __threadfence_system();
    wave_sync();
    if (threadIdx.x == 0u) __hip_atomic_store(a.done, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// coup_slot_ops: n independent State ops in one launch, block b = request b
// (a Deep CFR node's children, a frontier of states).  The requests sit in
// mapped pinned host memory next to the results; the host has checked that
// no destination lane repeats or is another request's source.
struct SlotBatchArgs {
  uint4* state;               // the env's records / histories (destinations)
  uint8_t* hist;
  const uint4* src_state;     // the source env's (copies)
  const uint8_t* src_hist;
  const coup_slot_req* reqs;  // [n]
  coup_slot_result* out;      // [n] or null
  float* obs;                 // [n][2][98] or null
  uint32_t* done = nullptr;   // [n] completion flags in mapped host memory (null: none)
  uint32_t seq = 0;           // the value block b stores in done[b] once its results are visible
};

template <bool OBS>
__global__ __launch_bounds__(64) void k_slot_batch(SlotBatchArgs b) {
  __shared__ __attribute__((aligned(16))) uint8_t hist[kHist];
  __shared__ __attribute__((aligned(16))) uint32_t bits[OBS ? 64 * 8 : 1];
  const coup_slot_req r = b.reqs[blockIdx.x];
  SlotArgs a;
  a.dst_state = b.state + r.lane;
  a.dst_hist = b.hist + r.lane * kHist;
  a.src_state = r.src_lane >= 0 ? b.src_state + r.src_lane : nullptr;
  a.src_hist = r.src_lane >= 0 ? b.src_hist + r.src_lane * kHist : nullptr;
  a.action = r.action;
  a.init = (r.flags & COUP_SLOT_INIT) ? 1 : 0;
  a.mode = (r.flags & COUP_SLOT_UNCHECKED) ? kSlotUnchecked : 0u;
  a.store = (r.src_lane >= 0 || a.init || r.action >= 0) ? 1 : 0;
  a.out = b.out ? b.out + blockIdx.x : nullptr;
  a.obs = OBS ? b.obs + (size_t)blockIdx.x * (2 * kObsSize) : nullptr;
  slot_op<OBS>(a, hist, bits);
  if (b.done) {  // as k_slot: the host polls the flags instead of synchronising
    __threadfence_system();
    wave_sync();
    if (threadIdx.x == 0u) __hip_atomic_store(b.done + blockIdx.x, b.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ------------------------------------------------- device-resident op server
// coup_server: ONE resident wave serves the per-game
// State ops of the envs attached to it, so an answered op costs a host write
// the wave sees, the op itself and a device->host write -- no kernel launch,
// no queue.  Requests sit in a ring of kSrvRing slots in mapped, coherent
// pinned host memory, one 64-byte host cache line each.  The wave polls the
// next slot by reading the WHOLE line -- 16 lanes x 4 bytes, one request per
// 32-byte half -- so the request arrives with the poll that finds it, one
// host round trip instead of two.  Each half carries the slot's sequence
// number, written after the fields of its half (x86 stores become visible in
// program order, and a half is read as one snapshot), so a match of both
// means every field is current.  The poll and the stop word are loaded
// together (one round trip per pass), then s_sleep.  The op runs with no
// fences (server_op: sc1 / sc0 sc1 accesses), its stores are drained, and
// the number goes to ctl.served.  Requests are served in order.  Exit: when
// the host stores the wave's epoch in ctl.stop (after the pending requests),
// or after idle_ticks (s_memrealtime, 100 MHz) with no request -- a host that
// stops calling, or dies, never leaves a spinning wave; the next op
// relaunches it.
constexpr uint32_t kSrvRing = 64;

struct SrvReq {        // one ring slot (host memory), 64 bytes = one host cache line
  // first half (32 bytes)
  uint64_t dst_state;  // uint4*  (device)
  uint64_t dst_hist;   // uint8_t* (device)
  uint64_t src_state;  // 0: no copy
  uint32_t op;         // action (int8) [7:0] | init [8] | result [9] | obs [10] | info [11]
  uint32_t seq_a;      // the sequence number, stored after the half's fields
  // second half
  uint64_t src_hist;
  uint32_t seed_lo, seed_hi, env_id;  // the lane's sampling-contract stream (deal / reset)
  uint32_t check;      // srv_check of the fields and the number (a torn read of the line is polled again)
  uint32_t pad;
  uint32_t seq_b;      // stored last of all
};
static_assert(sizeof(SrvReq) == 64, "SrvReq layout");

// Checksum of a request's words 0-6 and 8-12 and its number.  The wave reads
// the line as 16 separate 4-byte system-scope loads; neither the HIP memory
// model nor PCIe ordering promises that they see one snapshot of it, so
// matching numbers alone could pair a new number with an older request's
// fields.  A mismatch is treated as "not posted yet".  Host and device use
// this one function (scalar arithmetic on the device: the words are
// readlane'd into SGPRs anyway).
__host__ __device__ __forceinline__ uint32_t srv_check(const uint32_t* w, uint32_t seq) {
  uint32_t h = seq * 0x9E3779B1u + 0x7F4A7C15u;
  for (int k = 0; k < 13; ++k) {
    if (k == 7) continue;
    h = (h ^ w[k]) * 0x85EBCA6Bu;
    h ^= h >> 13;
  }
  return h;
}
constexpr uint32_t kSrvInit = 1u << 8, kSrvResult = 1u << 9, kSrvObs = 1u << 10, kSrvInfo = 1u << 11;
constexpr uint32_t kSrvModeShift = 12;  // [14:12]: kSlotReset | kSlotDeal | kSlotUnchecked

struct SrvCtl {        // host memory, one word per 128-byte line
  uint32_t served;     // last sequence number served (the wave writes)
  uint32_t pad0[31];
  uint32_t stop;       // the host writes the epoch of the wave to stop
  uint32_t pad1[31];
};

struct ServerArgs {
  SrvReq* ring;        // device addresses of the mapped host memory
  SrvCtl* ctl;
  uint8_t* result;     // coup_slot_result, then obs [2][98], then info [2][2492] floats (mapped host)
  uint32_t epoch;      // this launch's epoch (never 0)
  uint64_t idle_ticks; // exit after this many 100 MHz ticks without a request
};

template <class T>
__device__ __forceinline__ T srv_ld(const T* p) {  // host-written word: vector load, system scope
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// 16-byte accesses through a buffer resource with explicit cache bits:
// aux 16 = sc1 (device scope: past the CU's L1; stores write through),
// 17 = sc0 sc1 (system scope).
template <int AUX>
__device__ __forceinline__ uint4 ld16(uint64_t base, uint32_t off) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(base), (short)0, (int)(off + 16u), 0x00020000);
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const v4u v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, AUX);
  return make_uint4(v.x, v.y, v.z, v.w);
}
template <int AUX>
__device__ __forceinline__ void st16(uint64_t base, uint32_t off, uint4 x) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(base), (short)0, (int)(off + 16u), 0x00020000);
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  __builtin_amdgcn_raw_buffer_store_b128(v4u{x.x, x.y, x.z, x.w}, r, (int)off, 0, AUX);
}
constexpr int kAuxDevice = 16, kAuxSystem = 17;

// One coup_slot_op on one lane by the server's wave: slot_op's steps with
// the server's cache policy, which needs no fence: the lanes and histories
// are read with sc1 loads (past this CU's L1: kernels on other XCDs may have
// written them) and written with sc1 stores (write-through, so later kernels
// on any XCD read them); the result and tensors go to host memory with
// sc0 sc1 stores (system write-through -- plain stores would sit in this
// XCD's L2 until a buffer_wbl2).  rs / hs: the lane (and history) to start
// from; the transition and the accessors run out of line on thread 0
// (slot_transition / slot_result, as in k_slot: DESIGN.md section 12).
__device__ __forceinline__ void server_op(uint64_t rs, uint64_t hs, uint64_t dst_state, uint64_t dst_hist,
                                          int32_t action, int32_t init, bool store, uint64_t out, uint64_t obs,
                                          uint64_t info, uint32_t mode, uint32_t seed_lo, uint32_t seed_hi,
                                          uint32_t env_id, uint8_t* hist, uint32_t* bits, uint32_t* pre,
                                          coup_slot_result* res) {
  const uint32_t t = threadIdx.x;
  // the record's load goes out with the history's: one round trip for both
  uint4 rec = make_uint4(0u, 0u, 0u, 0u);
  if (t == 0u) rec = init ? pack(initial_lane(0u)) : ld16<kAuxDevice>(rs, 0u);
  if (t < 6u)
    reinterpret_cast<uint4*>(hist)[t] = init ? make_uint4(~0u, ~0u, ~0u, ~0u) : ld16<kAuxDevice>(hs, 16u * t);
  wave_sync();
  Lane L = initial_lane(0u);
  if (t == 0u) {
    uint32_t ok = 1u;
    if (mode & (kSlotReset | kSlotDeal)) {
      ok = slot_step(rec, action >= 0 ? (uint32_t)action : 0xFFu, mode, seed_lo, seed_hi, env_id, &rec, hist);
    } else if (action >= 0) {
      const uint32_t r = slot_transition(rec, (uint32_t)action, mode & kSlotUnchecked, &rec);
      ok = r & 5u;
      if (r & 2u) hist[(r >> 8) & 0xFFu] = (uint8_t)(r >> 16);
    }
    if (store) st16<kAuxDevice>(dst_state, 0u, rec);
    if (out) slot_result(rec, ok, res);
    L = unpack(rec);
    if (info) info_prefix_to_lds(L, pre);
  }
  wave_sync();
  if (t < 6u) {
    const uint4 h = reinterpret_cast<const uint4*>(hist)[t];
    if (store) st16<kAuxDevice>(dst_hist, 16u * t, h);
    if (out) reinterpret_cast<uint4*>(res->history)[t] = h;
  }
  wave_sync();
  if (out && t < 8u) st16<kAuxSystem>(out, 16u * t, reinterpret_cast<const uint4*>(res)[t]);
  if (obs) {
    if (t == 0u) obs_bits_to_lds(L, bits);
    wave_sync();
    write_obs_wave_bits<3, false>(reinterpret_cast<float*>(obs), bits, 1u);
  }
  if (info) {
    // 19,936 bytes: plain stores, which the L2 gathers into whole lines, then
    // one system-scope write-back, WAITED FOR by an asm wait after the fence
    // (a builtin wait in front of it let the compiler drop the one after the
    // buffer_wbl2: cdna_hip_programming.md G16 pitfall 12).  16-byte
    // write-through stores straight to host memory took ~100 us here.
    for (uint32_t c = t; c < (uint32_t)kInfoF4; c += 64u)
      reinterpret_cast<float4*>(info)[c] = info_f4(pre, hist, c);
    __threadfence_system();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

__global__ __launch_bounds__(64) void k_server(ServerArgs s) {
  __shared__ __attribute__((aligned(16))) uint8_t hist[kHist];
  __shared__ __attribute__((aligned(16))) uint32_t bits[64 * 8];
  __shared__ __attribute__((aligned(16))) uint32_t pre[kPreWords];
  __shared__ __attribute__((aligned(16))) coup_slot_result res;
  const uint32_t t = threadIdx.x;
  // the first unserved request, read here rather than passed at launch: a
  // wave queued behind another on the server stream (two relaunches) starts
  // after the earlier one has left, so it never serves a request again
  uint32_t next = (uint32_t)__builtin_amdgcn_readfirstlane((int)srv_ld(&s.ctl->served)) + 1u;
  uint64_t idle0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    // the slot's 16 words (lanes 0..15) and the stop word in one round trip
    const uint32_t* line = reinterpret_cast<const uint32_t*>(s.ring + (next & (kSrvRing - 1u)));
    const uint32_t w = srv_ld(line + (t & 15u));
    const uint32_t stop = srv_ld(&s.ctl->stop);
    const uint32_t seq_a = (uint32_t)__builtin_amdgcn_readlane((int)w, 7);
    const uint32_t seq_b = (uint32_t)__builtin_amdgcn_readlane((int)w, 15);
    if (seq_a != next || seq_b != next) {
      if ((uint32_t)__builtin_amdgcn_readfirstlane((int)stop) == s.epoch) break;
      if (__builtin_amdgcn_s_memrealtime() - idle0 > s.idle_ticks) break;
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    auto word = [&](int k) { return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)w, k); };
    {
      uint32_t fw[13];
#pragma unroll
      for (int k = 0; k < 13; ++k) fw[k] = (uint32_t)word(k);
      if (srv_check(fw, next) != (uint32_t)word(13)) {  // a torn snapshot of the line: poll again
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
    }
    const uint64_t dst_state = word(0) | (word(1) << 32), dst_hist = word(2) | (word(3) << 32);
    const uint64_t src_state = word(4) | (word(5) << 32), src_hist = word(8) | (word(9) << 32);
    const uint32_t op = (uint32_t)word(6);
    const int32_t action = (int32_t)(int8_t)(op & 0xFFu);
    const int32_t init = (op & kSrvInit) ? 1 : 0;
    const uint64_t res_base = reinterpret_cast<uint64_t>(s.result);
    const uint64_t out = (op & kSrvResult) ? res_base : 0u;
    const uint64_t obs = (op & kSrvObs) ? res_base + sizeof(coup_slot_result) : 0u;
    const uint64_t info =
        (op & kSrvInfo) ? res_base + sizeof(coup_slot_result) + ((op & kSrvObs) ? 2u * kObsSize * 4u : 0u) : 0u;
    const uint32_t mode = (op >> kSrvModeShift) & 7u;
    const bool store = src_state != 0u || init != 0 || action >= 0 || (mode & (kSlotReset | kSlotDeal)) != 0u;
    server_op(src_state ? src_state : dst_state, src_state ? src_hist : dst_hist, dst_state, dst_hist, action, init,
              store, out, obs, info, mode, (uint32_t)word(10), (uint32_t)word(11), (uint32_t)word(12), hist, bits, pre,
              &res);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();
    if (t == 0u) __hip_atomic_store(&s.ctl->served, next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    next += 1u;
    idle0 = __builtin_amdgcn_s_memrealtime();
  }
}
}  // namespace coup

// ====================================================================== C ABI

// coup_slot_op's mapped scratch: result, obs, info state, then (64-byte
// aligned) the completion flag k_slot raises
constexpr size_t kSlotFlagOffset =
    (sizeof(coup_slot_result) + 2u * COUP_OBS_SIZE * sizeof(float) + 2u * COUP_INFO_STATE_SIZE * sizeof(float) + 63u) &
    ~size_t(63);

struct coup_env {
  int64_t batch;
  uint64_t seed;
  uint32_t env_id_base;
  int flags;
  int players;
  bool generic;   // N-player engine (coup_nplayer.hip): num_players != 2 or COUP_FLAG_GENERIC
  uint4* state;   // [B] records, or the N-player engine's two [B] planes back to back
  uint8_t* hist;  // [B][96] when COUP_FLAG_HISTORY
  uint32_t* err_count;
  hipStream_t stream;
  uint8_t* slot_scratch;  // coup_slot_op results: pinned host memory the kernels write directly (lazy)
  uint8_t* slot_scratch_dev;  // its device address
  uint32_t slot_seq;          // last completion value k_slot stored in the scratch's flag word
  uint8_t* batch_scratch;     // coup_slot_ops: requests + results (mapped pinned, grown on demand)
  uint8_t* batch_scratch_dev;
  size_t batch_cap;
  uint32_t batch_seq;         // last completion value k_slot_batch stored in the batch flags
  uint8_t* host_scratch;      // coup_step_host: input actions + outputs (mapped pinned, grown on demand)
  uint8_t* host_scratch_dev;
  size_t host_cap;
  uint8_t* host_stage;        // coup_step_host with info_state: device staging of the outputs (grown on demand)
  size_t host_stage_cap;
  bool batch_pending;         // an asynchronous coup_slot_ops may still read the requests
  coup_server* server;        // coup_attach_server: coup_slot_op goes through this resident wave
  bool dirty;                 // work enqueued on `stream` since its last synchronisation
  hipEvent_t stream_event;    // coup_set_stream: orders a new stream after the old one's pending work
  uint4* traj_rec;            // 2 players: [traj_cap][B] records of coup_step_many's rules trajectories
                              // ([2][traj_cap][B] once the overlapped form's resources exist)
  int64_t traj_cap;           // steps per rules-trajectory launch the buffer holds (COUP_TRAJ_CHUNK at create)
  uint4* state2;              // = traj_rec: the second record buffer of the merged pipelined step
  hipStream_t aux;            // kManyOverlap (measurement builds): the rules trajectories' stream
  hipEvent_t ev_fork, ev_rules[2], ev_writers[2];  // kManyOverlap's fork / chunk events
  coup::Knobs knobs;          // dispatch knobs, read once at coup_create (coup_knobs.h)
};

// coup_server (coup_mi355x.h; kernel coup::k_server).  The ring, the control
// words and the result area live in one mapped, coherent pinned host block.
struct coup_server {
  hipStream_t stream = nullptr;   // its own non-blocking stream: the wave never holds up other work
  uint8_t* host = nullptr;        // ring [kSrvRing] | ctl | result (coup_slot_result + obs + info)
  uint8_t* host_dev = nullptr;
  coup::SrvReq* ring = nullptr;   // host views
  coup::SrvCtl* ctl = nullptr;
  uint8_t* result = nullptr;
  uint8_t* result_dev = nullptr;
  uint32_t posted = 0;            // last sequence number posted
  uint32_t epoch = 0;             // epoch of the last launch
  bool running = false;           // a wave was launched and may still be serving
  uint64_t idle_us = 2000;
  std::chrono::steady_clock::time_point last_post;
  uint64_t requests = 0, launches = 0;
  // Every host path that reads or writes the fields above, the ring or the
  // result area holds this: a post, its wait and the copy of its result are
  // one critical section (the result area is shared by all requests), and
  // drains / stops from other threads (coup_destroy of another env, a stream
  // op on a served env) cannot interleave with them.  Recursive: srv_post
  // waits and stops inside its own section.
  std::recursive_mutex mu;
};

namespace {
// Live op servers: coup_destroy stops their waves before it frees memory
// (hipFree / hipHostFree synchronise the device, which would otherwise wait
// out a resident wave's idle time).
std::mutex g_servers_mu;
std::vector<coup_server*> g_servers;
}  // namespace

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define COUP_TRY(expr)   \
  do {                   \
    const int _r = (expr); \
    if (_r != COUP_OK) return _r; \
  } while (0)
#define COUP_HIP_TRY(expr)                                                                    \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess) return fail(COUP_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

#define COUP_CHECK_ENV(env) \
  if (!(env)) return fail(COUP_E_INVALID, "null coup_env")

// The fused step's observation writer: mode 9 (coup::ObsMode), the
// wave-cooperative bitmap with sc1 (write-through) buffer stores -- 1-4 us
// per 2^20-lane step faster than the non-temporal stores of mode 4 in every
// same-process A/B (tools/ab_step.py).  Measurement
// builds take COUP_OBS_MODE=1..9 (the modes at coup::ObsMode).
int obs_mode(const coup::Knobs& k) {
#ifdef COUP_AB_VARIANTS
  return k.obs_mode;
#else
  (void)k;
  return coup::kObsWaveBitsSc1;
#endif
}

// The observation step of n lanes: the split form from kObsSplitMinLanes
// lanes -- the rules step without tensors plus k_obs_sweep_rows<512, 2>
// (variant 11) in address order, 140.6-146.1 us against 160.2-161.5 for the
// fused step per 2^20-lane step in the same process (calls r04r / r04s,
// profiles/r04/ab/c3_obs_split_shapes_*.jsonl) -- else the fused
// k_step<*, kObsWaveBitsSc1> (0; the split form lost below 2^20 lanes).
// COUP_OBS_SPLIT forces 0 or 11 (measurement builds: the rejected writer
// shapes 1..17).
constexpr int64_t kObsSplitMinLanes = int64_t(1) << 20;
int obs_split(const coup::Knobs& k, int64_t n) {
  const int v = k.obs_split >= 0 ? k.obs_split : (n >= kObsSplitMinLanes ? coup::kObsSplitDefault : 0);
#ifdef COUP_AB_VARIANTS
  return v;
#else
  return v == 0 ? 0 : coup::kObsSplitDefault;
#endif
}
// The InformationStateTensor step: from 2^18 lanes (c3i's batch) the
// history-keeping rules step plus k_info_sweep<1024, 2> (variant 3), 837 us
// against 978 us for the fused step in the same process (call r04v,
// profiles/r04/ab/c3i_info_split_shapes.jsonl); else the fused
// k_step<*, kObsNone, 256, kInfoWrite> (0).  COUP_INFO_SPLIT forces 0 or 3
// (measurement builds: the shapes 1..5).
constexpr int64_t kInfoSplitMinLanes = int64_t(1) << 18;
int info_split(const coup::Knobs& k, int64_t n) {
  const int v = k.info_split >= 0 ? k.info_split : (n >= kInfoSplitMinLanes ? coup::kInfoSplitDefault : 0);
#ifdef COUP_AB_VARIANTS
  return v;
#else
  return v == 0 ? 0 : coup::kInfoSplitDefault;
#endif
}

#ifdef COUP_AB_VARIANTS
// The merged pipelined form of the split step (coup_step_many kManyPipe,
// coup::k_step_obs_pipe): the shipped split kernels' bodies, the regrouped
// 512-lane rules step and the 512 x 2 writer (variant 11).
constexpr int kPipeT = 512, kPipeS = 2;
#endif

// The XCD-aware block -> lane group mapping of the fused step (coup::
// xcd_group; measurement builds: COUP_XCD_REMAP=0 turns it off).
int xcd_remap(const coup::Knobs& k) {
#ifdef COUP_AB_VARIANTS
  return k.xcd_remap;
#else
  (void)k;
  return 1;
#endif
}

// Threads per lane of the rules-bound in-place step (coup::k_step_group):
// 1, the Philox blocks computed ahead with ILP, 7.08 -> 6.95 us per c2 step;
// 2 and 4 threads per lane measured 7.59 and 9.74 us
// (profiles/r04/ab/c2_tpl.jsonl) and k_step (0) 7.08: measurement builds
// take COUP_STEP_TPL=0/2/4.
int step_tpl(const coup::Knobs& k) {
#ifdef COUP_AB_VARIANTS
  return k.step_tpl;
#else
  (void)k;
  return 1;
#endif
}

// Blocks of the step kernel: one per group of T lanes.
unsigned step_grid(int64_t groups, int) { return (unsigned)(groups > 0 ? groups : 1); }

template <bool U, int M, int T, int I, bool UC = false>
void launch_step(const coup_env*, const coup::StepArgs& a, int64_t n, unsigned dyn_lds, hipStream_t s) {
  const int64_t groups = (n + T - 1) / T;
  coup::note_launch("coup::k_step<{b}, {}, {}, {}, {b}>", U, M, T, I, UC);
  coup::k_step<U, M, T, I, UC><<<step_grid(groups, T), T, dyn_lds, s>>>(a);
}
unsigned grid_for(int64_t n) { return (unsigned)((n + coup::kThreads - 1) / coup::kThreads); }

coup::np::Env np_env(const coup_env* env) {
  coup::np::Env e;
  e.sa = env->state;
  e.sb = env->state + env->batch;
  e.n = env->batch;
  e.players = env->players;
  e.seed_lo = (uint32_t)env->seed;
  e.seed_hi = (uint32_t)(env->seed >> 32);
  e.env_id_base = env->env_id_base;
  e.auto_reset = (env->flags & COUP_FLAG_AUTO_RESET) ? 1 : 0;
  e.err_count = env->err_count;
  e.stream = env->stream;
  e.knobs = env->knobs;
  return e;
}

int np_result(hipError_t e, const char* what) {
  if (e != hipSuccess) return fail(COUP_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
  return COUP_OK;
}

int launching(coup_env* env);

int launch_reset(coup_env* env, const uint8_t* mask, int mode, int deal) {
  if (env->batch == 0) return COUP_OK;
  COUP_TRY(launching(env));
  if (env->generic) return np_result(coup::np::launch_reset(np_env(env), mask, mode, deal), "reset");
  coup::k_reset<<<grid_for(env->batch), coup::kThreads, 0, env->stream>>>(
      env->state, env->batch, mask, mode, deal, (uint32_t)env->seed, (uint32_t)(env->seed >> 32), env->env_id_base,
      env->hist);
  COUP_HIP_TRY(hipGetLastError());
  return COUP_OK;
}

size_t align16(size_t n) { return (n + 15u) & ~size_t(15); }

// ---- coup_server host side
constexpr size_t kSrvCtlOff = coup::kSrvRing * sizeof(coup::SrvReq);  // 4 KiB: the ring starts the (page-aligned) block
constexpr size_t kSrvResultOff = kSrvCtlOff + sizeof(coup::SrvCtl);
constexpr size_t kSrvBytes = kSrvResultOff + sizeof(coup_slot_result) + 2u * COUP_OBS_SIZE * sizeof(float) +
                             2u * COUP_INFO_STATE_SIZE * sizeof(float);

uint32_t srv_served(const coup_server* s) { return __atomic_load_n(&s->ctl->served, __ATOMIC_ACQUIRE); }

// (Re)launch the resident wave, serving from the first unserved request.
int srv_launch(coup_server* s) {
  coup::ServerArgs a;
  a.ring = reinterpret_cast<coup::SrvReq*>(s->host_dev);
  a.ctl = reinterpret_cast<coup::SrvCtl*>(s->host_dev + kSrvCtlOff);
  a.result = s->result_dev;
  s->epoch = s->epoch + 1u == 0u ? 1u : s->epoch + 1u;
  a.epoch = s->epoch;
  a.idle_ticks = s->idle_us * 100u;  // s_memrealtime: 100 MHz
  coup::k_server<<<1, 64, 0, s->stream>>>(a);
  COUP_HIP_TRY(hipGetLastError());
  s->running = true;
  s->launches += 1u;
  return COUP_OK;
}

// Stop the wave after the requests already posted (it serves them first)
// and wait for it to leave.
int srv_stop(coup_server* s) {
  std::lock_guard<std::recursive_mutex> lk(s->mu);
  if (!s->running) return COUP_OK;
  __atomic_store_n(&s->ctl->stop, s->epoch, __ATOMIC_RELEASE);
  s->running = false;
  COUP_HIP_TRY(hipStreamSynchronize(s->stream));
  return COUP_OK;
}

// Wait until request `seq` has been served.  A wave that left (idle timeout
// racing a post, or an error) is found by querying its stream every ~50 us of
// waiting; the pending requests are still in the ring, so a relaunch from
// the first unserved one completes them.
int srv_wait(coup_server* s, uint32_t seq) {
  std::lock_guard<std::recursive_mutex> lk(s->mu);
  auto t0 = std::chrono::steady_clock::now(), tq = t0;
  for (uint32_t k = 1; (int32_t)(srv_served(s) - seq) < 0; ++k) {
    __builtin_ia32_pause();
    if ((k & 255u) != 0u) continue;
    const auto now = std::chrono::steady_clock::now();
    if (now - tq < std::chrono::microseconds(50)) continue;
    tq = now;
    const hipError_t q = hipStreamQuery(s->stream);
    if (q == hipSuccess) {  // no wave: serve the rest with a new one
      if ((int32_t)(srv_served(s) - seq) >= 0) break;
      COUP_TRY(srv_launch(s));
      t0 = now;
    } else if (q != hipErrorNotReady) {
      return fail(COUP_E_HIP, std::string("coup_server: ") + hipGetErrorString(q));
    } else if (now - t0 > std::chrono::seconds(10)) {
      return fail(COUP_E_HIP, "coup_server: a request was not served within 10 s");
    }
  }
  return COUP_OK;
}

// Before work on `env` that does not go through its server: the server's
// pending requests (they may write env's lanes) are served first.
int srv_drain(const coup_env* env) {
  if (!env || !env->server) return COUP_OK;
  coup_server* s = env->server;
  std::lock_guard<std::recursive_mutex> lk(s->mu);
  if (s->running && s->posted != srv_served(s)) COUP_TRY(srv_wait(s, s->posted));
  return COUP_OK;
}

// Every entry point that enqueues work on an env's stream calls this first.
int launching(coup_env* env) {
  COUP_TRY(srv_drain(env));
  env->dirty = true;
  return COUP_OK;
}

// Post one request (a filled SrvReq without its number) and return its number.
int srv_post(coup_server* s, const coup::SrvReq& req, uint32_t* seq_out) {
  std::lock_guard<std::recursive_mutex> lk(s->mu);
  const auto now = std::chrono::steady_clock::now();
  if (s->posted >= 0xFFFFFF00u) {
    // the numbers would wrap: drain, stop, restart the count
    COUP_TRY(srv_wait(s, s->posted));
    COUP_TRY(srv_stop(s));
    for (uint32_t k = 0; k < coup::kSrvRing; ++k) s->ring[k].seq_a = s->ring[k].seq_b = 0u;
    __atomic_store_n(&s->ctl->served, 0u, __ATOMIC_RELEASE);
    s->posted = 0u;
  }
  // The wave leaves after idle_us without a request.  A post within idle_us
  // / 2 of the last one is seen long before that; otherwise the wave may be
  // leaving: stop it for sure and start a new one (cheap next to the idle time).
  if (s->running && now - s->last_post > std::chrono::microseconds(s->idle_us / 2u)) COUP_TRY(srv_stop(s));
  if (!s->running) COUP_TRY(srv_launch(s));
  const uint32_t seq = s->posted + 1u;
  if (seq - srv_served(s) >= coup::kSrvRing) COUP_TRY(srv_wait(s, seq - coup::kSrvRing));  // ring full
  coup::SrvReq* q = s->ring + (seq & (coup::kSrvRing - 1u));
  coup::SrvReq r = req;
  r.check = coup::srv_check(reinterpret_cast<const uint32_t*>(&r), seq);
  // each half's fields, then its number, the second half's last (x86 makes
  // stores visible in program order; the compiler keeps them in order here)
  std::memcpy(q, &r, offsetof(coup::SrvReq, seq_a));
  std::memcpy(&q->src_hist, &r.src_hist, offsetof(coup::SrvReq, seq_b) - offsetof(coup::SrvReq, src_hist));
  __atomic_store_n(&q->seq_a, seq, __ATOMIC_RELEASE);
  __atomic_store_n(&q->seq_b, seq, __ATOMIC_RELEASE);
  s->posted = seq;
  s->last_post = now;
  s->requests += 1u;
  *seq_out = seq;
  return COUP_OK;
}

}  // namespace

// coup_step_host's output layout (coup_mi355x.h): section offsets of legal
// mask, player, step type, rewards, actions and the tensors; returns the size.
extern "C" size_t coup_step_host_layout(int64_t batch, int num_players, int want, size_t* off) {
  const size_t B = (size_t)(batch > 0 ? batch : 0), P = (size_t)num_players;
  size_t o = 0;
  off[0] = o;
  o += align16(4 * B);
  off[1] = o;
  o += align16(B);
  off[2] = o;
  o += align16(B);
  off[3] = o;
  o += align16(B * P);
  off[4] = o;
  o += align16(B);
  off[5] = o;
  if (want & COUP_HOST_OBS) o += align16(B * P * 49u * P * 4u);
  if (want & COUP_HOST_INFO) o += B * 2u * COUP_INFO_STATE_SIZE * 4u;
  return o;
}

namespace {

void release(coup_env* env) {
  (void)hipFree(env->state);
  (void)hipFree(env->traj_rec);
  if (env->aux) {
    (void)hipStreamDestroy(env->aux);
    for (hipEvent_t ev : {env->ev_fork, env->ev_rules[0], env->ev_rules[1], env->ev_writers[0], env->ev_writers[1]})
      if (ev) (void)hipEventDestroy(ev);
  }
  (void)hipFree(env->hist);
  (void)hipFree(env->err_count);
  if (env->slot_scratch) (void)hipHostFree(env->slot_scratch);
  if (env->batch_scratch) (void)hipHostFree(env->batch_scratch);
  if (env->host_scratch) (void)hipHostFree(env->host_scratch);
  if (env->host_stage) (void)hipFree(env->host_stage);
  delete env;
}

#ifdef COUP_AB_VARIANTS
// coup_step_many's overlapped form (kManyOverlap, measurement builds): a
// second stream for the rules trajectories, the fork / chunk events, and the
// record buffer grown to two chunks.  Created at coup_create where the form
// applies, else at the first call that needs them outside a graph capture.
int overlap_resources(coup_env* env) {
  if (env->aux) return COUP_OK;
  const size_t lanes = (size_t)(env->batch > 0 ? env->batch : 1);
  uint4* rec = nullptr;
  hipError_t e = hipMalloc(&rec, lanes * sizeof(uint4) * 2 * env->traj_cap);
  if (e != hipSuccess) return fail(COUP_E_HIP, std::string("coup_step_many: ") + hipGetErrorString(e));
  hipStream_t aux = nullptr;
  hipEvent_t ev[5] = {};
  e = hipStreamCreateWithFlags(&aux, hipStreamNonBlocking);
  for (int i = 0; i < 5 && e == hipSuccess; ++i) e = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming);
  if (e != hipSuccess) {
    for (hipEvent_t x : ev)
      if (x) (void)hipEventDestroy(x);
    if (aux) (void)hipStreamDestroy(aux);
    (void)hipFree(rec);
    return fail(COUP_E_HIP, std::string("coup_step_many: ") + hipGetErrorString(e));
  }
  (void)hipFree(env->traj_rec);  // synchronises: no launch in flight still reads it
  env->traj_rec = env->state2 = rec;
  env->aux = aux;
  env->ev_fork = ev[0];
  env->ev_rules[0] = ev[1];
  env->ev_rules[1] = ev[2];
  env->ev_writers[0] = ev[3];
  env->ev_writers[1] = ev[4];
  return COUP_OK;
}
#endif

}  // namespace

extern "C" {

int coup_abi_version(void) { return COUP_ABI_VERSION; }

const char* coup_last_error(void) { return g_last_error.c_str(); }

int coup_create(int64_t batch, uint64_t seed, uint32_t env_id_base, int flags, coup_env** out) {
  return coup_create_ex(batch, seed, env_id_base, flags, COUP_NUM_PLAYERS, out);
}

int coup_create_ex(int64_t batch, uint64_t seed, uint32_t env_id_base, int flags, int num_players, coup_env** out) {
  if (!out) return fail(COUP_E_INVALID, "coup_create: out is null");
  *out = nullptr;
  if (batch < 0 || batch > (int64_t(1) << 32)) return fail(COUP_E_INVALID, "coup_create: batch out of range");
  if ((int64_t)env_id_base + batch > (int64_t(1) << 32))
    return fail(COUP_E_INVALID, "coup_create: env_id_base + batch exceeds 2^32 (lanes would share random streams)");
  if (flags & ~(COUP_FLAG_AUTO_RESET | COUP_FLAG_HISTORY | COUP_FLAG_GENERIC | COUP_FLAG_UNCHECKED))
    return fail(COUP_E_INVALID, "coup_create: unknown flags");
  if (num_players < 2 || num_players > COUP_MAX_PLAYERS)
    return fail(COUP_E_INVALID, "coup_create: num_players must be 2..6");
  const bool generic = num_players != 2 || (flags & COUP_FLAG_GENERIC);
  if (generic && (flags & COUP_FLAG_UNCHECKED))
    return fail(COUP_E_INVALID, "coup_create: COUP_FLAG_UNCHECKED is the 2-player engine's (the reference's rules)");
  if (generic && (flags & COUP_FLAG_HISTORY))
    return fail(COUP_E_INVALID, "coup_create: COUP_FLAG_HISTORY is 2-player only (no N-player InformationStateTensor)");
  coup_env* env = new coup_env();
  env->batch = batch;
  env->seed = seed;
  env->env_id_base = env_id_base;
  env->flags = flags;
  env->players = num_players;
  env->generic = generic;
  env->stream = nullptr;
  env->state = nullptr;
  env->hist = nullptr;
  env->err_count = nullptr;
  env->slot_scratch = nullptr;
  env->slot_scratch_dev = nullptr;
  env->slot_seq = 0;
  env->batch_scratch = nullptr;
  env->batch_scratch_dev = nullptr;
  env->batch_cap = 0;
  env->batch_pending = false;
  env->batch_seq = 0;
  env->host_scratch = nullptr;
  env->host_scratch_dev = nullptr;
  env->host_cap = 0;
  env->host_stage = nullptr;
  env->host_stage_cap = 0;
  env->server = nullptr;
  env->dirty = false;
  env->stream_event = nullptr;
  env->traj_rec = nullptr;
  env->traj_cap = 0;
  env->state2 = nullptr;
  env->aux = nullptr;
  env->ev_fork = env->ev_rules[0] = env->ev_rules[1] = env->ev_writers[0] = env->ev_writers[1] = nullptr;
  env->knobs = coup::read_knobs();
  const size_t lanes = (size_t)(batch > 0 ? batch : 1);
  hipError_t e = hipMalloc(&env->state, lanes * sizeof(uint4) * (generic ? 2 : 1));
  // coup_step_many's per-step record buffer (allocated here: coup_step_many
  // may be captured into a HIP graph, where no allocation may happen), only
  // where its rules-trajectory split step can apply -- the split observation
  // step's batch (or COUP_OBS_SPLIT forced), no history, COUP_PIPE not 0
  // (every 2-player env paid traj_chunk x 16 B per lane for it);
  // many_form runs one coup_step per step where it is missing
  if (e == hipSuccess && !generic && !(flags & COUP_FLAG_HISTORY) && env->knobs.pipe != coup::kManySerial &&
      obs_split(env->knobs, batch) != 0) {
    env->traj_cap = env->knobs.traj_chunk;
    e = hipMalloc(&env->traj_rec, lanes * sizeof(uint4) * env->traj_cap);
    env->state2 = env->traj_rec;
  }
  if (e == hipSuccess) e = hipMalloc(&env->err_count, sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemset(env->err_count, 0, sizeof(uint32_t));
  if (e == hipSuccess && (flags & COUP_FLAG_HISTORY)) {
    e = hipMalloc(&env->hist, lanes * COUP_HISTORY_BYTES);
    if (e == hipSuccess) e = hipMemset(env->hist, 0xFF, lanes * COUP_HISTORY_BYTES);
  }
  if (e != hipSuccess) {
    release(env);
    return fail(COUP_E_HIP, std::string("coup_create: ") + hipGetErrorString(e));
  }
  int rc = launch_reset(env, nullptr, /*mode=*/0, /*deal=*/1);
  if (rc == COUP_OK) {
    e = hipStreamSynchronize(env->stream);
    if (e != hipSuccess) rc = fail(COUP_E_HIP, std::string("coup_create: ") + hipGetErrorString(e));
  }
#ifdef COUP_AB_VARIANTS
  // the overlapped coup_step_many's stream, events and second record
  // buffer, where the split observation step applies (a graph capture cannot
  // create them later)
  if (rc == COUP_OK && !generic && (batch >= kObsSplitMinLanes || env->knobs.obs_split > 0) &&
      env->knobs.pipe == coup::kManyOverlap)
    rc = overlap_resources(env);
#endif
  if (rc != COUP_OK) {
    release(env);
    return rc;
  }
  *out = env;
  return COUP_OK;
}

int coup_destroy(coup_env* env) {
  COUP_CHECK_ENV(env);
  (void)srv_drain(env);
  hipError_t e1 = hipStreamSynchronize(env->stream);
  // release() frees device and pinned memory, which synchronises the whole
  // device: a resident op-server wave (this env's or any other's) would hold
  // that up for its idle time.  Stop every wave first; the next op on a
  // server starts a new one.
  {
    std::lock_guard<std::mutex> g(g_servers_mu);
    for (coup_server* s : g_servers) (void)srv_stop(s);
  }
  if (env->stream_event) (void)hipEventDestroy(env->stream_event);
  release(env);
  if (e1 != hipSuccess) return fail(COUP_E_HIP, "coup_destroy: HIP error while releasing the env");
  return COUP_OK;
}

int coup_reload_knobs(coup_env* env) {
  COUP_CHECK_ENV(env);
  env->knobs = coup::read_knobs();
  return COUP_OK;
}

int coup_set_stream(coup_env* env, void* hip_stream) {
  COUP_CHECK_ENV(env);
  const hipStream_t next = (hipStream_t)hip_stream;
  if (env->dirty && next != env->stream) {
    // work still queued on the old stream: the new one waits for it, so
    // everything later on env (and the op server's dirty check, which
    // synchronises env->stream) is ordered after it
    if (!env->stream_event) COUP_HIP_TRY(hipEventCreateWithFlags(&env->stream_event, hipEventDisableTiming));
    COUP_HIP_TRY(hipEventRecord(env->stream_event, env->stream));
    COUP_HIP_TRY(hipStreamWaitEvent(next, env->stream_event, 0));
  }
  env->stream = next;
  return COUP_OK;
}

int64_t coup_batch(const coup_env* env) { return env ? env->batch : -1; }

int coup_num_players(const coup_env* env) { return env ? env->players : -1; }

int coup_state_bytes(const coup_env* env) { return env ? (env->generic ? 32 : COUP_STATE_BYTES) : -1; }

int coup_reset(coup_env* env, const uint8_t* lane_mask) {
  COUP_CHECK_ENV(env);
  return launch_reset(env, lane_mask, /*mode=*/1, /*deal=*/1);
}

int coup_new_initial_state(coup_env* env, const uint8_t* lane_mask) {
  COUP_CHECK_ENV(env);
  return launch_reset(env, lane_mask, /*mode=*/1, /*deal=*/0);
}

#ifdef COUP_WAVE_TRACE
static uint64_t* g_trace = nullptr;
// measurement builds only: per-wave timestamps of the following coup_step
// launches go to `buf` ([blocks * waves per block][5] u64), or nowhere (null)
int coup_debug_set_trace(uint64_t* buf) {
  g_trace = buf;
  return COUP_OK;
}
// the buffer for the N-player step (coup_nplayer.hip)
uint64_t* coup_debug_get_trace() { return g_trace; }
#endif

int coup_step(coup_env* env, const int8_t* actions, const coup_step_outputs* out) {
  COUP_CHECK_ENV(env);
  if (env->batch == 0) return COUP_OK;
  {
    // the accumulators are checked here for both engines (the N-player
    // launch relies on it)
    coup::EpAcc ep;
    if (const char* why = coup::ep_acc_of(out, ep)) return fail(COUP_E_INVALID, std::string("coup_step: ") + why);
  }
  COUP_TRY(launching(env));
  if (env->generic) {
    if (out && out->info_state) return fail(COUP_E_INVALID, "coup_step: info_state is 2-player only");
    return np_result(coup::np::launch_step(np_env(env), actions, out), "coup_step");
  }
  coup::StepArgs a;
  std::memset(&a, 0, sizeof(a));
  a.state = env->state;
  a.n = env->batch;
  a.seed_lo = (uint32_t)env->seed;
  a.seed_hi = (uint32_t)(env->seed >> 32);
  a.env_id_base = env->env_id_base;
  a.auto_reset = (env->flags & COUP_FLAG_AUTO_RESET) ? 1 : 0;
  a.actions_in = actions;
  a.err_count = env->err_count;
  a.hist = env->hist;
  a.xcd_remap = xcd_remap(env->knobs);
#ifdef COUP_WAVE_TRACE
  a.trace = g_trace;
#endif
#ifdef COUP_AB_VARIANTS
  // COUP_STEP_DYN_LDS: extra LDS per block of the fused step, to cap blocks
  // per CU (measurement builds)
  const unsigned dyn_lds = (unsigned)env->knobs.dyn_lds;
#else
  const unsigned dyn_lds = 0u;
#endif
  if (out) {
    a.actions = out->actions;
    a.rewards = out->rewards;
    a.step_type = out->step_type;
    a.legal = out->legal_mask;
    a.cur_player = out->cur_player;
    a.obs = out->obs;
    a.info = out->info_state;
  }
  if (const char* why = coup::ep_acc_of(out, a.ep)) return fail(COUP_E_INVALID, std::string("coup_step: ") + why);
  if (a.info && !a.hist)
    return fail(COUP_E_INVALID, "coup_step: info_state needs an env created with COUP_FLAG_HISTORY");
  const bool uniform = actions == nullptr;
  a.unchecked = (!uniform && (env->flags & COUP_FLAG_UNCHECKED)) ? 1 : 0;
  const int info = a.info ? coup::kInfoWrite : (a.hist ? coup::kInfoHistory : coup::kInfoNone);
  int mode = a.obs == nullptr ? coup::kObsNone : obs_mode(env->knobs);
  if (info != coup::kInfoNone && mode != coup::kObsNone) mode = coup::kObsWaveBits;
  hipStream_t s = env->stream;
  const int64_t n = env->batch;
  if (info == coup::kInfoWrite && mode == coup::kObsNone && n > 0) {
    if (const int split = info_split(env->knobs, n)) {
      // the rules step keeping the history (no tensor), then the
      // InformationStateTensor from the new records and histories
      coup_step_outputs bare = *out;
      bare.info_state = nullptr;
      const int r = coup_step(env, actions, &bare);
      if (r != COUP_OK) return r;
      const int64_t nf4 = n * coup::kInfoF4;
      auto go = [&](auto tt, auto ss) {
        constexpr int T = decltype(tt)::value, S = decltype(ss)::value;
        coup::note_launch("coup::k_info_sweep<{}, {}>", T, S);
        coup::k_info_sweep<T, S><<<(unsigned)((nf4 + T * S - 1) / (T * S)), T, 0, s>>>(env->state, env->hist, a.info,
                                                                                        n);
      };
#ifdef COUP_AB_VARIANTS
      switch (split) {
        case 2: go(std::integral_constant<int, 256>(), std::integral_constant<int, 2>()); break;
        case 3: {
          // the shipped shape; COUP_WRITER_POL: its stores plain / sc1 / sc1 nt (-1, 0: the shipped nt)
          const unsigned g = (unsigned)((nf4 + 2047) / 2048);
          if (env->knobs.writer_pol == 1)
            coup::note_launch("coup::k_info_sweep<1024, 2, 1>"), coup::k_info_sweep<1024, 2, 1><<<g, 1024, 0, s>>>(env->state, env->hist, a.info, n);
          else if (env->knobs.writer_pol == 2)
            coup::note_launch("coup::k_info_sweep<1024, 2, 2>"), coup::k_info_sweep<1024, 2, 2><<<g, 1024, 0, s>>>(env->state, env->hist, a.info, n);
          else if (env->knobs.writer_pol == 3)
            coup::note_launch("coup::k_info_sweep<1024, 2, 3>"), coup::k_info_sweep<1024, 2, 3><<<g, 1024, 0, s>>>(env->state, env->hist, a.info, n);
          else
            go(std::integral_constant<int, 1024>(), std::integral_constant<int, 2>());
          break;
        }
        case 4: go(std::integral_constant<int, 512>(), std::integral_constant<int, 4>()); break;
        case 5: go(std::integral_constant<int, 256>(), std::integral_constant<int, 4>()); break;
        default: go(std::integral_constant<int, 512>(), std::integral_constant<int, 2>()); break;
      }
#else
      // variant 3, non-temporal global stores (sc1 nt buffer stores measured 816.7 against
      // 838.2 us in one call, r05x, and 865.0 against 864.4 in another, r05y: not shipped)
      (void)split;
      go(std::integral_constant<int, 1024>(), std::integral_constant<int, 2>());
#endif

      COUP_HIP_TRY(hipGetLastError());
      return COUP_OK;
    }
  }
  if (info == coup::kInfoNone && mode != coup::kObsNone && n > 0) {
    if (const int split = obs_split(env->knobs, n)) {
      // the rules step without tensors (its own kernel choice), then the
      // observations from the post-step records in address order
      coup_step_outputs bare = *out;
      bare.obs = nullptr;
      const int r = coup_step(env, actions, &bare);
      if (r != COUP_OK) return r;
      const int64_t nf4 = n * coup::kRowF4;
      auto rows = [&](auto tt, auto ss) {
        constexpr int T = decltype(tt)::value, S = decltype(ss)::value;
        coup::note_launch("coup::k_obs_sweep_rows<{}, {}>", T, S);
        coup::k_obs_sweep_rows<T, S><<<(unsigned)((nf4 + T * S - 1) / (T * S)), T, 0, s>>>(env->state, a.obs, n);
      };
#ifdef COUP_AB_VARIANTS
      const unsigned g = (unsigned)((nf4 + 255) / 256);
      switch (split) {
        case 2: coup::note_launch("coup::k_obs_sweep<0>"), coup::k_obs_sweep<0><<<g, 256, 0, s>>>(env->state, a.obs, n); break;
        case 3: rows(std::integral_constant<int, 256>(), std::integral_constant<int, 1>()); break;
        case 4: rows(std::integral_constant<int, 256>(), std::integral_constant<int, 2>()); break;
        case 5: rows(std::integral_constant<int, 128>(), std::integral_constant<int, 1>()); break;
        case 6: rows(std::integral_constant<int, 64>(), std::integral_constant<int, 1>()); break;
        case 7: rows(std::integral_constant<int, 512>(), std::integral_constant<int, 1>()); break;
        case 9: rows(std::integral_constant<int, 256>(), std::integral_constant<int, 3>()); break;
        case 10: rows(std::integral_constant<int, 256>(), std::integral_constant<int, 4>()); break;
        case 11: rows(std::integral_constant<int, 512>(), std::integral_constant<int, 2>()); break;
        case 12: rows(std::integral_constant<int, 128>(), std::integral_constant<int, 4>()); break;
        case 13: rows(std::integral_constant<int, 128>(), std::integral_constant<int, 2>()); break;
        case 14: rows(std::integral_constant<int, 1024>(), std::integral_constant<int, 2>()); break;
        case 15: rows(std::integral_constant<int, 1024>(), std::integral_constant<int, 1>()); break;
        case 16: rows(std::integral_constant<int, 512>(), std::integral_constant<int, 3>()); break;
        case 17: rows(std::integral_constant<int, 512>(), std::integral_constant<int, 4>()); break;
        default: coup::note_launch("coup::k_obs_sweep<1>"), coup::k_obs_sweep<1><<<g, 256, 0, s>>>(env->state, a.obs, n); break;
      }
#else
      (void)split;
      rows(std::integral_constant<int, 512>(), std::integral_constant<int, 2>());  // variant 11
#endif
      COUP_HIP_TRY(hipGetLastError());
      return COUP_OK;
    }
  }
  if (info == coup::kInfoNone && mode == coup::kObsNone && !a.unchecked && coup::regroup_lanes(env->knobs, n)) {
    auto go = [&](auto tb) {
      constexpr int TB = decltype(tb)::value;
      const unsigned g = (unsigned)((n + TB - 1) / TB);
      coup::note_launch("coup::k_step_sorted<{b}, {}>", uniform, TB);
      if (uniform)
        coup::k_step_sorted<true, TB><<<g, TB, 0, s>>>(a);
      else
        coup::k_step_sorted<false, TB><<<g, TB, 0, s>>>(a);
    };
#ifdef COUP_AB_VARIANTS
    // COUP_SORT_THREADS: lanes per regrouping block
    const int lanes = coup::sort_lanes(env->knobs.sort_lanes, coup::kStepSortLanes);
    if (lanes == 512)
      go(std::integral_constant<int, 512>());
    else if (lanes == 1024)
      go(std::integral_constant<int, 1024>());
    else
      go(std::integral_constant<int, 256>());
#else
    go(std::integral_constant<int, coup::kStepSortLanes>());
#endif
    COUP_HIP_TRY(hipGetLastError());
    return COUP_OK;
  }
  if (info == coup::kInfoNone && mode == coup::kObsNone && !a.unchecked) {
    // the group-Philox step (coup::k_step_group), TPL threads per lane
    const int tpl = step_tpl(env->knobs);
    if (tpl) {
      auto go = [&](auto tp) {
        constexpr int TP = decltype(tp)::value;
        const unsigned g = (unsigned)((n + 256 / TP - 1) / (256 / TP));
        coup::note_launch("coup::k_step_group<{}, {b}>", TP, uniform);
        if (uniform)
          coup::k_step_group<TP, true><<<g, 256, 0, s>>>(a);
        else
          coup::k_step_group<TP, false><<<g, 256, 0, s>>>(a);
      };
#ifdef COUP_AB_VARIANTS
      if (tpl == 4)
        go(std::integral_constant<int, 4>());
      else if (tpl == 2)
        go(std::integral_constant<int, 2>());
      else
#endif
        go(std::integral_constant<int, 1>());
      COUP_HIP_TRY(hipGetLastError());
      return COUP_OK;
    }
  }
#define COUP_LAUNCH_STEP(U, M, T, I) launch_step<U, M, T, I>(env, a, n, dyn_lds, s)
#ifdef COUP_AB_VARIANTS
#define COUP_LAUNCH_NO_INFO(U)                                                                       \
  switch (mode) {                                                                                    \
    case 0: COUP_LAUNCH_STEP(U, coup::kObsNone, 256, coup::kInfoNone); break;                        \
    case 1: COUP_LAUNCH_STEP(U, coup::kObsLaneRows, 256, coup::kInfoNone); break;                    \
    case 2: COUP_LAUNCH_STEP(U, coup::kObsWave, 256, coup::kInfoNone); break;                        \
    case 3: COUP_LAUNCH_STEP(U, coup::kObsWaveNT, 256, coup::kInfoNone); break;                      \
    case 5: COUP_LAUNCH_STEP(U, coup::kObsBlockBits, 256, coup::kInfoNone); break;                   \
    case 6: COUP_LAUNCH_STEP(U, coup::kObsBlockBits, 1024, coup::kInfoNone); break;                  \
    case 7: COUP_LAUNCH_STEP(U, coup::kObsBlockBitsNT, 1024, coup::kInfoNone); break;                \
    case 8: COUP_LAUNCH_STEP(U, coup::kObsWaveBitsPlain, 256, coup::kInfoNone); break;               \
    default: COUP_LAUNCH_STEP(U, coup::kObsWaveBitsSc1, 256, coup::kInfoNone); break;                \
    case 4: COUP_LAUNCH_STEP(U, coup::kObsWaveBits, 256, coup::kInfoNone); break;                    \
  }
#else
  // the product: without tensors the sorted / group steps above took every
  // checked launch, so what is left writes observations with writer 9
#define COUP_LAUNCH_NO_INFO(U) COUP_LAUNCH_STEP(U, coup::kObsWaveBitsSc1, 256, coup::kInfoNone);
#endif
#define COUP_LAUNCH_MODES(U)                                                                         \
  if (info == coup::kInfoNone) {                                                                     \
    COUP_LAUNCH_NO_INFO(U)                                                                           \
  } else if (info == coup::kInfoHistory) {                                                           \
    if (mode == 0) COUP_LAUNCH_STEP(U, coup::kObsNone, 256, coup::kInfoHistory);                     \
    else COUP_LAUNCH_STEP(U, coup::kObsWaveBits, 256, coup::kInfoHistory);                           \
  } else {                                                                                           \
    if (mode == 0) COUP_LAUNCH_STEP(U, coup::kObsNone, 256, coup::kInfoWrite);                       \
    else COUP_LAUNCH_STEP(U, coup::kObsWaveBits, 256, coup::kInfoWrite);                             \
  }
  if (uniform) {
    COUP_LAUNCH_MODES(true)
  } else if (a.unchecked) {
    // COUP_FLAG_UNCHECKED: the caller-action kernels with the reference's
    // unchecked transition compiled in (the default writers only)
    if (info == coup::kInfoNone) {
      if (mode == 0)
        launch_step<false, coup::kObsNone, 256, coup::kInfoNone, true>(env, a, n, dyn_lds, s);
      else
        launch_step<false, coup::kObsWaveBitsSc1, 256, coup::kInfoNone, true>(env, a, n, dyn_lds, s);
    } else if (info == coup::kInfoHistory) {
      if (mode == 0)
        launch_step<false, coup::kObsNone, 256, coup::kInfoHistory, true>(env, a, n, dyn_lds, s);
      else
        launch_step<false, coup::kObsWaveBits, 256, coup::kInfoHistory, true>(env, a, n, dyn_lds, s);
    } else {
      if (mode == 0)
        launch_step<false, coup::kObsNone, 256, coup::kInfoWrite, true>(env, a, n, dyn_lds, s);
      else
        launch_step<false, coup::kObsWaveBits, 256, coup::kInfoWrite, true>(env, a, n, dyn_lds, s);
    }
  } else {
    COUP_LAUNCH_MODES(false)
  }
#undef COUP_LAUNCH_MODES
#undef COUP_LAUNCH_NO_INFO
#undef COUP_LAUNCH_STEP
  COUP_HIP_TRY(hipGetLastError());
  return COUP_OK;
}

int coup_rollout(coup_env* env, int64_t steps, const coup_rollout_stats* stats) {
  COUP_CHECK_ENV(env);
  if (steps < 0) return fail(COUP_E_INVALID, "coup_rollout: negative steps");
  if (env->hist) return fail(COUP_E_INVALID, "coup_rollout: not available on an env with COUP_FLAG_HISTORY");
  if (stats) {
    coup::EpAcc ep;  // checked for both engines (the N-player launch relies on it)
    if (const char* why = coup::ep_acc_of(stats, ep)) return fail(COUP_E_INVALID, std::string("coup_rollout: ") + why);
  }
  if (env->batch == 0 || steps == 0) return COUP_OK;
  COUP_TRY(launching(env));
  if (env->generic) return np_result(coup::np::launch_rollout(np_env(env), steps, stats), "coup_rollout");
  coup::RolloutArgs a;
  std::memset(&a, 0, sizeof(a));
  a.state = env->state;
  a.n = env->batch;
  a.seed_lo = (uint32_t)env->seed;
  a.seed_hi = (uint32_t)(env->seed >> 32);
  a.env_id_base = env->env_id_base;
  a.steps = steps;
  a.err_count = env->err_count;
  if (stats) {
    if (const char* why = coup::ep_acc_of(stats, a.ep)) return fail(COUP_E_INVALID, std::string("coup_rollout: ") + why);
    a.length_sum = stats->length_sum;
  }
  if (coup::regroup_lanes(env->knobs, env->batch)) {
    const int64_t n = env->batch;
#ifdef COUP_AB_VARIANTS
    switch (coup::sort_lanes(env->knobs.sort_lanes, coup::kRolloutSortLanes)) {
      case 256: coup::note_launch("coup::k_rollout_sorted<256>"), coup::k_rollout_sorted<256><<<grid_for(n), 256, 0, env->stream>>>(a); break;
      case 512: coup::note_launch("coup::k_rollout_sorted<512>"), coup::k_rollout_sorted<512><<<(unsigned)((n + 511) / 512), 512, 0, env->stream>>>(a); break;
      default: coup::note_launch("coup::k_rollout_sorted<1024>"), coup::k_rollout_sorted<1024><<<(unsigned)((n + 1023) / 1024), 1024, 0, env->stream>>>(a); break;
    }
#else
    constexpr int TB = coup::kRolloutSortLanes;
    coup::note_launch("coup::k_rollout_sorted<{}>", TB);
    coup::k_rollout_sorted<TB><<<(unsigned)((n + TB - 1) / TB), TB, 0, env->stream>>>(a);
#endif
  } else {
    coup::note_launch("coup::k_rollout");
    coup::k_rollout<<<grid_for(env->batch), coup::kThreads, 0, env->stream>>>(a);
  }
  COUP_HIP_TRY(hipGetLastError());
  return COUP_OK;
}

int coup_step_host(coup_env* env, const int8_t* actions, int want, void* host_out) {
  COUP_CHECK_ENV(env);
  if (!host_out) return fail(COUP_E_INVALID, "coup_step_host: host_out is null");
  if (want & ~(COUP_HOST_OBS | COUP_HOST_INFO | COUP_HOST_ACTIVE))
    return fail(COUP_E_INVALID, "coup_step_host: unknown flags");
  if ((want & COUP_HOST_INFO) && !env->hist)
    return fail(COUP_E_INVALID, "coup_step_host: info_state needs an env created with COUP_FLAG_HISTORY");
  const bool active = (want & COUP_HOST_ACTIVE) && (want & (COUP_HOST_OBS | COUP_HOST_INFO));
  if ((want & COUP_HOST_ACTIVE) && (!actions || env->generic))
    return fail(COUP_E_INVALID, "coup_step_host: COUP_HOST_ACTIVE needs host actions and 2 players");
  const int64_t B = env->batch;
  if (B == 0) return COUP_OK;
  const size_t in_bytes = align16((size_t)B);
  size_t off[6];
  const size_t total = coup_step_host_layout(B, env->players, want, off);
  if (active) {
    // the active lanes' tensors, gathered after a step that writes none
    int64_t m = 0;
    for (int64_t i = 0; i < B; ++i) m += actions[i] >= 0 ? 1 : 0;
    const size_t req_off = align16(in_bytes + total), req_bytes = (size_t)(m > 0 ? m : 1) * sizeof(coup_slot_req);
    if (req_off + req_bytes > env->host_cap) {
      if (env->host_scratch) (void)hipHostFree(env->host_scratch);
      env->host_scratch = nullptr;
      env->host_cap = 0;
      COUP_HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&env->host_scratch), req_off + req_bytes,
                                 hipHostMallocMapped | hipHostMallocCoherent));
      COUP_HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&env->host_scratch_dev), env->host_scratch, 0));
      env->host_cap = req_off + req_bytes;
    }
    coup_slot_req* reqs = reinterpret_cast<coup_slot_req*>(env->host_scratch + req_off);
    for (int64_t i = 0, k = 0; i < B; ++i)
      if (actions[i] >= 0) reqs[k++] = coup_slot_req{i, -1, 0, 0};
    const int rc = coup_step_host(env, actions, 0, host_out);  // small outputs, no tensors (synchronises)
    if (rc != COUP_OK || m == 0) return rc;
    COUP_TRY(launching(env));
    const coup_slot_req* reqs_dev = reinterpret_cast<const coup_slot_req*>(env->host_scratch_dev + req_off);
    const size_t obs_bytes = (want & COUP_HOST_OBS) ? align16((size_t)m * 2u * COUP_OBS_SIZE * 4u) : 0u;
    const size_t tensor_bytes = obs_bytes + ((want & COUP_HOST_INFO) ? (size_t)m * 2u * COUP_INFO_STATE_SIZE * 4u : 0u);
    if (tensor_bytes > env->host_stage_cap) {
      if (env->host_stage) (void)hipFree(env->host_stage);
      env->host_stage = nullptr;
      env->host_stage_cap = 0;
      COUP_HIP_TRY(hipMalloc(reinterpret_cast<void**>(&env->host_stage), tensor_bytes));
      env->host_stage_cap = tensor_bytes;
    }
    hipStream_t s = env->stream;
    if (want & COUP_HOST_OBS) {
      coup::k_obs_lanes<<<(unsigned)((m + coup::kThreads - 1) / coup::kThreads), coup::kThreads, 0, s>>>(
          env->state, reqs_dev, m, reinterpret_cast<float*>(env->host_stage));
      COUP_HIP_TRY(hipGetLastError());
    }
    if (want & COUP_HOST_INFO) {
      const int64_t nf4 = m * coup::kInfoF4;
      coup::k_info_elems<<<(unsigned)((nf4 + coup::kThreads - 1) / coup::kThreads), coup::kThreads, 0, s>>>(
          env->state, env->hist, m, reinterpret_cast<float*>(env->host_stage + obs_bytes), reqs_dev);
      COUP_HIP_TRY(hipGetLastError());
    }
    COUP_HIP_TRY(hipMemcpyAsync(static_cast<uint8_t*>(host_out) + off[5], env->host_stage, tensor_bytes,
                                hipMemcpyDeviceToHost, s));
    COUP_HIP_TRY(hipStreamSynchronize(s));
    env->dirty = false;
    return COUP_OK;
  }
  if (in_bytes + total > env->host_cap) {
    if (env->host_scratch) (void)hipHostFree(env->host_scratch);
    env->host_scratch = nullptr;
    env->host_cap = 0;
    COUP_HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&env->host_scratch), in_bytes + total,
                               hipHostMallocMapped | hipHostMallocCoherent));
    COUP_HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&env->host_scratch_dev), env->host_scratch, 0));
    env->host_cap = in_bytes + total;
  }
  if (actions) std::memcpy(env->host_scratch, actions, (size_t)B);
  // small outputs (and obs) go straight into the mapped host buffer.  The
  // 19,936-byte InformationStateTensor per lane is written after the step by
  // k_info_elems (one thread per float4: the step kernel's wave-cooperative
  // writer is one wave per 64 lanes, 218 us for one lane) into device memory,
  // and everything comes over in one copy.
  const bool stage = (want & COUP_HOST_INFO) != 0;
  if (stage && total > env->host_stage_cap) {
    if (env->host_stage) (void)hipFree(env->host_stage);
    env->host_stage = nullptr;
    env->host_stage_cap = 0;
    COUP_HIP_TRY(hipMalloc(reinterpret_cast<void**>(&env->host_stage), total));
    env->host_stage_cap = total;
  }
  uint8_t* dev = stage ? env->host_stage : env->host_scratch_dev + in_bytes;
  coup_step_outputs o;
  std::memset(&o, 0, sizeof(o));
  o.legal_mask = reinterpret_cast<uint32_t*>(dev + off[0]);
  o.cur_player = reinterpret_cast<int8_t*>(dev + off[1]);
  o.step_type = dev + off[2];
  o.rewards = reinterpret_cast<int8_t*>(dev + off[3]);
  o.actions = reinterpret_cast<int8_t*>(dev + off[4]);
  if (want & COUP_HOST_OBS) o.obs = reinterpret_cast<float*>(dev + off[5]);
  float* info_out = nullptr;
  if (want & COUP_HOST_INFO)
    info_out = reinterpret_cast<float*>(dev + off[5] +
                                        ((want & COUP_HOST_OBS) ? align16((size_t)B * env->players * 49u * env->players * 4u) : 0u));
  const int r = coup_step(env, actions ? reinterpret_cast<const int8_t*>(env->host_scratch_dev) : nullptr, &o);
  if (r != COUP_OK) return r;
  if (info_out) {
    const int64_t nf4 = B * coup::kInfoF4;
    coup::k_info_elems<<<(unsigned)((nf4 + coup::kThreads - 1) / coup::kThreads), coup::kThreads, 0, env->stream>>>(
        env->state, env->hist, B, info_out);
    COUP_HIP_TRY(hipGetLastError());
  }
  if (stage)
    COUP_HIP_TRY(hipMemcpyAsync(env->host_scratch + in_bytes, env->host_stage, total, hipMemcpyDeviceToHost,
                                env->stream));
  COUP_HIP_TRY(hipStreamSynchronize(env->stream));
  env->dirty = false;
  std::memcpy(host_out, env->host_scratch + in_bytes, total);
  return COUP_OK;
}

}  // extern "C"

namespace {

// coup_step_many / coup_step_trajectory with observations: which form of
// the split step runs them?  Uniform policy, 2 players, no history,
// observations and no information state, the split step with the shipped
// writer is this batch's form (from 2^20 lanes, or COUP_OBS_SPLIT) and the
// rules regroup (from 2^18): COUP_PIPE's form (kManyTraj by default), else
// kManySerial (one coup_step per step).
int many_form(const coup_env* env, const coup_step_outputs* out) {
  if (env->generic || env->hist || !env->traj_rec || !out || !out->obs || out->info_state) return coup::kManySerial;
  if (obs_split(env->knobs, env->batch) != coup::kObsSplitDefault) return coup::kManySerial;
  if ((env->knobs.pipe == coup::kManyTraj || env->knobs.pipe == coup::kManyOverlap ||
       env->knobs.pipe == coup::kManyFused) &&
      !coup::regroup_lanes(env->knobs, env->batch))
    return coup::kManySerial;
  return env->knobs.pipe;
}

// Output slice t of a [steps][B][...] coup_step_outputs (the accumulators
// are [B] and not sliced).
coup_step_outputs slice_outputs(const coup_step_outputs& o, int64_t B, int64_t P, int64_t t) {
  coup_step_outputs s = o;
  if (o.actions) s.actions = o.actions + t * B;
  if (o.rewards) s.rewards = o.rewards + t * B * P;
  if (o.step_type) s.step_type = o.step_type + t * B;
  if (o.legal_mask) s.legal_mask = o.legal_mask + t * B;
  if (o.cur_player) s.cur_player = o.cur_player + t * B;
  if (o.obs) s.obs = o.obs + t * B * P * 49 * P;  // [B][P][49 P] (98 per player at P = 2)
  if (o.info_state) s.info_state = o.info_state + t * B * 2 * COUP_INFO_STATE_SIZE;
  return s;
}

coup::StepArgs uniform_args(const coup_env* env, const coup_step_outputs* out) {
  coup::StepArgs a;
  std::memset(&a, 0, sizeof(a));
  a.state = env->state;
  a.n = env->batch;
  a.seed_lo = (uint32_t)env->seed;
  a.seed_hi = (uint32_t)(env->seed >> 32);
  a.env_id_base = env->env_id_base;
  a.auto_reset = (env->flags & COUP_FLAG_AUTO_RESET) ? 1 : 0;
  a.err_count = env->err_count;
  (void)coup::ep_acc_of(out, a.ep);  // validated by the caller
  return a;
}

// kManyTraj: `steps` uniform split steps in chunks of up to
// knobs.traj_chunk steps.  A chunk is ONE launch of the regrouped rules
// trajectory (k_trajectory_sorted<1024, true>: the records stay in registers
// from step to step, one record load and one LDS regroup setup per chunk
// instead of per step) that also stores every step's post-step records to
// env->traj_rec[s], then one k_obs_sweep_rows<512, 2> launch per step
// writing step s's observations from them.  Results -- outputs, records,
// accumulators -- equal `steps` coup_step calls; `slices`: step t's outputs
// go to slice t of [steps][B][...] buffers, else every step overwrites out's.
// `overlap` (kManyOverlap, measurement builds): the rules trajectories run
// on env->aux, chunk c + 1's beside chunk c's writers on env->stream, the records alternating between two chunk buffers; events
// order each writer chunk after its rules and each rules chunk after the
// writers that last read its buffer.  The streams join back into
// env->stream, so the call is one fork / join, capturable into a HIP graph.
int step_many_traj(coup_env* env, int64_t steps, const coup_step_outputs* out, bool slices, bool overlap);

#ifdef COUP_AB_VARIANTS
// kManyFused (measurement builds): the `steps` uniform split steps as ONE
// launch of the regrouped rules trajectory that also writes every step's
// observations itself, in address order per block (k_trajectory_sorted<
// 1024, false, true, 4>): no record round trip through HBM, a CU's blocks
// overlapping one block's rules with another's stores.  Results equal
// `steps` coup_step calls; measured slower than kManyTraj (153.4 against
// 134.7 us per 2^20-lane step, call r05k): the store stream runs best alone.
int step_many_fused(coup_env* env, int64_t steps, const coup_step_outputs* out, bool slices) {
  const int64_t n = env->batch;
  constexpr int TB = coup::kRolloutSortLanes;
  coup::StepArgs a = uniform_args(env, out);
  a.actions = out->actions;
  a.rewards = out->rewards;
  a.step_type = out->step_type;
  a.legal = out->legal_mask;
  a.cur_player = out->cur_player;
  a.obs = out->obs;
  const coup::TrajOut x{nullptr, slices ? n : 0, slices ? n * 2 * COUP_OBS_SIZE : 0};
  auto go = [&](auto tt, auto ww) {
    constexpr int T = decltype(tt)::value, W = decltype(ww)::value;
    coup::note_launch("coup::k_trajectory_sorted<{}, false, true, {}, 0>", T, W);
    coup::k_trajectory_sorted<T, false, true, W><<<(unsigned)((n + T - 1) / T), T, 0, env->stream>>>(a, steps, x);
  };
  switch (env->knobs.fused_shape) {  // COUP_FUSED_SHAPE
    case 1: go(std::integral_constant<int, 512>(), std::integral_constant<int, 4>()); break;
    case 2: go(std::integral_constant<int, 1024>(), std::integral_constant<int, 8>()); break;
    case 3: go(std::integral_constant<int, 512>(), std::integral_constant<int, 8>()); break;
    default: go(std::integral_constant<int, TB>(), std::integral_constant<int, 4>()); break;
  }
  COUP_HIP_TRY(hipGetLastError());
  return COUP_OK;
}
#endif

int step_many_traj(coup_env* env, int64_t steps, const coup_step_outputs* out, bool slices, bool overlap) {
  const int64_t n = env->batch;
  constexpr int TB = coup::kRolloutSortLanes;
  const int64_t chunk = std::min<int64_t>(env->knobs.traj_chunk, env->traj_cap);
  const int64_t nf4 = n * coup::kRowF4;
  const unsigned wgrid = (unsigned)((nf4 + 1023) / 1024);  // 512 threads x 2 passes
  const hipStream_t R = overlap ? env->aux : env->stream;
  const hipStream_t S = env->stream;  // the writers'
  if (overlap) {
    COUP_HIP_TRY(hipEventRecord(env->ev_fork, env->stream));
    COUP_HIP_TRY(hipStreamWaitEvent(R, env->ev_fork, 0));
    if (S != env->stream) COUP_HIP_TRY(hipStreamWaitEvent(S, env->ev_fork, 0));
  }
  // the fewest chunks of at most `chunk` steps, balanced (K = 20 at the
  // default 10: 10 + 10; at 8: 7 + 7 + 6, not 8 + 8 + 4): each launch costs a
  // fixed ~14 us beside its ~14.5 us per step (the c3 trace, call r06q), and
  // a short last chunk pays it for few steps (call r06w)
  const int64_t nchunks = (steps + chunk - 1) / chunk;
  int64_t k = 0;  // chunk index
  for (int64_t t0 = 0, c = 0; t0 < steps; t0 += c, ++k) {
    c = (steps - t0 + (nchunks - k) - 1) / (nchunks - k);
    const int b = (int)(k & 1);
    uint4* const rec = env->traj_rec + (overlap ? b * env->traj_cap * n : 0);
    const coup_step_outputs o = slices ? slice_outputs(*out, n, 2, t0) : *out;
    coup::StepArgs a = uniform_args(env, out);
    a.actions = o.actions;
    a.rewards = o.rewards;
    a.step_type = o.step_type;
    a.legal = o.legal_mask;
    a.cur_player = o.cur_player;
    if (overlap && k >= 2) COUP_HIP_TRY(hipStreamWaitEvent(R, env->ev_writers[b], 0));
    const coup::TrajOut x{rec, slices ? n : 0, 0};
    const unsigned grid = (unsigned)((n + TB - 1) / TB);
#ifdef COUP_AB_VARIANTS
    auto shape = [&](auto tt, auto ww) {  // COUP_MANY_SHAPE: lanes per block, waves per SIMD budget
      constexpr int T = decltype(tt)::value, W = decltype(ww)::value;
      coup::note_launch("coup::k_trajectory_sorted<{}, true, false, {}, 0>", T, W);
      coup::k_trajectory_sorted<T, true, false, W, 0><<<(unsigned)((n + T - 1) / T), T, 0, R>>>(a, c, x);
    };
    if (env->knobs.many_stage)  // outputs staged by lane: 148.3 against 134.5 us per step (call r05m)
      coup::note_launch("coup::k_trajectory_sorted<{}, true, false, 8, 1>", TB),
          coup::k_trajectory_sorted<TB, true, false, 8, 1><<<grid, TB, 0, R>>>(a, c, x);
    else if (env->knobs.many_shape == 1)
      shape(std::integral_constant<int, 512>(), std::integral_constant<int, 8>());
    else if (env->knobs.many_shape == 2)
      shape(std::integral_constant<int, 512>(), std::integral_constant<int, 6>());
    else if (env->knobs.many_shape == 3)
      shape(std::integral_constant<int, 256>(), std::integral_constant<int, 8>());
    else if (env->knobs.many_shape == 4)
      shape(std::integral_constant<int, 1024>(), std::integral_constant<int, 4>());
    else if (overlap && env->knobs.overlap_lds > 0)  // COUP_OVERLAP_LDS: cap the rules' blocks per CU
      coup::note_launch("coup::k_trajectory_sorted<{}, true, false, 8, 0>", TB),
          coup::k_trajectory_sorted<TB, true, false, 8, 0><<<grid, TB, (unsigned)env->knobs.overlap_lds, R>>>(a, c, x);
    else
#endif
#ifndef COUP_TRAJ_NOFULL
    // every output present (the env's own buffers, bench.py's c3): the FULL
    // form, no pointer tests (c3 132.3 against 133.6-133.9 us per step, call
    // r06f; within the process-to-process spread, and fewer instructions)
    if (a.actions && a.rewards && a.step_type && a.legal && a.cur_player)
      coup::note_launch("coup::k_trajectory_sorted<{}, true, false, 8, {}, true>", TB, coup::kTrajStage),
          coup::k_trajectory_sorted<TB, true, false, 8, coup::kTrajStage, true><<<grid, TB, 0, R>>>(a, c, x);
    else
#endif
      coup::note_launch("coup::k_trajectory_sorted<{}, true, false, 8, {}>", TB, coup::kTrajStage),
          coup::k_trajectory_sorted<TB, true, false, 8, coup::kTrajStage><<<grid, TB, 0, R>>>(a, c, x);
    COUP_HIP_TRY(hipGetLastError());
    if (overlap) {
      COUP_HIP_TRY(hipEventRecord(env->ev_rules[b], R));
      COUP_HIP_TRY(hipStreamWaitEvent(S, env->ev_rules[b], 0));
    }
    for (int64_t s = 0; s < c; ++s) {
      float* obs = out->obs + (slices ? (t0 + s) * n * 2 * COUP_OBS_SIZE : 0);
#ifdef COUP_AB_VARIANTS
      auto nib = [&](auto tt, auto ss) {  // COUP_WRITER_FORM: the nibble writer's shapes
        constexpr int TT = decltype(tt)::value, SS = decltype(ss)::value;
        coup::note_launch("coup::k_obs_sweep_nib<{}, {}>", TT, SS);
        coup::k_obs_sweep_nib<TT, SS><<<(unsigned)((nf4 + TT * SS - 1) / (TT * SS)), TT, 0, S>>>(rec + s * n, obs, n);
      };
      if (env->knobs.writer_form == 1)
        nib(std::integral_constant<int, 512>(), std::integral_constant<int, 2>());
      else if (env->knobs.writer_form == 2)
        nib(std::integral_constant<int, 512>(), std::integral_constant<int, 4>());
      else if (env->knobs.writer_form == 3)
        nib(std::integral_constant<int, 1024>(), std::integral_constant<int, 2>());
      else if (env->knobs.writer_form == 4)
        nib(std::integral_constant<int, 256>(), std::integral_constant<int, 4>());
      else if (env->knobs.writer_pol == 1)  // (-1 / 0: the shipped non-temporal stores)
        coup::note_launch("coup::k_obs_sweep_rows<512, 2, 1>"), coup::k_obs_sweep_rows<512, 2, 1><<<wgrid, 512, 0, S>>>(rec + s * n, obs, n);
      else if (env->knobs.writer_pol == 2)
        coup::note_launch("coup::k_obs_sweep_rows<512, 2, 2>"), coup::k_obs_sweep_rows<512, 2, 2><<<wgrid, 512, 0, S>>>(rec + s * n, obs, n);
      else if (env->knobs.writer_pol == 3)
        coup::note_launch("coup::k_obs_sweep_rows<512, 2, 3>"), coup::k_obs_sweep_rows<512, 2, 3><<<wgrid, 512, 0, S>>>(rec + s * n, obs, n);
      else if (env->knobs.writer_dyn_lds > 0)  // COUP_WRITER_DYN_LDS: fewer writer blocks per CU
        coup::note_launch("coup::k_obs_sweep_rows<512, 2>"),
            coup::k_obs_sweep_rows<512, 2><<<wgrid, 512, (unsigned)env->knobs.writer_dyn_lds, S>>>(rec + s * n, obs, n);
      else if (env->knobs.writer_prio == 1)
        coup::note_launch("coup::k_obs_sweep_rows<512, 2, 0, 1>"), coup::k_obs_sweep_rows<512, 2, 0, 1><<<wgrid, 512, 0, S>>>(rec + s * n, obs, n);
      else if (env->knobs.writer_prio >= 2)
        coup::note_launch("coup::k_obs_sweep_rows<512, 2, 0, 3>"), coup::k_obs_sweep_rows<512, 2, 0, 3><<<wgrid, 512, 0, S>>>(rec + s * n, obs, n);
      else
#endif
        coup::note_launch("coup::k_obs_sweep_rows<512, 2>"), coup::k_obs_sweep_rows<512, 2><<<wgrid, 512, 0, S>>>(rec + s * n, obs, n);
      COUP_HIP_TRY(hipGetLastError());
    }
    if (overlap) COUP_HIP_TRY(hipEventRecord(env->ev_writers[b], S));
  }
  if (overlap && S != env->stream)  // join: the last writers (which waited for the last rules)
    COUP_HIP_TRY(hipStreamWaitEvent(env->stream, env->ev_writers[(k - 1) & 1], 0));
  return COUP_OK;
}

#ifdef COUP_AB_VARIANTS
// kManyOverlap's resources, or false where they cannot be made now -- a graph
// capture on env->stream without them: the call then runs as kManyTraj, same
// results.
bool overlap_ready(coup_env* env) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  const bool capturing =
      hipStreamIsCapturing(env->stream, &st) != hipSuccess || st != hipStreamCaptureStatusNone;
  if (env->aux) return true;
  if (capturing) return false;
  return overlap_resources(env) == COUP_OK;
}
#endif

#ifdef COUP_AB_VARIANTS
// kManyPipe (measurement builds): `steps` uniform split steps as steps + 1
// launches of k_step_obs_pipe:
// launch m runs the rules of step m (m < steps) beside the observation
// writer of step m - 1 (m >= 1).  Both read the records after step m - 1;
// the rules write the records of step m to the other buffer, so the
// records ping-pong between env->state and env->state2.  With an odd step
// count the first rules launch (no writer beside it) runs in place, so the
// last records always land in env->state.  Results equal kManyTraj's.
int step_many_pipelined(coup_env* env, int64_t steps, const coup_step_outputs* out, bool slices) {
  const int64_t n = env->batch;
  coup::PipeArgs p;
  std::memset(&p, 0, sizeof(p));
  coup::StepArgs& a = p.a;
  a = uniform_args(env, out);
  const uint32_t R = (uint32_t)((n + kPipeT - 1) / kPipeT);
  const uint32_t W = (uint32_t)((n * coup::kRowF4 + kPipeT * kPipeS - 1) / (kPipeT * kPipeS));
  uint4* const X = env->state;
  uint4* const Y = env->state2;
  uint4* cur = X;  // the records after the last rules launch
  for (int64_t m = 0; m <= steps; ++m) {
    const bool rules = m < steps, writer = m >= 1;
    uint4* next = cur;
    if (rules) {
      const coup_step_outputs o = slices ? slice_outputs(*out, n, 2, m) : *out;
      a.state = cur;
      a.actions = o.actions;
      a.rewards = o.rewards;
      a.step_type = o.step_type;
      a.legal = o.legal_mask;
      a.cur_player = o.cur_player;
      next = (m == 0 && (steps & 1)) ? cur : (cur == X ? Y : X);
      p.rules_out = next;
    }
    p.rules_blocks = rules ? R : 0u;
    p.writer_blocks = writer ? W : 0u;
    p.obs_state = cur;
    p.obs = writer ? out->obs + (slices ? (m - 1) * n * 2 * COUP_OBS_SIZE : 0) : nullptr;
    const uint32_t total = p.rules_blocks + p.writer_blocks;
    p.stride = (rules && writer) ? std::max<uint32_t>(1u, (uint32_t)(env->knobs.pipe_span * total / R)) : 1u;
    coup::note_launch("coup::k_step_obs_pipe<{}, {}>", kPipeT, kPipeS);
    coup::k_step_obs_pipe<kPipeT, kPipeS><<<total, kPipeT, 0, env->stream>>>(p);
    COUP_HIP_TRY(hipGetLastError());
    cur = next;
  }
  if (cur != X) return fail(COUP_E_HIP, "coup_step_many: internal error (records left in the second buffer)");
  return COUP_OK;
}
#endif

}  // namespace

extern "C" {

namespace {
// coup_step_many without tensors (no observations, information state or
// history): the `steps` steps as ONE trajectory launch -- the records in
// registers, every step's outputs stored over the [B] buffers (stride 0),
// so they end as the last step's -- the kernels of coup_step_trajectory
// (2 players: k_step_trajectory in place, k_trajectory_sorted from 2^18
// lanes; N players: np::k_step_trajectory / np::k_trajectory_sorted).
// Results equal `steps` coup_step calls.  COUP_PIPE=0 keeps one coup_step
// per step.
bool many_bare(const coup_env* env, const coup_step_outputs* out) {
  return env->knobs.pipe != coup::kManySerial && !env->hist && !(out && (out->obs || out->info_state));
}

int step_many_bare(coup_env* env, int64_t steps, const coup_step_outputs* out) {
  if (env->generic) return np_result(coup::np::launch_trajectory(np_env(env), steps, out, false), "coup_step_many");
  const int64_t n = env->batch;
  coup::StepArgs a = uniform_args(env, out);
  if (out) {
    a.actions = out->actions;
    a.rewards = out->rewards;
    a.step_type = out->step_type;
    a.legal = out->legal_mask;
    a.cur_player = out->cur_player;
  }
  if (coup::regroup_lanes(env->knobs, n)) {
#ifdef COUP_AB_VARIANTS
    // measurement builds: COUP_SORT_THREADS=256 / 512 lanes per regrouping block
    if (env->knobs.sort_lanes == 256 || env->knobs.sort_lanes == 512) {
      if (env->knobs.sort_lanes == 256)
        coup::note_launch("coup::k_trajectory_sorted<256, false, false, 8, 0>"),
            coup::k_trajectory_sorted<256><<<(unsigned)((n + 255) / 256), 256, 0, env->stream>>>(a, steps, {nullptr, 0});
      else
        coup::note_launch("coup::k_trajectory_sorted<512, false, false, 8, 0>"),
            coup::k_trajectory_sorted<512><<<(unsigned)((n + 511) / 512), 512, 0, env->stream>>>(a, steps, {nullptr, 0});
      COUP_HIP_TRY(hipGetLastError());
      return COUP_OK;
    }
#endif
    constexpr int TB = coup::kRolloutSortLanes;
    coup::note_launch("coup::k_trajectory_sorted<{}, false, false, 8, {}>", TB, coup::kTrajStage);
    coup::k_trajectory_sorted<TB, false, false, 8, coup::kTrajStage><<<(unsigned)((n + TB - 1) / TB), TB, 0, env->stream>>>(
        a, steps, {nullptr, 0});
  } else {
    coup::note_launch("coup::k_step_trajectory");
    coup::k_step_trajectory<<<grid_for(n), coup::kThreads, 0, env->stream>>>(a, steps, 0);
  }
  COUP_HIP_TRY(hipGetLastError());
  return COUP_OK;
}
}  // namespace

int coup_step_many(coup_env* env, int64_t steps, const coup_step_outputs* out) {
  COUP_CHECK_ENV(env);
  if (steps < 0) return fail(COUP_E_INVALID, "coup_step_many: negative steps");
  if (out && out->info_state && !env->hist)
    return fail(COUP_E_INVALID, "coup_step_many: info_state needs an env created with COUP_FLAG_HISTORY");
  {
    coup::EpAcc ep;
    if (const char* why = coup::ep_acc_of(out, ep)) return fail(COUP_E_INVALID, std::string("coup_step_many: ") + why);
  }
  if (env->batch == 0 || steps == 0) return COUP_OK;
  if (many_bare(env, out)) {
    COUP_TRY(launching(env));
    return step_many_bare(env, steps, out);
  }
  switch (many_form(env, out)) {
    case coup::kManyTraj: COUP_TRY(launching(env)); return step_many_traj(env, steps, out, false, false);
#ifdef COUP_AB_VARIANTS
    case coup::kManyFused: COUP_TRY(launching(env)); return step_many_fused(env, steps, out, false);
    case coup::kManyOverlap:
      COUP_TRY(launching(env));
      return step_many_traj(env, steps, out, false, overlap_ready(env));
    case coup::kManyPipe: COUP_TRY(launching(env)); return step_many_pipelined(env, steps, out, false);
#endif
    default: break;
  }
  for (int64_t k = 0; k < steps; ++k) COUP_TRY(coup_step(env, nullptr, out));
  return COUP_OK;
}

int coup_step_trajectory(coup_env* env, int64_t steps, const coup_step_outputs* out) {
  COUP_CHECK_ENV(env);
  if (steps < 0) return fail(COUP_E_INVALID, "coup_step_trajectory: negative steps");
  if (out && (out->obs || out->info_state)) {
    // with tensors: coup_step_many's rules-trajectory form where it applies
    // (from 2^20 lanes), else one coup_step per slice.  (A one-launch form
    // writing obs every step inside the rules kernel measured slower than
    // per-step launches: 196 vs 162 us per 2^20-lane step, DESIGN.md
    // section 5.)
    if (out->info_state && !env->hist)
      return fail(COUP_E_INVALID, "coup_step_trajectory: info_state needs an env created with COUP_FLAG_HISTORY");
    {
      coup::EpAcc ep;
      if (const char* why = coup::ep_acc_of(out, ep))
        return fail(COUP_E_INVALID, std::string("coup_step_trajectory: ") + why);
    }
    if (env->batch == 0 || steps == 0) return COUP_OK;
    switch (many_form(env, out)) {
      case coup::kManyTraj: COUP_TRY(launching(env)); return step_many_traj(env, steps, out, true, false);
#ifdef COUP_AB_VARIANTS
      case coup::kManyFused: COUP_TRY(launching(env)); return step_many_fused(env, steps, out, true);
      case coup::kManyOverlap:
        COUP_TRY(launching(env));
        return step_many_traj(env, steps, out, true, overlap_ready(env));
      case coup::kManyPipe: COUP_TRY(launching(env)); return step_many_pipelined(env, steps, out, true);
#endif
      default: break;
    }
    for (int64_t t = 0; t < steps; ++t) {
      const coup_step_outputs o = slice_outputs(*out, env->batch, env->players, t);
      COUP_TRY(coup_step(env, nullptr, &o));
    }
    return COUP_OK;
  }
  if (env->hist) return fail(COUP_E_INVALID, "coup_step_trajectory: not available on an env with COUP_FLAG_HISTORY");
  {
    coup::EpAcc ep;
    if (const char* why = coup::ep_acc_of(out, ep))
      return fail(COUP_E_INVALID, std::string("coup_step_trajectory: ") + why);
  }
  if (env->batch == 0 || steps == 0) return COUP_OK;
  COUP_TRY(launching(env));
  if (env->generic) return np_result(coup::np::launch_trajectory(np_env(env), steps, out), "coup_step_trajectory");
  coup::StepArgs a;
  std::memset(&a, 0, sizeof(a));
  a.state = env->state;
  a.n = env->batch;
  a.seed_lo = (uint32_t)env->seed;
  a.seed_hi = (uint32_t)(env->seed >> 32);
  a.env_id_base = env->env_id_base;
  a.auto_reset = (env->flags & COUP_FLAG_AUTO_RESET) ? 1 : 0;
  a.err_count = env->err_count;
  if (out) {
    a.actions = out->actions;
    a.rewards = out->rewards;
    a.step_type = out->step_type;
    a.legal = out->legal_mask;
    a.cur_player = out->cur_player;
  }
  (void)coup::ep_acc_of(out, a.ep);
  const int64_t n = env->batch;
  if (coup::regroup_lanes(env->knobs, n)) {
#ifdef COUP_AB_VARIANTS
    switch (coup::sort_lanes(env->knobs.sort_lanes, coup::kRolloutSortLanes)) {
      case 256:
        coup::note_launch("coup::k_trajectory_sorted<256, false, false, 8, 0>");
        coup::k_trajectory_sorted<256><<<grid_for(n), 256, 0, env->stream>>>(a, steps, {nullptr, n});
        break;
      case 512:
        coup::note_launch("coup::k_trajectory_sorted<512, false, false, 8, 0>");
        coup::k_trajectory_sorted<512><<<(unsigned)((n + 511) / 512), 512, 0, env->stream>>>(a, steps, {nullptr, n});
        break;
      default:
        coup::note_launch("coup::k_trajectory_sorted<1024, false, false, 8, {}>", coup::kTrajStage);
        coup::k_trajectory_sorted<1024, false, false, 8, coup::kTrajStage>
            <<<(unsigned)((n + 1023) / 1024), 1024, 0, env->stream>>>(a, steps, {nullptr, n});
        break;
    }
#else
    constexpr int TB = coup::kRolloutSortLanes;
    coup::note_launch("coup::k_trajectory_sorted<{}, false, false, 8, {}>", TB, coup::kTrajStage);
    coup::k_trajectory_sorted<TB, false, false, 8, coup::kTrajStage><<<(unsigned)((n + TB - 1) / TB), TB, 0, env->stream>>>(
        a, steps, {nullptr, n});
#endif
  } else {
    coup::note_launch("coup::k_step_trajectory");
    coup::k_step_trajectory<<<grid_for(n), coup::kThreads, 0, env->stream>>>(a, steps, n);
  }
  COUP_HIP_TRY(hipGetLastError());
  return COUP_OK;
}

int coup_apply_action(coup_env* env, const int8_t* actions) {
  COUP_CHECK_ENV(env);
  if (!actions) return fail(COUP_E_INVALID, "coup_apply_action: actions is null");
  if (env->batch == 0) return COUP_OK;
  COUP_TRY(launching(env));
  if (env->generic) return np_result(coup::np::launch_apply(np_env(env), actions), "coup_apply_action");
  if (env->flags & COUP_FLAG_UNCHECKED)
    coup::k_apply<true><<<grid_for(env->batch), coup::kThreads, 0, env->stream>>>(env->state, env->batch, actions,
                                                                                env->hist, env->err_count);
  else
    coup::k_apply<false><<<grid_for(env->batch), coup::kThreads, 0, env->stream>>>(env->state, env->batch, actions,
                                                                                 env->hist, env->err_count);
  COUP_HIP_TRY(hipGetLastError());
  return COUP_OK;
}

int coup_query(coup_env* env, const coup_query_outputs* out) {
  COUP_CHECK_ENV(env);
  if (!out) return fail(COUP_E_INVALID, "coup_query: out is null");
  if (out->info_state && !env->hist)
    return fail(COUP_E_INVALID, "coup_query: info_state needs an env created with COUP_FLAG_HISTORY");
  if (env->batch == 0) return COUP_OK;
  COUP_TRY(launching(env));
  if (env->generic) return np_result(coup::np::launch_query(np_env(env), out), "coup_query");
  coup::QueryArgs a;
  a.state = env->state;
  a.n = env->batch;
  a.legal = out->legal_mask;
  a.cur_player = out->cur_player;
  a.terminal = out->terminal;
  a.rewards = out->rewards;
  a.returns = out->returns;
  a.obs = out->obs;
  a.hist = env->hist;
  a.info = out->info_state;
  const unsigned g = grid_for(env->batch);
  hipStream_t s = env->stream;
  if (a.info && env->batch <= coup::kInfoElemsMaxBatch) {
    const int64_t nf4 = env->batch * coup::kInfoF4;
    coup::k_info_elems<<<(unsigned)((nf4 + coup::kThreads - 1) / coup::kThreads), coup::kThreads, 0, s>>>(
        env->state, env->hist, env->batch, a.info);
    a.info = nullptr;
  }
  if (a.obs && a.info)
    coup::k_query<true, true><<<g, coup::kThreads, 0, s>>>(a);
  else if (a.obs)
    coup::k_query<true, false><<<g, coup::kThreads, 0, s>>>(a);
  else if (a.info)
    coup::k_query<false, true><<<g, coup::kThreads, 0, s>>>(a);
  else
    coup::k_query<false, false><<<g, coup::kThreads, 0, s>>>(a);
  COUP_HIP_TRY(hipGetLastError());
  return COUP_OK;
}

// Wait on the host until the n completion flags in mapped host memory hold
// `seq` (k_slot / k_slot_batch raise them after their results), instead of
// synchronising the stream.  A kernel that never gets there (a HIP error) is
// caught by a stream synchronisation after a bounded wait.
// COUP_SLOT_SYNC=1: synchronise the stream instead (A/B of the two waits).
static bool slot_poll() {
  static const bool poll = [] {
    const char* e = std::getenv("COUP_SLOT_SYNC");
    return !(e && std::atoi(e) != 0);
  }();
  return poll;
}

static int wait_flags(const uint32_t* flags, int64_t n, uint32_t seq, hipStream_t s, const char* what) {
  const auto t0 = std::chrono::steady_clock::now();
  for (int64_t i = 0; i < n; ++i) {
    for (uint32_t k = 1; __atomic_load_n(flags + i, __ATOMIC_ACQUIRE) != seq; ++k) {
      if ((k & 4095u) == 0u && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
        COUP_HIP_TRY(hipStreamSynchronize(s));
        for (int64_t j = i; j < n; ++j)
          if (__atomic_load_n(flags + j, __ATOMIC_ACQUIRE) != seq)
            return fail(COUP_E_HIP, std::string(what) + ": a request raised no completion flag");
        return COUP_OK;
      }
      __builtin_ia32_pause();
    }
  }
  return COUP_OK;
}

int coup_slot_op(coup_env* env, int64_t lane, const coup_env* src_env, int64_t src_lane, int action, int flags,
                 void* host_out) {
  COUP_CHECK_ENV(env);
  if (env->generic || !env->hist)
    return fail(COUP_E_INVALID, "coup_slot_op: needs a 2-player env created with COUP_FLAG_HISTORY");
  if (flags & ~(COUP_SLOT_INIT | COUP_SLOT_OBS | COUP_SLOT_INFO | COUP_SLOT_NO_RESULT | COUP_SLOT_DEAL | COUP_SLOT_RESET |
                COUP_SLOT_UNCHECKED))
    return fail(COUP_E_INVALID, "coup_slot_op: unknown flags");
  if ((flags & COUP_SLOT_RESET) && (src_env || (flags & COUP_SLOT_INIT)))
    return fail(COUP_E_INVALID, "coup_slot_op: COUP_SLOT_RESET takes no src_env and no COUP_SLOT_INIT");
  const uint32_t mode = ((flags & COUP_SLOT_RESET) ? coup::kSlotReset : 0u) | ((flags & COUP_SLOT_DEAL) ? coup::kSlotDeal : 0u) |
                        ((flags & COUP_SLOT_UNCHECKED) ? coup::kSlotUnchecked : 0u);
  const uint32_t env_id = env->env_id_base + (uint32_t)lane;  // the lane's stream (sampling contract)
  if (lane < 0 || lane >= env->batch) return fail(COUP_E_INVALID, "coup_slot_op: lane out of range");
  if (src_env) {
    if (src_env->generic || !src_env->hist)
      return fail(COUP_E_INVALID, "coup_slot_op: src_env needs COUP_FLAG_HISTORY (2 players)");
    if (src_lane < 0 || src_lane >= src_env->batch) return fail(COUP_E_INVALID, "coup_slot_op: src_lane out of range");
  }
  // 18..127 reach the transition, which rejects them (result.ok = 0: the
  // reference's DoApplyAction raises, coup.cc:493, :806), as on the host
  if (action < -1 || action > 127) return fail(COUP_E_INVALID, "coup_slot_op: action out of range");
  const bool result = !(flags & COUP_SLOT_NO_RESULT);
  if (result && !host_out) return fail(COUP_E_INVALID, "coup_slot_op: host_out is null");
  const bool obs = result && (flags & COUP_SLOT_OBS), info = result && (flags & COUP_SLOT_INFO);
  const size_t obs_bytes = 2u * COUP_OBS_SIZE * sizeof(float), info_bytes = 2u * COUP_INFO_STATE_SIZE * sizeof(float);
  if (env->server && (!src_env || src_env->server == env->server)) {
    // the resident wave: no launch.  Stream work still in flight on either
    // env may write the lanes it reads -- wait for it first.
    coup_server* sv = env->server;
    std::lock_guard<std::recursive_mutex> lk(sv->mu);  // post, wait and the result copy as one section
    if (env->dirty) {
      COUP_HIP_TRY(hipStreamSynchronize(env->stream));
      env->dirty = false;
    }
    if (src_env && src_env != env && src_env->dirty) {
      COUP_HIP_TRY(hipStreamSynchronize(src_env->stream));
      const_cast<coup_env*>(src_env)->dirty = false;
    }
    coup::SrvReq r;
    std::memset(&r, 0, sizeof(r));
    r.dst_state = reinterpret_cast<uint64_t>(env->state + lane);
    r.dst_hist = reinterpret_cast<uint64_t>(env->hist + lane * COUP_HISTORY_BYTES);
    if (src_env) {
      r.src_state = reinterpret_cast<uint64_t>(src_env->state + src_lane);
      r.src_hist = reinterpret_cast<uint64_t>(src_env->hist + src_lane * COUP_HISTORY_BYTES);
    }
    // the result and tensors land in the server's result area
    r.op = ((uint32_t)action & 0xFFu) | ((flags & COUP_SLOT_INIT) ? coup::kSrvInit : 0u) |
           (result ? coup::kSrvResult : 0u) | (obs ? coup::kSrvObs : 0u) | (info ? coup::kSrvInfo : 0u) |
           (mode << coup::kSrvModeShift);
    r.seed_lo = (uint32_t)env->seed;
    r.seed_hi = (uint32_t)(env->seed >> 32);
    r.env_id = env_id;
    uint32_t seq = 0;
    COUP_TRY(srv_post(sv, r, &seq));
    if (!result) return COUP_OK;
    COUP_TRY(srv_wait(sv, seq));
    std::memcpy(host_out, sv->result, sizeof(coup_slot_result) + (obs ? obs_bytes : 0) + (info ? info_bytes : 0));
    return COUP_OK;
  }
  COUP_TRY(launching(env));
  COUP_TRY(srv_drain(src_env));
  if (result && !env->slot_scratch) {
    // the kernels store the result straight into pinned host memory over
    // PCIe: no copy kernel before the synchronisation
    COUP_HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&env->slot_scratch), kSlotFlagOffset + 64,
                               hipHostMallocMapped | hipHostMallocCoherent));
    COUP_HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&env->slot_scratch_dev), env->slot_scratch, 0));
    std::memset(env->slot_scratch + kSlotFlagOffset, 0, 64);  // no completion raised yet
  }
  coup::SlotArgs a;
  a.dst_state = env->state + lane;
  a.dst_hist = env->hist + lane * COUP_HISTORY_BYTES;
  a.src_state = src_env ? src_env->state + src_lane : nullptr;
  a.src_hist = src_env ? src_env->hist + src_lane * COUP_HISTORY_BYTES : nullptr;
  a.action = action;
  a.init = (flags & COUP_SLOT_INIT) ? 1 : 0;
  a.store = (src_env || a.init || action >= 0 || (mode & (coup::kSlotReset | coup::kSlotDeal))) ? 1 : 0;
  a.mode = mode;
  a.seed_lo = (uint32_t)env->seed;
  a.seed_hi = (uint32_t)(env->seed >> 32);
  a.env_id = env_id;
  uint8_t* sc = env->slot_scratch_dev;
  a.out = result ? reinterpret_cast<coup_slot_result*>(sc) : nullptr;
  a.obs = obs ? reinterpret_cast<float*>(sc + sizeof(coup_slot_result)) : nullptr;
  // an answered op without the InformationStateTensor (one kernel) raises a
  // completion flag the host polls; with it, k_info_elems follows and the
  // stream is synchronised
  const bool poll = result && !info && slot_poll();
  a.done = poll ? reinterpret_cast<uint32_t*>(sc + kSlotFlagOffset) : nullptr;
  a.seq = 0u;
  if (poll) {
    a.seq = env->slot_seq + 1u == 0u ? 1u : env->slot_seq + 1u;  // 0 is the flag's initial value
    env->slot_seq = a.seq;
  }
  hipStream_t s = env->stream;
  // the InformationStateTensor is written by k_info_elems after the op
  // (1246 threads instead of one wave)
  float* info_out = info ? reinterpret_cast<float*>(sc + sizeof(coup_slot_result) + (obs ? obs_bytes : 0)) : nullptr;
  if (obs)
    coup::k_slot<true><<<1, 64, 0, s>>>(a);
  else
    coup::k_slot<false><<<1, 64, 0, s>>>(a);
  COUP_HIP_TRY(hipGetLastError());
  if (info_out) {
    coup::k_info_elems<<<(unsigned)((coup::kInfoF4 + coup::kThreads - 1) / coup::kThreads), coup::kThreads, 0, s>>>(
        a.dst_state, a.dst_hist, 1, info_out);
    COUP_HIP_TRY(hipGetLastError());
  }
  if (!result) return COUP_OK;
  const size_t n = sizeof(coup_slot_result) + (obs ? obs_bytes : 0) + (info ? info_bytes : 0);
  if (poll) {
    COUP_TRY(wait_flags(reinterpret_cast<const uint32_t*>(env->slot_scratch + kSlotFlagOffset), 1, a.seq, s,
                        "coup_slot_op"));
  } else {
    COUP_HIP_TRY(hipStreamSynchronize(s));
  }
  env->dirty = false;  // the op's stores are visible (flag after a system-scope fence, or the synchronisation)
  std::memcpy(host_out, env->slot_scratch, n);
  return COUP_OK;
}

int coup_slot_ops(coup_env* env, int64_t n, const coup_slot_req* reqs, const coup_env* src_env, int flags,
                  void* host_out) {
  COUP_CHECK_ENV(env);
  if (env->generic || !env->hist)
    return fail(COUP_E_INVALID, "coup_slot_ops: needs a 2-player env created with COUP_FLAG_HISTORY");
  if (flags & ~(COUP_SLOT_OBS | COUP_SLOT_INFO | COUP_SLOT_NO_RESULT))
    return fail(COUP_E_INVALID, "coup_slot_ops: unknown flags");
  if (n < 0 || n > (int64_t(1) << 20)) return fail(COUP_E_INVALID, "coup_slot_ops: n out of range");
  if (n == 0) return COUP_OK;
  if (!reqs) return fail(COUP_E_INVALID, "coup_slot_ops: reqs is null");
  if (src_env && (src_env->generic || !src_env->hist))
    return fail(COUP_E_INVALID, "coup_slot_ops: src_env needs COUP_FLAG_HISTORY (2 players)");
  const bool result = !(flags & COUP_SLOT_NO_RESULT);
  if (result && !host_out) return fail(COUP_E_INVALID, "coup_slot_ops: host_out is null");
  // every request in range; destinations distinct and not a source of
  // another request of the same env (the blocks run in any order)
  std::vector<int64_t> dst((size_t)n), srcs;
  for (int64_t k = 0; k < n; ++k) {
    const coup_slot_req& r = reqs[k];
    if (r.lane < 0 || r.lane >= env->batch) return fail(COUP_E_INVALID, "coup_slot_ops: lane out of range");
    if (r.flags & ~(COUP_SLOT_INIT | COUP_SLOT_UNCHECKED))
      return fail(COUP_E_INVALID, "coup_slot_ops: request flags other than INIT / UNCHECKED");
    if (r.action < -1 || r.action > 127) return fail(COUP_E_INVALID, "coup_slot_ops: action out of range");
    if (r.src_lane >= 0) {
      if (!src_env) return fail(COUP_E_INVALID, "coup_slot_ops: a request copies but src_env is null");
      if (r.src_lane >= src_env->batch) return fail(COUP_E_INVALID, "coup_slot_ops: src_lane out of range");
      if (src_env == env) srcs.push_back(r.src_lane);
    }
    dst[(size_t)k] = r.lane;
  }
  std::sort(dst.begin(), dst.end());
  if (std::adjacent_find(dst.begin(), dst.end()) != dst.end())
    return fail(COUP_E_INVALID, "coup_slot_ops: a destination lane repeats");
  for (int64_t s : srcs)
    if (std::binary_search(dst.begin(), dst.end(), s))
      return fail(COUP_E_INVALID, "coup_slot_ops: a source lane is also a destination");
  const bool obs = result && (flags & COUP_SLOT_OBS), info = result && (flags & COUP_SLOT_INFO);
  const size_t obs_bytes = 2u * COUP_OBS_SIZE * sizeof(float), info_bytes = 2u * COUP_INFO_STATE_SIZE * sizeof(float);
  const size_t req_bytes = ((size_t)n * sizeof(coup_slot_req) + 127u) & ~(size_t)127u;
  const size_t out_bytes = result ? (size_t)n * (sizeof(coup_slot_result) + (obs ? obs_bytes : 0) +
                                                  (info ? info_bytes : 0)) : 0;
  // answered batches without the InformationStateTensor raise one completion
  // flag per request (after the results, 128-byte aligned) that the host polls
  const bool poll = result && !info && slot_poll();
  const size_t flag_off = (req_bytes + out_bytes + 127u) & ~(size_t)127u;
  const size_t flag_bytes = poll ? (size_t)n * sizeof(uint32_t) : 0;
  if (env->batch_pending) {
    // the last (asynchronous) batch may still be reading its requests
    COUP_HIP_TRY(hipStreamSynchronize(env->stream));
    env->batch_pending = false;
  }
  COUP_TRY(launching(env));
  COUP_TRY(srv_drain(src_env));
  if (flag_off + flag_bytes > env->batch_cap) {
    if (env->batch_scratch) (void)hipHostFree(env->batch_scratch);
    env->batch_scratch = nullptr;
    env->batch_cap = 0;
    const size_t cap = std::max<size_t>(flag_off + flag_bytes, 64u << 10);
    COUP_HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&env->batch_scratch), cap,
                               hipHostMallocMapped | hipHostMallocCoherent));
    COUP_HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&env->batch_scratch_dev), env->batch_scratch, 0));
    std::memset(env->batch_scratch, 0, cap);  // no completion flag raised yet
    env->batch_cap = cap;
  }
  std::memcpy(env->batch_scratch, reqs, (size_t)n * sizeof(coup_slot_req));
  uint8_t* dev = env->batch_scratch_dev;
  coup::SlotBatchArgs b;
  b.state = env->state;
  b.hist = env->hist;
  b.src_state = src_env ? src_env->state : nullptr;
  b.src_hist = src_env ? src_env->hist : nullptr;
  b.reqs = reinterpret_cast<const coup_slot_req*>(dev);
  b.out = result ? reinterpret_cast<coup_slot_result*>(dev + req_bytes) : nullptr;
  float* obs_out = obs ? reinterpret_cast<float*>(dev + req_bytes + (size_t)n * sizeof(coup_slot_result)) : nullptr;
  float* info_out = info ? reinterpret_cast<float*>(dev + req_bytes + (size_t)n * (sizeof(coup_slot_result) +
                                                                                    (obs ? obs_bytes : 0)))
                         : nullptr;
  b.obs = obs_out;
  if (poll) {
    // flag_off moves with n and the tensor flags, so the words it lands on
    // may hold an earlier call's requests or results -- even a value equal
    // to this call's seq.  Clear them before the launch (0 is never a seq):
    // a flag then equals seq only once its block has stored its result.
    std::memset(env->batch_scratch + flag_off, 0, flag_bytes);
    b.done = reinterpret_cast<uint32_t*>(dev + flag_off);
    b.seq = env->batch_seq + 1u == 0u ? 1u : env->batch_seq + 1u;  // 0: a cleared flag
    env->batch_seq = b.seq;
  }
  hipStream_t s = env->stream;
  if (obs)
    coup::k_slot_batch<true><<<(unsigned)n, 64, 0, s>>>(b);
  else
    coup::k_slot_batch<false><<<(unsigned)n, 64, 0, s>>>(b);
  COUP_HIP_TRY(hipGetLastError());
  if (info_out) {
    const int64_t nf4 = n * coup::kInfoF4;
    coup::k_info_elems<<<(unsigned)((nf4 + coup::kThreads - 1) / coup::kThreads), coup::kThreads, 0, s>>>(
        env->state, env->hist, n, info_out, b.reqs);
    COUP_HIP_TRY(hipGetLastError());
  }
  if (!result) {
    env->batch_pending = true;
    return COUP_OK;
  }
  if (poll) {
    COUP_TRY(wait_flags(reinterpret_cast<const uint32_t*>(env->batch_scratch + flag_off), n, b.seq, s,
                        "coup_slot_ops"));
  } else {
    COUP_HIP_TRY(hipStreamSynchronize(s));
  }
  env->dirty = false;
  std::memcpy(host_out, env->batch_scratch + req_bytes, out_bytes);
  return COUP_OK;
}

int coup_server_create(int64_t idle_us, coup_server** out) {
  if (!out) return fail(COUP_E_INVALID, "coup_server_create: out is null");
  *out = nullptr;
  if (idle_us < 100 || idle_us > 10000000) return fail(COUP_E_INVALID, "coup_server_create: idle_us must be 100..1e7");
  coup_server* s = new coup_server();
  s->idle_us = (uint64_t)idle_us;
  hipError_t e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking);
  if (e == hipSuccess)
    e = hipHostMalloc(reinterpret_cast<void**>(&s->host), kSrvBytes, hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void**>(&s->host_dev), s->host, 0);
  if (e != hipSuccess) {
    if (s->host) (void)hipHostFree(s->host);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
    return fail(COUP_E_HIP, std::string("coup_server_create: ") + hipGetErrorString(e));
  }
  std::memset(s->host, 0, kSrvBytes);  // every slot number 0 (never a request's), served 0, stop 0
  s->ring = reinterpret_cast<coup::SrvReq*>(s->host);
  s->ctl = reinterpret_cast<coup::SrvCtl*>(s->host + kSrvCtlOff);
  s->result = s->host + kSrvResultOff;
  s->result_dev = s->host_dev + kSrvResultOff;
  s->last_post = std::chrono::steady_clock::now();
  {
    std::lock_guard<std::mutex> g(g_servers_mu);
    g_servers.push_back(s);
  }
  *out = s;
  return COUP_OK;
}

int coup_server_destroy(coup_server* s) {
  if (!s) return fail(COUP_E_INVALID, "null coup_server");
  {
    std::lock_guard<std::mutex> g(g_servers_mu);
    g_servers.erase(std::remove(g_servers.begin(), g_servers.end(), s), g_servers.end());
  }
  int rc = COUP_OK, rc2 = COUP_OK;
  {
    std::lock_guard<std::recursive_mutex> lk(s->mu);
    if (s->running && s->posted != srv_served(s)) rc = srv_wait(s, s->posted);
    rc2 = srv_stop(s);
  }
  (void)hipStreamDestroy(s->stream);
  (void)hipHostFree(s->host);
  delete s;
  return rc != COUP_OK ? rc : rc2;
}

int coup_server_stats(const coup_server* s, uint64_t* out) {
  if (!s || !out) return fail(COUP_E_INVALID, "coup_server_stats: null argument");
  std::lock_guard<std::recursive_mutex> lk(const_cast<coup_server*>(s)->mu);
  out[0] = s->requests;
  out[1] = s->launches;
  out[2] = s->running ? 1u : 0u;
  out[3] = s->idle_us;
  return COUP_OK;
}

int coup_attach_server(coup_env* env, coup_server* srv) {
  COUP_CHECK_ENV(env);
  if (srv && (env->generic || !env->hist))
    return fail(COUP_E_INVALID, "coup_attach_server: needs a 2-player env created with COUP_FLAG_HISTORY");
  COUP_TRY(srv_drain(env));  // the old server's requests on env are done
  env->server = srv;
  return COUP_OK;
}

int coup_export_state(coup_env* env, uint32_t* dst) {
  COUP_CHECK_ENV(env);
  if (!dst) return fail(COUP_E_INVALID, "coup_export_state: dst is null");
  COUP_TRY(launching(env));
  if (env->generic) return np_result(coup::np::launch_export(np_env(env), dst), "coup_export_state");
  COUP_HIP_TRY(hipMemcpyAsync(dst, env->state, (size_t)env->batch * sizeof(uint4), hipMemcpyDeviceToDevice,
                              env->stream));
  return COUP_OK;
}

int coup_import_state(coup_env* env, const uint32_t* src) {
  COUP_CHECK_ENV(env);
  if (!src) return fail(COUP_E_INVALID, "coup_import_state: src is null");
  COUP_TRY(launching(env));
  if (env->generic) return np_result(coup::np::launch_import(np_env(env), src), "coup_import_state");
  COUP_HIP_TRY(hipMemcpyAsync(env->state, src, (size_t)env->batch * sizeof(uint4), hipMemcpyDeviceToDevice,
                              env->stream));
  return COUP_OK;
}

int coup_export_history(coup_env* env, uint8_t* dst) {
  COUP_CHECK_ENV(env);
  if (!dst) return fail(COUP_E_INVALID, "coup_export_history: dst is null");
  if (!env->hist) return fail(COUP_E_INVALID, "coup_export_history: env has no history (COUP_FLAG_HISTORY)");
  COUP_TRY(launching(env));
  COUP_HIP_TRY(hipMemcpyAsync(dst, env->hist, (size_t)env->batch * COUP_HISTORY_BYTES, hipMemcpyDeviceToDevice,
                              env->stream));
  return COUP_OK;
}

int coup_import_history(coup_env* env, const uint8_t* src) {
  COUP_CHECK_ENV(env);
  if (!src) return fail(COUP_E_INVALID, "coup_import_history: src is null");
  if (!env->hist) return fail(COUP_E_INVALID, "coup_import_history: env has no history (COUP_FLAG_HISTORY)");
  COUP_TRY(launching(env));
  COUP_HIP_TRY(hipMemcpyAsync(env->hist, src, (size_t)env->batch * COUP_HISTORY_BYTES, hipMemcpyDeviceToDevice,
                              env->stream));
  return COUP_OK;
}

int coup_write_lane(coup_env* env, int64_t lane, const coup_slot_result* src) {
  COUP_CHECK_ENV(env);
  if (!src) return fail(COUP_E_INVALID, "coup_write_lane: src is null");
  if (env->generic || !env->hist)
    return fail(COUP_E_INVALID, "coup_write_lane: needs a 2-player env created with COUP_FLAG_HISTORY");
  if (lane < 0 || lane >= env->batch) return fail(COUP_E_INVALID, "coup_write_lane: lane out of range");
  COUP_TRY(launching(env));  // after the server's pending requests and the stream's work
  COUP_HIP_TRY(hipMemcpyAsync(env->state + lane, src->record, sizeof(uint4), hipMemcpyHostToDevice, env->stream));
  COUP_HIP_TRY(hipMemcpyAsync(env->hist + lane * COUP_HISTORY_BYTES, src->history, COUP_HISTORY_BYTES,
                              hipMemcpyHostToDevice, env->stream));
  // src is the caller's memory (pageable): the copies are done on return
  COUP_HIP_TRY(hipStreamSynchronize(env->stream));
  env->dirty = false;
  return COUP_OK;
}

int coup_error_count(coup_env* env, int64_t* out) {
  COUP_CHECK_ENV(env);
  if (!out) return fail(COUP_E_INVALID, "coup_error_count: out is null");
  COUP_TRY(launching(env));
  uint32_t h = 0;
  COUP_HIP_TRY(hipMemcpyAsync(&h, env->err_count, sizeof(uint32_t), hipMemcpyDeviceToHost, env->stream));
  COUP_HIP_TRY(hipMemsetAsync(env->err_count, 0, sizeof(uint32_t), env->stream));
  COUP_HIP_TRY(hipStreamSynchronize(env->stream));
  env->dirty = false;
  *out = (int64_t)h;
  return COUP_OK;
}

int coup_obs_split_variant(int64_t batch) { return batch > 0 ? obs_split(coup::read_knobs(), batch) : 0; }

int coup_info_split_variant(int64_t batch) { return batch > 0 ? info_split(coup::read_knobs(), batch) : 0; }

int coup_launch_log(char* buf, int cap, int reset) {
  const std::string t = coup::launch_log_text();
  if (buf && cap > 0) {
    const size_t m = std::min<size_t>(t.size(), (size_t)cap - 1);
    std::memcpy(buf, t.data(), m);
    buf[m] = 0;
  }
  if (reset) coup::clear_launch_log();
  return (int)t.size();
}

int coup_build_flags(void) {
  const int stage = coup::kTrajStage << COUP_BUILD_TRAJ_STAGE_SHIFT;
#ifdef COUP_AB_VARIANTS
  return COUP_BUILD_AB_VARIANTS | stage;
#else
  return stage;
#endif
}

int coup_measure_step_traffic(int64_t batch, uint32_t* records, const coup_step_outputs* out, void* hip_stream) {
  if (batch < 0 || batch > (int64_t(1) << 32)) return fail(COUP_E_INVALID, "coup_measure_step_traffic: bad batch");
  if (!records) return fail(COUP_E_INVALID, "coup_measure_step_traffic: records is null");
  if (batch == 0) return COUP_OK;
  coup::StepArgs a;
  std::memset(&a, 0, sizeof(a));
  a.state = reinterpret_cast<uint4*>(records);
  a.n = batch;
  a.xcd_remap = xcd_remap(coup::read_knobs());
  if (out) {
    a.actions = out->actions;
    a.rewards = out->rewards;
    a.step_type = out->step_type;
    a.legal = out->legal_mask;
    a.cur_player = out->cur_player;
    a.obs = out->obs;
  }
  coup::k_measure_traffic<<<grid_for(batch), coup::kThreads, 0, (hipStream_t)hip_stream>>>(a);
  COUP_HIP_TRY(hipGetLastError());
  return COUP_OK;
}

int coup_measure_store_sweep(float* dst, int64_t n_float4, int threads, int passes, int mode, void* hip_stream) {
  if (!dst || n_float4 < 0) return fail(COUP_E_INVALID, "coup_measure_store_sweep: bad buffer");
#ifdef COUP_AB_VARIANTS
  const int pad = (mode >> 8) & 0xFF;  // measurement builds: bits 8-15, a paced sweep (k_store_sweep_paced)
  const bool writerlike = (mode & 0x10000) != 0;  // bit 16: k_store_sweep_writerlike (reads dst's first words)
  const int dens = (mode >> 17) & 0x1F;           // bits 17-21: k_store_sweep_density's dens
  mode &= ~0x3FFF00;
#else
  const bool writerlike = false;
  const int pad = 0, dens = 0;
#endif
  if (mode & ~(COUP_SWEEP_RESIDENT | COUP_SWEEP_INDEX_BITS))
    return fail(COUP_E_INVALID, "coup_measure_store_sweep: unknown mode bits");
  if (n_float4 == 0) return COUP_OK;
  hipStream_t s = (hipStream_t)hip_stream;
  const bool resident = (mode & COUP_SWEEP_RESIDENT) != 0;
  const int bits = (mode & COUP_SWEEP_INDEX_BITS) ? 1 : 0;
  auto go = [&](auto tt, auto ss) -> int {
    constexpr int T = decltype(tt)::value, S = decltype(ss)::value;
    const int64_t blocks = (n_float4 + T * S - 1) / (T * S);
    if (resident) {
#ifdef COUP_AB_VARIANTS
      int dev = 0, cus = 0;
      COUP_HIP_TRY(hipGetDevice(&dev));
      COUP_HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
      const int64_t grid = std::min<int64_t>(blocks, (int64_t)cus * (2048 / T));
      coup::k_store_sweep_resident<T, S><<<(unsigned)grid, T, 0, s>>>(dst, n_float4, bits);
#else
      return fail(COUP_E_INVALID, "coup_measure_store_sweep: the resident form is a measurement build's");
#endif
    } else if (pad > 0 || writerlike || dens > 0) {
#ifdef COUP_AB_VARIANTS
      if (dens > 0)
        coup::k_store_sweep_density<T, S><<<(unsigned)blocks, T, 0, s>>>(dst, n_float4, dens);
      else if (writerlike)  // the "records": the buffer's own first n_float4 / 49 uint4 (read, then overwritten)
        coup::k_store_sweep_writerlike<T, S><<<(unsigned)blocks, T, 0, s>>>(dst, reinterpret_cast<const uint4*>(dst),
                                                                           n_float4);
      else
        coup::k_store_sweep_paced<T, S><<<(unsigned)blocks, T, 0, s>>>(dst, n_float4, pad);
#endif
    } else {
      coup::k_store_sweep<T, S><<<(unsigned)blocks, T, 0, s>>>(dst, n_float4, bits);
    }
    COUP_HIP_TRY(hipGetLastError());
    return COUP_OK;
  };
  // the shipped writers' shapes: 512 x 2 (observations), 1024 x 2 (info state)
  if (threads == 512 && passes == 2) return go(std::integral_constant<int, 512>(), std::integral_constant<int, 2>());
  if (threads == 1024 && passes == 2) return go(std::integral_constant<int, 1024>(), std::integral_constant<int, 2>());
#ifdef COUP_AB_VARIANTS
  if (threads == 256 && passes == 2) return go(std::integral_constant<int, 256>(), std::integral_constant<int, 2>());
  if (threads == 512 && passes == 4) return go(std::integral_constant<int, 512>(), std::integral_constant<int, 4>());
  if (threads == 1024 && passes == 4) return go(std::integral_constant<int, 1024>(), std::integral_constant<int, 4>());
  if (threads == 1024 && passes == 8) return go(std::integral_constant<int, 1024>(), std::integral_constant<int, 8>());
#endif
  return fail(COUP_E_INVALID, "coup_measure_store_sweep: shape not in this build");
}

}  // extern "C"

#ifdef COUP_TRAJ_PHASES
// Measurement builds (-DCOUP_TRAJ_PHASES): k_trajectory_sorted's per-phase
// shader cycles summed over waves, then wave-steps (kTrajPhases + 1 values).
extern "C" int coup_debug_traj_phases(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_traj_phases), sizeof(g_traj_phases)) != hipSuccess) return 2;
  if (reset) {
    const unsigned long long z[kTrajPhases + 1] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_traj_phases), z, sizeof(z)) != hipSuccess) return 2;
  }
  return 0;
}
#endif
#ifdef COUP_COUNT_PHILOX
extern "C" int coup_debug_philox_counts(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_philox_counts), sizeof(unsigned long long) * 2) != hipSuccess) return 2;
  if (reset) {
    const unsigned long long z[2] = {0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_philox_counts), z, sizeof(z)) != hipSuccess) return 2;
  }
  return 0;
}
#endif
