// coup_regroup.h -- block-level regrouping of lanes by their next decision
// (the sorted step / rollout kernels of both engines).
//
// A wave executes the union of its lanes' branches of the rules.  The
// sorted kernels give every lane a small key (its decision 0..17, or
// kKeyReset / kKeyDead), counting-sort the block's lanes by key through
// LDS (one LDS atomic per lane for its rank within the key, an exclusive
// prefix over the key counts for the key's base), and let thread t play
// the lane in slot t, so the waves of the apply phase hold lanes taking the
// same branch.  The RNG is stateless per (lane, episode, draw index), so a
// lane can be played by any thread with the same results.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace coup {

constexpr uint32_t kKeyReset = 18u;  // the lane finished: deal its next episode, then decide
constexpr uint32_t kKeyDead = 19u;   // no decision to play (errored lane, or past the batch)
constexpr uint32_t kKeyCount = 20u;

// Keys finer than the decision (refine_key in coup_lane.h / coup_nlane.h):
// a Pass that ends a block or completes a claim (one key per claim), and a
// Challenge the challenged player wins, get their own keys so a wave of the
// rules runs one branch of apply_decision.  They sit above kKeyReset /
// kKeyDead; key_action (coup_lane.h) maps a key back to its decision.
constexpr uint32_t kKeyPassBlock = 20u;      // Pass after a Block: next turn
constexpr uint32_t kKeyPassComplete = 21u;   // + 0..3: Pass completing Foreign Aid / Tax / Exchange / Steal
constexpr uint32_t kKeyChallengeLost = 25u;  // Challenge of a player who holds the claimed card

// Trajectory kernels only (k_trajectory_sorted): the lane is terminal as the
// step starts (no auto-reset, or a terminal record at launch): it restarts
// and reports FIRST, with no decision.  Never passed to is_decision_key.
constexpr uint32_t kKeyFirst = 26u;

// a key that carries a decision to apply (not kKeyReset / kKeyDead)
__host__ __device__ __forceinline__ bool is_decision_key(uint32_t k) { return k < kKeyReset || k >= kKeyPassBlock; }

// Exclusive prefix of the key counts below `key`: Q broadcast 16-byte LDS
// reads (every lane reads the same addresses, no bank conflicts); Q = 5 for
// the 20 decision keys, 7 with the N-player refined keys (coup_nlane.h).
template <int Q = 5>
__device__ __forceinline__ uint32_t bins_below(const uint32_t* bin, uint32_t key) {
  uint32_t below = 0u;
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const uint4 b = reinterpret_cast<const uint4*>(bin)[q];
    below += (4u * q + 0u < key ? b.x : 0u) + (4u * q + 1u < key ? b.y : 0u) + (4u * q + 2u < key ? b.z : 0u) +
             (4u * q + 3u < key ? b.w : 0u);
  }
  return below;
}

// The same prefix from a wave-level scan of the 32 bins in DPP row
// operations (no LDS round trip, no per-lane selects): every lane reads bin
// (lane & 31), an inclusive scan over each 32-lane half (row_shr 1..3, then
// row_shr 4 / 8 on the upper banks, then row 0's total broadcast into row 1:
// the cross-lane prefix of the GCN ISA's DPP examples), the exclusive prefix
// of bin `key` taken from lane `key` with ds_bpermute.  6 DPP adds and one
// permute per wave against bins_below's Q 16-byte reads and ~12 Q selects
// and adds per lane (Q = 7: ~84 VALU per wave-step of the 2-player sorted
// kernels).  All 32 bins must hold valid counts (unused ones zero); key < 32.
#ifndef COUP_HOST_STANDIN
template <int CTRL, int ROW_MASK = 0xF, int BANK_MASK = 0xF>
__device__ __forceinline__ uint32_t dpp_src(uint32_t x) {
  // lanes without a source in their row (bound_ctrl) or masked off read 0
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROW_MASK, BANK_MASK, true);
}
__device__ __forceinline__ uint32_t bins_below_dpp(const uint32_t* bin, uint32_t key) {
  const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const uint32_t v = bin[lane & 31u];
  uint32_t x = v + dpp_src<0x111>(v) + dpp_src<0x112>(v) + dpp_src<0x113>(v);  // row_shr:1..3
  x += dpp_src<0x114, 0xF, 0xE>(x);                                            // row_shr:4, banks 1..3
  x += dpp_src<0x118, 0xF, 0xC>(x);                                            // row_shr:8, banks 2..3
  x += dpp_src<0x142, 0xA, 0xF>(x);  // row_bcast:15 into rows 1 and 3: the 32-lane inclusive scan
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(key << 2), (int)(x - v));
}
#endif

// The host-side choice of regrouping and block sizes is coup_knobs.h's
// (regroup_lanes, sort_lanes), read once per env at coup_create.

}  // namespace coup
