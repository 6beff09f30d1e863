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

// The host-side choice of regrouping and block sizes is coup_knobs.h's
// (regroup_lanes, sort_lanes), read once per env at coup_create.

}  // namespace coup
