// coup_np.h -- host-side launchers of the N-player engine (coup_nplayer.hip),
// called by the C ABI in coup_kernels.hip for envs created with
// num_players != 2 or COUP_FLAG_GENERIC.  Internal: not part of the ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "coup_episodes.h"
#include "coup_knobs.h"
#include "coup_mi355x.h"

namespace coup {
namespace np {

// One N-player env: lane records as two uint4 planes (coup_nlane.h).
struct Env {
  uint4* sa;  // [B] words 0..3
  uint4* sb;  // [B] words 4..7
  int64_t n;
  int players;
  uint32_t seed_lo, seed_hi, env_id_base;
  int auto_reset;
  uint32_t* err_count;
  hipStream_t stream;
  Knobs knobs;  // the env's dispatch knobs (coup_knobs.h), read at coup_create
};

// mode 0: episode 0, mode 1: next episode; deal: resolve the initial deals
hipError_t launch_reset(const Env& e, const uint8_t* mask, int mode, int deal);
hipError_t launch_step(const Env& e, const int8_t* actions, const coup_step_outputs* out);
hipError_t launch_rollout(const Env& e, int64_t steps, const coup_rollout_stats* stats);
// slices: step t's outputs to slice t of [steps][B] buffers; else every step
// overwrites the [B] outputs (coup_step_many)
hipError_t launch_trajectory(const Env& e, int64_t steps, const coup_step_outputs* out, bool slices = true);
hipError_t launch_apply(const Env& e, const int8_t* actions);
hipError_t launch_query(const Env& e, const coup_query_outputs* out);
// [B][8] u32 records <-> the two planes
hipError_t launch_export(const Env& e, uint32_t* dst);
hipError_t launch_import(const Env& e, const uint32_t* src);

}  // namespace np
}  // namespace coup
