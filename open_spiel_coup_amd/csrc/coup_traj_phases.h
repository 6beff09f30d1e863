// coup_traj_phases.h -- the shader-clock phase stamps of the sorted rules
// trajectories (measurement builds, -DCOUP_TRAJ_PHASES).
//
// Each wave stamps s_memtime (the shader clock) at fixed points of every
// step and accumulates the cycles between consecutive stamps per phase:
// [0] the count atomic and the count barrier, [1] the prefix and the slot
// writes, [2] the slot barrier, [3] the slot read, unpack and the FIRST /
// reset / rejected paths, [4] the decision and its deals, [5] the outputs,
// the legal mask and the next draw; [6] wave-steps.  At the kernel's end lane
// 0 of each wave adds them to a __device__ array of 7 counters (one per
// translation unit: g_traj_phases, g_np_traj_phases; coup_debug_traj_phases,
// coup_debug_np_traj_phases).  A stamp in a branch no lane of the wave takes
// is skipped, and its cycles go to the next stamp's phase; the compiler may
// schedule work across a stamp, so a phase is wall clock around the code
// between its stamps, not that code's instructions.
#pragma once

#ifdef COUP_TRAJ_PHASES
constexpr int kTrajPhases = 6;
#define COUP_TRAJ_STAMP(k)                                        \
  do {                                                             \
    const uint32_t now_ = (uint32_t)__builtin_amdgcn_s_memtime(); \
    ph_[k] += now_ - ph_last_;                                     \
    ph_last_ = now_;                                               \
  } while (0)
#define COUP_TRAJ_STAMP_DECL uint32_t ph_[kTrajPhases] = {}, ph_last_ = (uint32_t)__builtin_amdgcn_s_memtime();
#define COUP_TRAJ_STAMP_FLUSH(sym, steps)                                                            \
  do {                                                                                                \
    if ((threadIdx.x & 63u) == 0u) {                                                                  \
      for (int k_ = 0; k_ < kTrajPhases; ++k_) atomicAdd(&(sym)[k_], (unsigned long long)ph_[k_]); \
      atomicAdd(&(sym)[kTrajPhases], (unsigned long long)(steps));                                   \
    }                                                                                                 \
  } while (0)
#else
#define COUP_TRAJ_STAMP(k)
#define COUP_TRAJ_STAMP_DECL
#define COUP_TRAJ_STAMP_FLUSH(sym, steps)
#endif
