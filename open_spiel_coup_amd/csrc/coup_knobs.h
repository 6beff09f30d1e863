// coup_knobs.h -- host-side dispatch knobs of an env, read ONCE at
// coup_create from environment variables (not at every launch).
//
// The product library instantiates only the shipped kernels; its knobs pick
// between shipped forms (the fused or split observation step, regrouping,
// coup_step_many's serial or rules-trajectory split step).  A measurement build (-DCOUP_AB_VARIANTS:
// `python -m open_spiel_coup_amd.build` also writes it to
// build/ab/libcoup_mi355x.so) adds every variant that was measured and
// rejected, selected by the knobs marked "measurement
// builds" below, for same-process A/B runs (tools/ab_step.py,
// tools/pipe_ab.py) and their equality tests (tests/ab_variants/, run by
// tests/test_gpu_ab_variants.py with COUP_LIB_PATH at that build).
#pragma once

#include <stdint.h>

#include <cstdlib>

namespace coup {

// The split observation step's shipped writer (k_obs_sweep_rows<512, 2>)
// and the split InformationStateTensor step's (k_info_sweep<1024, 2>).
constexpr int kObsSplitDefault = 11;
constexpr int kInfoSplitDefault = 3;
// coup_step_many's forms of the split observation step (COUP_PIPE): each
// step's rules then its writer (kManySerial); chunks of up to kTrajChunkMax
// steps as ONE regrouped rules-trajectory launch writing every step's
// records, then a writer launch per step (kManyTraj, shipped); measurement
// builds also: the same with the rules trajectory of chunk c + 1 on a second
// stream beside the writers of chunk c, the records double-buffered
// (kManyOverlap), and the rules of step t + 1 beside the writer of step t
// in one launch (kManyPipe), and ONE regrouped rules-trajectory launch for
// all the steps that writes every step's observations itself, block by
// block in address order (kManyFused) -- all measured slower, DESIGN.md
// section 5.
constexpr int kManySerial = 0, kManyTraj = 1, kManyPipe = 2, kManyOverlap = 3, kManyFused = 4;
constexpr int kTrajChunkDefault = 10, kTrajChunkMax = 32;  // 10: c3 131.8 against 132.8 us per step at 8 (call r06w)
// rules blocks spread over the first kPipeSpanDefault of a pipelined
// launch's block positions (COUP_PIPE_SPAN)
constexpr double kPipeSpanDefault = 0.85;

struct Knobs {
  // -- every build
  int obs_split = -1;   // COUP_OBS_SPLIT: -1 by batch (from 2^20 lanes), 0 fused, 11 the shipped writer
  int info_split = -1;  // COUP_INFO_SPLIT: -1 by batch (from 2^18 lanes), 0 fused, 3 the shipped writer
  int regroup = -1;     // COUP_REGROUP: -1 by batch (from 2^18 lanes), 0 / 1 forced
  int pipe = kManyTraj;  // COUP_PIPE: coup_step_many's form of the split step (kMany*)
  int traj_chunk = kTrajChunkDefault;  // COUP_TRAJ_CHUNK 1..kTrajChunkMax: steps per rules-trajectory launch
                                       // (the record buffer is sized by its value at coup_create)
  // -- measurement builds (-DCOUP_AB_VARIANTS); the product ignores them
  int obs_mode = 9;       // COUP_OBS_MODE 1..9: the fused step's observation writer
  int xcd_remap = 1;      // COUP_XCD_REMAP: XCD-aware block -> lane-group mapping of the fused step
  int step_tpl = 1;       // COUP_STEP_TPL 0 / 1 / 2 / 4: threads per lane of the rules-bound step
  int dyn_lds = 0;        // COUP_STEP_DYN_LDS: extra dynamic LDS per block of the fused step
  int sort_lanes = 0;     // COUP_SORT_THREADS 256 / 512 / 1024 (0: each kernel's default)
  int np_sort_lanes = 0;  // COUP_NP_SORT_THREADS
  int np_ahead = 1;       // COUP_AHEAD: the 6-player step draws the next decision ahead
  int np_reset_inline = 0;  // COUP_NP_RESET_INLINE
  int np_reset_group = 0;   // COUP_NP_RESET_GROUP (1: one thread per reset)
  int np_traj_stage = 1;    // COUP_TRAJ_STAGE
  int np_scan = 1;          // COUP_NP_SCAN
  double pipe_span = kPipeSpanDefault;  // COUP_PIPE_SPAN in (0, 1] (kManyPipe)
  int many_stage = 0;   // COUP_MANY_STAGE: the rules trajectory's outputs staged by lane (coalesced stores)
  int writer_pol = -1;  // COUP_WRITER_POL: the split writers' stores (-1 shipped, 0 nt, 1 plain, 2 sc1, 3 sc1 nt)
  int writer_prio = 0;  // COUP_WRITER_PRIO: the split writer's waves at s_setprio 1 (1) or 3 (2)
  int writer_dyn_lds = 0;  // COUP_WRITER_DYN_LDS: extra dynamic LDS per block of the rules-trajectory form's writer
  int writer_form = 0;  // COUP_WRITER_FORM: 0 the rows writer, 1..4 the nibble writer <512,2> <512,4> <1024,2> <256,4>
  int overlap_lds = 0;  // COUP_OVERLAP_LDS: extra dynamic LDS per rules block of kManyOverlap (fewer per CU)
  int many_shape = 0;   // COUP_MANY_SHAPE: its block / register budget (1: 512 x 8, 2: 512 x 6, 3: 256 x 8, 4: 1024 x 4)
  int fused_shape = 0;  // COUP_FUSED_SHAPE: kManyFused's block / register budget (0: 1024 lanes, 4 waves per SIMD)
};

inline int knob_int(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}

inline Knobs read_knobs() {
  Knobs k;
  k.obs_split = knob_int("COUP_OBS_SPLIT", -1);
  k.info_split = knob_int("COUP_INFO_SPLIT", -1);
  k.regroup = knob_int("COUP_REGROUP", -1);
  k.pipe = knob_int("COUP_PIPE", kManyTraj);
  if (k.pipe != kManySerial && k.pipe != kManyPipe && k.pipe != kManyOverlap && k.pipe != kManyFused)
    k.pipe = kManyTraj;
  k.traj_chunk = knob_int("COUP_TRAJ_CHUNK", kTrajChunkDefault);
  if (k.traj_chunk < 1 || k.traj_chunk > kTrajChunkMax) k.traj_chunk = kTrajChunkDefault;
#ifdef COUP_AB_VARIANTS
  if (const char* f = std::getenv("COUP_PIPE_SPAN")) {
    const double v = std::atof(f);
    if (v > 0.0 && v <= 1.0) k.pipe_span = v;
  }
  k.obs_mode = knob_int("COUP_OBS_MODE", 9);
  if (k.obs_mode < 1 || k.obs_mode > 9) k.obs_mode = 9;
  k.xcd_remap = knob_int("COUP_XCD_REMAP", 1) != 0;
  k.step_tpl = knob_int("COUP_STEP_TPL", 1);
  if (k.step_tpl != 1 && k.step_tpl != 2 && k.step_tpl != 4) k.step_tpl = 0;
  k.dyn_lds = knob_int("COUP_STEP_DYN_LDS", 0);
  k.sort_lanes = knob_int("COUP_SORT_THREADS", 0);
  k.np_sort_lanes = knob_int("COUP_NP_SORT_THREADS", 0);
  k.np_ahead = knob_int("COUP_AHEAD", 1) != 0;
  k.np_reset_inline = knob_int("COUP_NP_RESET_INLINE", 0) != 0;
  k.np_reset_group = knob_int("COUP_NP_RESET_GROUP", 0);
  k.np_traj_stage = knob_int("COUP_TRAJ_STAGE", 1);
  k.np_scan = knob_int("COUP_NP_SCAN", 1) != 0;
  k.fused_shape = knob_int("COUP_FUSED_SHAPE", 0);
  k.many_stage = knob_int("COUP_MANY_STAGE", 0) != 0;
  k.many_shape = knob_int("COUP_MANY_SHAPE", 0);
  k.writer_pol = knob_int("COUP_WRITER_POL", -1);
  k.writer_prio = knob_int("COUP_WRITER_PRIO", 0);
  k.writer_form = knob_int("COUP_WRITER_FORM", 0);
  k.writer_dyn_lds = knob_int("COUP_WRITER_DYN_LDS", 0);
  k.overlap_lds = knob_int("COUP_OVERLAP_LDS", 0);
#else
  // the merged launch, the two-stream overlap and the fused trajectory ship
  // in measurement builds only
  if (k.pipe == kManyPipe || k.pipe == kManyOverlap || k.pipe == kManyFused) k.pipe = kManyTraj;
#endif
  return k;
}

// Regroup a launch of n lanes by decision?  Measured on MI355X
// (tools/ab_step.py): the sort's barriers and LDS
// round trips cost more than the divergence they remove below ~4 waves per
// SIMD (2^18 lanes on 256 CUs) and win above it (2-player rollout 2^20:
// 20.5 -> 18.6 us per step; 6-player 2^20: step 56.8 -> 43.0, rollout 41.5
// -> 29.1).  COUP_REGROUP forces it off / on (tests, A/B).
constexpr int64_t kRegroupMinLanes = int64_t{1} << 18;
inline bool regroup_lanes(const Knobs& k, int64_t n) {
  return k.regroup >= 0 ? k.regroup != 0 : n >= kRegroupMinLanes;
}

// Lanes per regrouping block: the kernel's default, or (measurement builds)
// 256 / 512 / 1024 from the knob.
inline int sort_lanes(int knob, int dflt) {
  return (knob == 256 || knob == 512 || knob == 1024) ? knob : dflt;
}

}  // namespace coup
