// coup_nplayer.hip -- gfx950 kernels of the N-player extension (N = 2..6).
//
// Same execution model as coup_kernels.hip: one thread per lane, the
// 32-byte record loaded as two fully coalesced uint4 planes, the rules run
// in registers (coup_nlane.h), the record stored back.  The
// ObservationTensor is produced by a separate expansion kernel (k_obs):
// with N players a lane's tensor is N x 49N floats (7 KiB at N = 6), so it
// is written by all threads of a block as one contiguous stream of
// non-temporal float4 stores decoded from the block's records in LDS.
#include <hip/hip_runtime.h>

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
__device__ unsigned long long g_np_traj_phases[7];  // coup_traj_phases.h
#endif
#include "coup_traj_phases.h"
#include "coup_launch_log.h"
#include "coup_nlane.h"
#include "coup_np.h"
#include "coup_regroup.h"

#ifdef COUP_WAVE_TRACE
extern "C" uint64_t* coup_debug_get_trace();  // coup_kernels.hip
#endif

namespace coup {
namespace np {

constexpr int kThreads = 256;

// The RNG key of lane i; -DCOUP_ABLATE_SAME_STREAM: one stream for every lane
// (measurement builds: the step without divergence, wrong results).
__device__ __forceinline__ uint32_t lane_stream_id(uint32_t env_id_base, int64_t i) {
#ifdef COUP_ABLATE_SAME_STREAM
  (void)i;
  return env_id_base;
#else
  return env_id_base + (uint32_t)i;
#endif
}

__device__ __forceinline__ void count_error(uint32_t* err_count) { atomicAdd(err_count, 1u); }

struct StepArgs {
  uint4* sa;
  uint4* sb;
  int64_t n;
  uint32_t seed_lo, seed_hi, env_id_base;
  int auto_reset;
  const int8_t* actions_in;
  int8_t* actions;
  int8_t* rewards;  // [B][N]
  uint8_t* step_type;
  uint32_t* legal;
  int8_t* cur_player;
  EpAcc ep;            // per-episode accumulators (coup_step_outputs.episodes / return_sum or episode_word)
  uint32_t* err_count;
  int64_t ostride;     // trajectories: output offset per step (B: [steps][B] slices; 0: every step overwrites)
#ifdef COUP_WAVE_TRACE
  // measurement builds only (tools/np_wave_trace.py): per wave of
  // k_step_sorted, 10 s_memrealtime (100 MHz) stamps at the phase edges
  uint64_t* trace;
#endif
};

#ifdef COUP_WAVE_TRACE
#define NP_TRACE(a, k)                                                                             \
  do {                                                                                             \
    if ((a).trace && (threadIdx.x & 63u) == 0u)                                                    \
      (a).trace[((size_t)blockIdx.x * (blockDim.x / 64u) + threadIdx.x / 64u) * 10u + (k)] =      \
          __builtin_amdgcn_s_memrealtime();                                                        \
  } while (0)
#define NP_TRACE_WAIT(a, k)                                                                        \
  do {                                                                                             \
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                               \
    NP_TRACE(a, k);                                                                                \
  } while (0)
#else
#define NP_TRACE(a, k) \
  do {                 \
  } while (0)
#define NP_TRACE_WAIT(a, k) \
  do {                      \
  } while (0)
#endif

// Episode accumulators (coup_episodes.h): the lane's word(s) are loaded
// with its record, before the rules, and every lane stores them back
// (coalesced; unchanged unless the episode ended), so no wave waits on a late
// load and no line is written partially (as the 2-player kernels,
// coup_kernels.hip ep_update).
__device__ __forceinline__ EpVal load_episode(const StepArgs& a, int64_t i) { return a.ep.load(i); }

__device__ __forceinline__ void store_episode(const StepArgs& a, int64_t i, EpVal e, uint32_t st, int32_t ret0) {
  const bool last = st == 2u;
  a.ep.store(i, e, last ? 1 : 0, last ? ret0 : 0);
}

// The per-lane outputs of a step: applied action, Rewards() as (loser,
// count), step type, post-step legal mask and current player.
template <int N>
__device__ __forceinline__ void store_step_head(const StepArgs& a, int64_t i, int act, uint32_t st, uint32_t rl,
                                                uint32_t rc) {
  if (a.actions) a.actions[i] = (int8_t)act;
  if (a.rewards) {
    // Rewards(): rc to everybody, -(N-1) rc to the loser; an even-N row
    // starts 2-byte aligned, so it goes out as N/2 16-bit stores
    const uint32_t win = rc & 0xFFu, lose = (uint32_t)(-(int32_t)((N - 1) * rc)) & 0xFFu;
    if (N % 2 == 0) {
      uint16_t* row = reinterpret_cast<uint16_t*>(a.rewards + i * N);
#pragma unroll
      for (int k = 0; k < N / 2; ++k) {
        const uint32_t lo = (uint32_t)(2 * k) == rl ? lose : win, hi = (uint32_t)(2 * k + 1) == rl ? lose : win;
        row[k] = (uint16_t)(lo | (hi << 8));
      }
    } else {
#pragma unroll
      for (int p = 0; p < N; ++p) a.rewards[i * N + p] = (int8_t)((uint32_t)p == rl ? lose : win);
    }
  }
  if (a.step_type) a.step_type[i] = (uint8_t)st;
}

__device__ __forceinline__ void store_legal_player(const StepArgs& a, int64_t i, uint32_t legal, int cp) {
  if (a.legal) a.legal[i] = legal;
  if (a.cur_player) a.cur_player[i] = (int8_t)cp;
}

template <int N>
__device__ __forceinline__ void store_step_outputs(const StepArgs& a, int64_t i, int act, uint32_t st, uint32_t rl,
                                                   uint32_t rc, uint32_t legal, int cp) {
  store_step_head<N>(a, i, act, st, rl, rc);
  store_legal_player(a, i, legal, cp);
}

// One rl_environment step per lane (step_lane, coup_nlane.h), lanes in
// place: the wave runs the union of its lanes' branches of the rules.
template <int N, bool UNIFORM>
__global__ __launch_bounds__(kThreads) void k_step(StepArgs a) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= a.n) return;
  NLane<N> L = unpack<N>(a.sa[i], a.sb[i]);
  const EpVal eps = load_episode(a, i);
  NRng rng{a.seed_lo, a.seed_hi, lane_stream_id(a.env_id_base, i), 0u, make_uint4(0, 0, 0, 0)};
  int act;
  uint32_t st, rl, rc;
  int32_t ret0;
  bool error;
  step_lane<N, UNIFORM>(L, rng, UNIFORM ? 0u : (uint32_t)(uint8_t)a.actions_in[i], a.auto_reset != 0, act, st, rl,
                        rc, ret0, error);
  if (error) count_error(a.err_count);
  store_episode(a, i, eps, st, ret0);
  uint4 wa, wb;
  pack(L, wa, wb);
  a.sa[i] = wa;
  a.sb[i] = wb;
  store_step_outputs<N>(a, i, act, st, rl, rc, legal_mask(L), current_player(L));
}

// The same step with the block's lanes regrouped by decision before the
// rules run (batches of 2^18 lanes and more: coup_regroup.h).  Phase 1: each thread
// takes its lane up to the decision (step_lane_pre) and the block
// counting-sorts its lanes by that decision through LDS, so a wave of the
// apply phase holds lanes playing the same action: the union of branches it
// executes shrinks to what those lanes need.  Phase 2: thread t applies
// slot t's decision and resolves the deals.  The lanes that finished and
// auto-reset are listed in LDS and dealt their new episode by the first
// threads of the block (new_episode needs only the episode number and the
// lane's RNG stream), so the 2N-deal reset runs in one wave instead of in
// every wave holding a finished lane.  Phase 3: each thread stores its own
// lane's record and outputs back in place, coalesced.  The RNG is
// stateless per (lane, episode, draw), so results equal k_step's.
// Decision drawn ahead (AHEAD): a uniform step also draws each lane's next
// decision where phase 2 has the lane's post-step legal mask in hand, in
// regrouped order, and parks it in bits [29:25] of record word 7 (+1; 0 =
// none).  The next uniform step takes it instead of running step_lane_pre
// on the unsorted lanes.  Every other kernel's pack() clears the field, and
// export masks it, so a parked decision never outlives the state it was
// drawn for.
constexpr uint32_t kAheadShift = 25u;

// The regrouping key of decision x at L: its refined key (coup_nlane.h
// refine_key: 6-player step 37.1 -> 36.4 us per 2^20-lane step,
// profiles/r02/ab/np_refined_keys.log), or x itself in -DCOUP_NP_PLAIN_KEYS
// builds (A/B).
template <int N>
__device__ __forceinline__ uint32_t ahead_key(const NLane<N>& L, uint32_t x) {
#ifdef COUP_NP_PLAIN_KEYS
  (void)L;
  return x;
#else
  return refine_key(L, x);
#endif
}

// kKeyEnding: a LoseCard that costs its player the last face-down card while
// two seats are alive -- the decision that ends the game.  Drawn ahead
// (step_key), such lanes sort into the same wave(s) of the block, and with
// INLINE the wave that ends their games deals their next episodes at once
// (below), which removes the block's reset phase and its barrier.  Any other
// way a game ends (a lost assassination challenge's double flip, truncation)
// resets inline too, in whatever wave holds the lane.  The decision is the
// one LoseCard the hand allows (only slots 0 and 1 are offered, coup.cc:
// 811-822, and exactly one face-down card is left).
constexpr uint32_t kKeyEnding = 27u;

template <int N>
__device__ __forceinline__ uint32_t step_key(const NLane<N>& L, uint32_t x) {
  if ((x == kLoseCard1 || x == kLoseCard2) && __popc(~hand(L, L.M) & 0x1111u) == 1u && __popc(alive_mask(L)) == 2)
    return kKeyEnding;
  return ahead_key(L, x);
}

template <int N>
__device__ __forceinline__ uint32_t ending_action(const NLane<N>& L) {
  return (nib(hand(L, L.M), 0) & 1u) ? (uint32_t)kLoseCard2 : (uint32_t)kLoseCard1;
}

// INLINE = false (the default): the block's auto-resets dealt after phase 2
// by its first threads behind one more barrier; INLINE = true: where the game
// ends (COUP_NP_RESET_INLINE=1, measured slower).  RG: threads per reset in
// that phase.  With RG = 4 thread q of a reset's group computes Philox block
// q of the new episode's draws (its 2N deals and the decision drawn ahead,
// draw 2N: at most 4 blocks), and the group shares them by cross-lane
// shuffles, so a reset waits for one Philox instead of up to four in a row.
// RG = 1 (COUP_NP_RESET_GROUP=1, A/B): one thread deals a reset alone.
template <int N, bool UNIFORM, bool AHEAD, int T = kThreads, bool INLINE = false, int RG = 4>
#ifdef COUP_WAVE_TRACE
// the stamps' registers must not cost the traced kernel its 8 blocks per CU
#define NP_STEP_SORTED_BOUNDS __launch_bounds__(T, 8)
#else
#define NP_STEP_SORTED_BOUNDS __launch_bounds__(T)
#endif
__global__ NP_STEP_SORTED_BOUNDS void k_step_sorted(StepArgs a) {
  __shared__ uint4 s_a[T], s_b[T];
  __shared__ uint32_t s_meta[T];   // slot -> owner thread | key << kO | st << kO + 5 | error << kO + 7
  __shared__ uint32_t s_out[T];    // slot -> act + 1 | st << 5 | rl << 7 | rc << 10 | error << 13 |
                                          //         (ret0 + 16) << 14 | cp << 24
  __shared__ uint32_t s_legal[T];  // slot -> post-step legal mask
  __shared__ uint32_t s_reset[T];  // slots whose lane auto-resets
  __shared__ uint32_t s_bin[32];
  __shared__ uint32_t s_nreset;
  static_assert((T & (T - 1)) == 0 && T >= 64 && T <= 1024, "power-of-two block of whole waves");
  constexpr uint32_t kO = T <= 256 ? 8u : 10u;  // owner-thread bits of s_meta
  const uint32_t t = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * T;
  const int64_t i = base + t;
  const bool live = i < a.n;
  NP_TRACE(a, 0);
  if (t < 32u) s_bin[t] = 0u;
  if (t == 0u) s_nreset = 0u;

  // phase 1: up to the decision.  A lane with a parked decision needs
  // nothing else here, so its record goes to LDS as loaded (phase 2's unpack
  // ignores the parked bits): no unpack / pack round trip for it.
  NLane<N> L;
  uint32_t key = kKeyDead, st = 0u;
  bool error = false, raw = false;
  const EpVal eps = live ? load_episode(a, i) : EpVal{0, 0};
  uint4 ra = make_uint4(0u, 0u, 0u, 0u), rb = ra;
  if (live) {
    ra = a.sa[i];
    rb = a.sb[i];
  }
  NP_TRACE_WAIT(a, 1);
  if (live) {
    const uint32_t parked = (rb.w >> kAheadShift) & 31u;
    if (UNIFORM && AHEAD && parked != 0u) {
      key = parked - 1u;  // drawn by the last step for this state: a decision node
      st = 1u;            // MID
      raw = true;
    } else {
      L = unpack<N>(ra, rb);
      NRng rng{a.seed_lo, a.seed_hi, lane_stream_id(a.env_id_base, i), 0u, make_uint4(0, 0, 0, 0)};
      uint32_t x = UNIFORM ? 0u : (uint32_t)(uint8_t)a.actions_in[i];
      key = step_lane_pre<N, UNIFORM>(L, rng, x, st, error);
      if (error) count_error(a.err_count);
    }
  }
  NP_TRACE(a, 2);
  __syncthreads();
  const uint32_t rank = atomicAdd(&s_bin[key], 1u);
  __syncthreads();
  // exclusive scan of the bin counts in wave 0.  (Every wave scanning the
  // bins for itself, wave_bins_below, saves this barrier but measured slower:
  // 34.12 vs 33.78 us per 2^20-lane step, profiles/r03/ab/
  // np_step_wave_scan_rejected.jsonl.)
  if (t < 64u) {
    const uint32_t v = t < 32u ? s_bin[t] : 0u;
    uint32_t inc = v;
#pragma unroll
    for (int d = 1; d < 32; d <<= 1) {
      const uint32_t u = __shfl_up(inc, d, 64);
      if (t >= (uint32_t)d) inc += u;
    }
    if (t < 32u) s_bin[t] = inc - v;
  }
  __syncthreads();
  const uint32_t pos = s_bin[key] + rank;
  if (raw) {
    s_a[pos] = ra;
    s_b[pos] = rb;
  } else if (live) {
    uint4 wa, wb;
    pack(L, wa, wb);
    s_a[pos] = wa;
    s_b[pos] = wb;
  }
  s_meta[pos] = t | (key << kO) | (st << (kO + 5)) | ((uint32_t)error << (kO + 7));
  __syncthreads();
  NP_TRACE(a, 3);

  // phase 2: thread t runs slot t's decision
  {
    const uint32_t m = s_meta[t], k = (m >> kO) & 31u;
    if (k != kKeyDead) {
      L = unpack<N>(s_a[t], s_b[t]);
      uint32_t out = (m >> (kO + 5)) & 3u, legal = 0u;  // a lane finished in phase 1: no action, its st
      bool pending = false, decision_node = false;
      NRng rng{a.seed_lo, a.seed_hi, lane_stream_id(a.env_id_base, base + (m & (T - 1u))), 0u, make_uint4(0, 0, 0, 0)};
      if (k != kStepDone) {
        const uint32_t x = k == kKeyEnding ? ending_action(L) : key_action(k);
        const uint32_t err_before = L.err;
        apply_decision(L, x);
        L.move += 1u;
        resolve_chance(L, rng);
        const bool err = L.err && !err_before;
        if (err) count_error(a.err_count);
        const bool term = is_terminal(L);
        out = (x + 1u) | ((term ? 2u : 1u) << 5) | (L.rloser << 7) | (L.rcount << 10) | ((uint32_t)err << 13);
        if (a.ep.on() && term) out |= (uint32_t)(returns(L, 0u) + 16) << 14;
        pending = term && a.auto_reset != 0;
        decision_node = !term;  // resolve_chance leaves a live lane at a decision node
        if (INLINE && pending) {
          // SyncVectorEnv's reset (vector_env.py:62-65) where the game ended;
          // a new episode is at a decision node
          L = new_episode<N>(L.episode + 1u, rng);
          pending = false;
          decision_node = true;
        }
        if (pending) s_reset[atomicAdd(&s_nreset, 1u)] = t;
        uint4 wa, wb;
        pack(L, wa, wb);
        s_a[t] = wa;
        s_b[t] = wb;
      } else {
        out = 0u | (((m >> (kO + 5)) & 3u) << 5);
      }
      if (!pending) {
        // at a decision node LegalActionsMask is decision_mask and the player
        // L.M, without legal_mask's / current_player's terminal and chance tests
        legal = decision_node ? decision_mask(L) : legal_mask(L);
        const int cp = decision_node ? (int)L.M : current_player(L);
        out |= ((uint32_t)cp & 0xFFu) << 24;
        if (UNIFORM && AHEAD && k != kStepDone && cp >= 0) {
          const uint32_t x = sample_action(legal, rng.draw(L.episode, L.move));
          s_b[t].w |= ((INLINE ? step_key(L, x) : ahead_key(L, x)) + 1u) << kAheadShift;
        }
      }
      s_out[t] = out;
      s_legal[t] = legal;
    }
  }
  NP_TRACE(a, 4);
  __syncthreads();
  NP_TRACE(a, 5);

  // the auto-resets, packed onto the first threads
  const uint32_t nreset = INLINE ? 0u : s_nreset;
  if (RG == 4) {
    static_assert(RG == 1 || (2 * N) / 4 < 4, "a reset's draws fit four Philox blocks");
    // whole groups: 4 * nreset and T are multiples of 4, so every shuffle's
    // source lane runs the same iteration
    for (uint32_t j = t; j < 4u * nreset; j += T) {
      const uint32_t slot = s_reset[j >> 2], q = j & 3u;
      const uint32_t env = lane_stream_id(a.env_id_base, base + (s_meta[slot] & (T - 1u)));
      const uint32_t ep = (plane_episode(s_b[slot]) + 1u) & kNpEpisodeMask;
      // NRng::draw's block q (draws 4q .. 4q + 3)
      const uint4 blk = philox4x32_10(make_uint4(q, ep, a.seed_hi, 0x436F7570u), env, a.seed_lo);
      const int g = (int)(t & 63u & ~3u);  // the group's first lane in the wave
      uint32_t u[4 * ((2 * N) / 4 + 1)];
#pragma unroll
      for (int b = 0; b <= (2 * N) / 4; ++b) {
        u[4 * b + 0] = __shfl(blk.x, g + b, 64);
        u[4 * b + 1] = __shfl(blk.y, g + b, 64);
        u[4 * b + 2] = __shfl(blk.z, g + b, 64);
        u[4 * b + 3] = __shfl(blk.w, g + b, 64);
      }
      const NLane<N> R = deal_episode<N>(ep, [&](uint32_t k) { return u[k]; });
      if (q == 0u) {
        uint4 wa, wb;
        pack(R, wa, wb);
        const uint32_t legal = decision_mask(R);  // a new episode is at a decision node
        if (UNIFORM && AHEAD) wb.w |= (ahead_key(R, sample_action(legal, u[2 * N])) + 1u) << kAheadShift;
        s_a[slot] = wa;
        s_b[slot] = wb;
        s_legal[slot] = legal;
        s_out[slot] = (s_out[slot] & 0x00FFFFFFu) | ((R.M & 0xFFu) << 24);
      }
    }
  }
  for (uint32_t j = t; RG == 1 && j < nreset; j += T) {
    const uint32_t slot = s_reset[j];
    NRng rng{a.seed_lo, a.seed_hi, lane_stream_id(a.env_id_base, base + (s_meta[slot] & (T - 1u))), 0u,
             make_uint4(0, 0, 0, 0)};
    const NLane<N> R = new_episode<N>(plane_episode(s_b[slot]) + 1u, rng);
    uint4 wa, wb;
    pack(R, wa, wb);
    s_a[slot] = wa;
    s_b[slot] = wb;
    const uint32_t legal = decision_mask(R);  // a new episode is at a decision node
    s_legal[slot] = legal;
    s_out[slot] = (s_out[slot] & 0x00FFFFFFu) | ((R.M & 0xFFu) << 24);
    if (UNIFORM && AHEAD) s_b[slot].w |= (ahead_key(R, sample_action(legal, rng.draw(R.episode, R.move))) + 1u) << kAheadShift;
  }
  NP_TRACE(a, 6);
  if (!INLINE) __syncthreads();
  NP_TRACE(a, 7);

  // phase 3: each thread stores its own lane
  if (!live) return;
  a.sa[i] = s_a[pos];
  a.sb[i] = s_b[pos];
  const uint32_t o = s_out[pos];
  store_step_outputs<N>(a, i, (int)(o & 31u) - 1, (o >> 5) & 3u, (o >> 7) & 7u, (o >> 10) & 7u, s_legal[pos],
                        (int)(int8_t)(o >> 24));
  store_episode(a, i, eps, (o >> 5) & 3u, (int32_t)((o >> 14) & 31u) - 16);
  NP_TRACE(a, 8);
  NP_TRACE_WAIT(a, 9);
}

// coup_step_trajectory for N players: `steps` uniform steps per lane in one
// launch (lanes in place), step t's outputs to slice t of the [steps][B]
// buffers; k_step's step_lane, so the results equal `steps` coup_step
// launches of the in-place kernel (and of the regrouped one, which the GPU
// tests hold equal).
template <int N>
__global__ __launch_bounds__(kThreads) void k_step_trajectory(StepArgs a, int64_t steps) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= a.n) return;
  NLane<N> L = unpack<N>(a.sa[i], a.sb[i]);
  NRng rng{a.seed_lo, a.seed_hi, lane_stream_id(a.env_id_base, i), 0u, make_uint4(0, 0, 0, 0)};
  int32_t eps = 0, ret_sum = 0;
  uint32_t errs = 0;
  for (int64_t t = 0; t < steps; ++t) {
    int act;
    uint32_t st, rl, rc;
    int32_t ret0;
    bool error;
    step_lane<N, true>(L, rng, 0u, a.auto_reset != 0, act, st, rl, rc, ret0, error);
    errs += error ? 1u : 0u;
    store_step_outputs<N>(a, t * a.ostride + i, act, st, rl, rc, legal_mask(L), current_player(L));
    if (st == 2u) {
      eps += 1;
      ret_sum += ret0;
    }
  }
  uint4 wa, wb;
  pack(L, wa, wb);
  a.sa[i] = wa;
  a.sb[i] = wb;
  a.ep.add(i, eps, ret_sum);
  if (errs) atomicAdd(a.err_count, errs);
}

struct RolloutArgs {
  uint4* sa;
  uint4* sb;
  int64_t n;
  uint32_t seed_lo, seed_hi, env_id_base;
  int64_t steps;
  EpAcc ep;  // coup_rollout_stats: episodes / return_sum or episode_word
  int32_t* length_sum;
  uint32_t* err_count;
};

// `steps` uniform-random env steps per lane with auto-reset in one launch.
template <int N>
__global__ __launch_bounds__(kThreads) void k_rollout(RolloutArgs a) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= a.n) return;
  NLane<N> L = unpack<N>(a.sa[i], a.sb[i]);
  NRng rng{a.seed_lo, a.seed_hi, lane_stream_id(a.env_id_base, i), 0u, make_uint4(0, 0, 0, 0)};
  int32_t eps = 0, ret = 0, len = 0, cur = 0;
  uint32_t errs = 0;
  for (int64_t s = 0; s < a.steps; ++s) {
    if (is_terminal(L)) L = new_episode<N>(L.episode + 1u, rng);  // a terminal starting record
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
      ret += returns(L, 0u);
      len += cur;
      cur = 0;
      L = new_episode<N>(L.episode + 1u, rng);
    }
  }
  uint4 wa, wb;
  pack(L, wa, wb);
  a.sa[i] = wa;
  a.sb[i] = wb;
  a.ep.add(i, eps, ret);
  if (a.length_sum) a.length_sum[i] += len;
  if (errs) atomicAdd(a.err_count, errs);
}

// The same rollout with the block's lanes regrouped by decision every step
// (batches of 2^18 lanes and more: coup_regroup.h).  A lane's next decision is
// drawn at the end of the step before (its "key"); the block counting-sorts
// its lanes by key through LDS, and thread t plays the lane in slot t, so
// the waves applying a step hold lanes playing the same action.  A lane
// that finished gets key kReset: the finished lanes of a block land in one
// wave, which deals their new episodes, draws and applies.  Lanes wander
// between threads from step to step (the RNG is keyed by lane, and the
// per-lane statistics live in LDS by lane) and go home at the end.
// Results equal k_rollout's.
// The decision key of a lane at a decision node: the uniform policy's draw,
// or kKeyDead (counted as an error) if the node has no legal decision.
template <int N>
__device__ __forceinline__ uint32_t draw_key(const NLane<N>& L, NRng& rng, uint32_t& errs) {
  const uint32_t m = decision_mask(L);
  if (m == 0u) {
    errs += 1u;
    return kKeyDead;
  }
  return ahead_key(L, sample_action(m, rng.draw(L.episode, L.move)));
}

// 8 waves per SIMD (64 VGPRs, a few spilled): 29.1 vs 30.3 us per step at
// 6 waves.  Carrying each lane's cached Philox block through LDS with the
// record measured no faster (30.2 us) and was dropped.
// bins_below (coup_regroup.h) computed by each wave for itself: lane j < 32 reads bin j,
// a shuffle scan over the wave, and each lane picks its key's exclusive
// prefix.  One LDS read and six cross-lane shuffles per wave instead of Q
// 16-byte reads and 4Q selects per lane.  Used by the N-player sorted
// rollout, where it measured faster; the 6-player step (wave-0 scan behind a
// barrier) and the trajectory (bins_below) measured slower with it
// (DESIGN.md section 5).  All 32 bins must be valid counts (zeroed when unused).
__device__ __forceinline__ uint32_t wave_bins_below(const uint32_t* bin, uint32_t key) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t v = lane < 32u ? bin[lane] : 0u;
  uint32_t inc = v;
#pragma unroll
  for (int d = 1; d < 32; d <<= 1) {
    const uint32_t u = __shfl_up(inc, d, 64);
    if (lane >= (uint32_t)d) inc += u;
  }
  return __shfl(inc - v, (int)key, 64);
}

// WS: the bin prefix per wave (wave_bins_below, default: 20.69 vs 21.46 us
// per 6-player 2^20-lane step, profiles/r03/ab/np_scan_forms_traj_rollout.jsonl)
// or per lane (bins_below, round 2; COUP_NP_SCAN=0 at 1024-lane blocks, A/B).
template <int N, int T = kThreads, bool WS = true>
__global__ __launch_bounds__(T, 8) void k_rollout_sorted(RolloutArgs a) {
  static_assert((T & (T - 1)) == 0 && T >= 64 && T <= 1024, "power-of-two block of whole waves");
  constexpr uint32_t kO = T <= 256 ? 8u : 10u;  // lane bits of s_meta
  __shared__ uint4 s_a[T], s_b[T];
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
  NRng rng{a.seed_lo, a.seed_hi, lane_stream_id(a.env_id_base, base + t), 0u, make_uint4(0, 0, 0, 0)};
  NLane<N> L = initial_lane<N>(0u);
  uint32_t lane = t, cur = 0u, key = kKeyDead, errs = 0u;
  if (live) {
    L = unpack<N>(a.sa[base + t], a.sb[base + t]);
    if (is_terminal(L)) L = new_episode<N>(L.episode + 1u, rng);  // a terminal starting record
    resolve_chance(L, rng);  // a lane left at a chance node
    key = draw_key(L, rng, errs);
  }
  // two barriers per step (coup_kernels.hip k_trajectory_sorted: this step's
  // bins were zeroed before the last step's slot barrier, and every thread
  // reads its slot before it reaches this step's count barrier)
  __syncthreads();  // the bins and by-lane counters above are initialised
  for (int64_t s = 0; s < a.steps; ++s) {
    uint32_t* bin = s_bin[s & 1];
#ifdef COUP_TRAJ_TOP_BARRIER
    __syncthreads();  // measurement builds: the third barrier of rounds 2-5
#endif
    const uint32_t rank = atomicAdd(&bin[key], 1u);
    __syncthreads();
#ifndef COUP_NP_BINS_LANE
    // the DPP wave scan: 6-player fused rollout 22.0-22.1 -> 20.9-21.0 us per
    // step against the shuffle scan of wave_bins_below (call r06f)
    const uint32_t pos = (WS ? bins_below_dpp(bin, key) : bins_below<7>(bin, key)) + rank;
#else
    const uint32_t pos = (WS ? wave_bins_below(bin, key) : bins_below<7>(bin, key)) + rank;  // keys up to kKeyChallengeLost = 25
#endif
    if (t < 32u) s_bin[(s + 1) & 1][t] = 0u;  // read for the last time in step s - 1
    uint4 wa, wb;
    pack(L, wa, wb);
    s_a[pos] = wa;
    s_b[pos] = wb;
    s_meta[pos] = lane | (key << kO) | (cur << (kO + 5));
    __syncthreads();
    const uint32_t m = s_meta[t];
    lane = m & (T - 1u);
    key = (m >> kO) & 31u;
    cur = m >> (kO + 5);
    L = unpack<N>(s_a[t], s_b[t]);
    if (key == kKeyDead) continue;
    rng.env_id = lane_stream_id(a.env_id_base, base + lane);
    rng.blk_tag = 0u;
    if (key == kKeyReset) {
      L = new_episode<N>(L.episode + 1u, rng);
      key = draw_key(L, rng, errs);
      if (key == kKeyDead) continue;
    }
    const uint32_t err_before = L.err;
    apply_decision(L, key_action(key));
    L.move += 1u;
    resolve_chance(L, rng);
    errs += (L.err && !err_before) ? 1u : 0u;
    cur += 1u;
    if (is_terminal(L)) {
      s_eps[lane] += 1;
      s_ret[lane] += returns(L, 0u);
      s_len[lane] += (int32_t)cur;
      cur = 0u;
      key = kKeyReset;
    } else if (s + 1 < a.steps) {
      key = draw_key(L, rng, errs);
    }
  }
  if (key == kKeyReset) L = new_episode<N>(L.episode + 1u, rng);  // finished on the last step
  __syncthreads();
  uint4 wa, wb;
  pack(L, wa, wb);
  s_a[lane] = wa;
  s_b[lane] = wb;
  __syncthreads();
  if (live) {
    const int64_t i = base + t;
    a.sa[i] = s_a[t];
    a.sb[i] = s_b[t];
    a.ep.add(i, s_eps[t], s_ret[t]);
    if (a.length_sum) a.length_sum[i] += s_len[t];
  }
  if (errs) atomicAdd(a.err_count, errs);
}

// coup_step_trajectory with the block's lanes regrouped by decision every
// step (N players, batches of 2^18 lanes and more): k_rollout_sorted's
// schedule with coup_step's outputs, stored to slice s of the [steps][B]
// buffers by lane (each step the block writes all of its lanes' range).
// Keys: a decision; kKeyFirst -- the lane is terminal as the step starts
// (no auto-reset, or a terminal record at launch): it restarts, FIRST;
// kKeyReset -- it finished the step before with auto-reset: coup_step
// reports that step's legal mask and player after the new deal, so the
// block's reset group deals the new episode, completes the finished step's
// outputs, then decides (the resets of a block sort into one wave instead
// of diverging every wave).  Results equal coup_step's, step for step.

// Step outputs staged in LDS by lane (s_out / s_olegal): the thread that
// plays a lane in regrouped order records them, and the lane's home thread
// stores them at the start of the next step -- behind that step's first
// barrier, which every trajectory step has anyway -- so each output of a
// step goes out as one coalesced store per wave instead of bytes scattered
// over the block's range (PMC WRITE was 1.8x the 13 B per
// lane-step).  s_out: act + 1 [4:0] | step type [6:5] | reward loser [9:7] |
// reward count [12:10] | legal mask and player staged [13] | player [23:16].
constexpr uint32_t kOutLegal = 1u << 13;

__device__ __forceinline__ uint32_t stage_head(int act, uint32_t st, uint32_t rl, uint32_t rc) {
  return (uint32_t)(act + 1) | (st << 5) | (rl << 7) | (rc << 10);
}
__device__ __forceinline__ uint32_t stage_player(int cp) { return kOutLegal | (((uint32_t)cp & 0xFFu) << 16); }

template <int N>
__device__ __forceinline__ void store_staged(const StepArgs& a, int64_t o, uint32_t w, uint32_t legal) {
  store_step_head<N>(a, o, (int)(w & 31u) - 1, (w >> 5) & 3u, (w >> 7) & 7u, (w >> 10) & 7u);
  if (w & kOutLegal) store_legal_player(a, o, legal, (int)(int8_t)(w >> 16));
}

// STAGE (A/B: COUP_TRAJ_STAGE=0): 1 (default) staged by lane, each lane's
// outputs stored by its home thread (store_staged); 0 the round-2 form, each
// output stored by the thread that plays the lane.  (A third form that also
// packed the byte outputs of four lanes per dword store measured slower:
// 27.5 vs 24.3 us per 2^20-lane step, profiles/r03/ab/traj_store_forms_6p.jsonl.)
template <int N, int T = kThreads, int STAGE = 1>
__global__ __launch_bounds__(T, 8) void k_trajectory_sorted(StepArgs a, int64_t steps) {
  static_assert((T & (T - 1)) == 0 && T >= 64 && T <= 1024, "power-of-two block of whole waves");
  constexpr uint32_t kO = T <= 256 ? 8u : 10u;  // lane bits of s_meta
  __shared__ uint4 s_a[T], s_b[T];
  __shared__ uint32_t s_meta[T];            // slot -> lane | key << kO
  __shared__ int32_t s_eps[T], s_ret[T];    // by lane
  __shared__ uint32_t s_out[T], s_olegal[T];  // last step's outputs, by lane
  __shared__ __attribute__((aligned(16))) uint32_t s_bin[2][32];
  const uint32_t t = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * T;
  const bool ar = a.auto_reset != 0;
  if (t < 64u) s_bin[t >> 5][t & 31u] = 0u;
  s_eps[t] = 0;
  s_ret[t] = 0;
  NRng rng{a.seed_lo, a.seed_hi, lane_stream_id(a.env_id_base, base + t), 0u, make_uint4(0, 0, 0, 0)};
  NLane<N> L = initial_lane<N>(0u);
  // ra, rb: the lane's packed record, the value that crosses the step
  // loop's back edge (the regroup moves it through LDS); every exit of a
  // lane's step packs its NLane into them, so the unpacked fields die inside
  // the step and the exits' join copies 8 registers, not the NLane's
  // (coup_kernels.hip k_trajectory_sorted: the 2-player form)
  uint4 ra = make_uint4(0u, 0u, 0u, 0u), rb = ra;
  uint32_t lane = t, key = kKeyDead, errs = 0u;
  if (base + t < a.n) {
    ra = a.sa[base + t];
    rb = a.sb[base + t];
    L = unpack<N>(ra, rb);
    if (is_terminal(L)) {
      key = kKeyFirst;
    } else {
      resolve_chance(L, rng);  // a lane left at a chance node
      const uint32_t m = decision_mask(L);
      key = m ? ahead_key(L, sample_action(m, rng.draw(L.episode, L.move))) : kKeyDead;
      pack(L, ra, rb);
    }
  }
  const uint32_t nvalid = base < a.n ? (uint32_t)(a.n - base < T ? a.n - base : T) : 0u;  // block-uniform
  // two barriers per step (coup_kernels.hip k_trajectory_sorted); the last
  // step's staged outputs are stored behind this step's count barrier, which
  // every thread reaches after staging them
  __syncthreads();  // the bins and by-lane counters above are initialised
  COUP_TRAJ_STAMP_DECL
  for (int64_t s = 0; s < steps; ++s) {
    uint32_t* bin = s_bin[s & 1];
#ifdef COUP_TRAJ_TOP_BARRIER
    __syncthreads();  // measurement builds: the third barrier of rounds 2-5
#endif
    const uint32_t rank = atomicAdd(&bin[key], 1u);
    __syncthreads();
    COUP_TRAJ_STAMP(0);
    if (STAGE == 1 && s > 0 && t < nvalid) store_staged<N>(a, (s - 1) * a.ostride + base + t, s_out[t], s_olegal[t]);
    // (the shuffle form, wave_bins_below, spilled 38 VGPRs instead of 22 here
    // and measured 26.07 vs 24.12 us per step: profiles/r03/ab/
    // np_scan_forms_traj_rollout.jsonl; the DPP form below does not spill)
#ifndef COUP_NP_BINS_LANE
    // the wave scan in DPP (coup_regroup.h): 6-player trajectory 26.36-26.72 ->
    // 25.06-25.50 us per 2^20-lane step against the per-lane prefix below,
    // alternating builds (call r06f)
    const uint32_t pos = bins_below_dpp(bin, key) + rank;
#else
    const uint32_t pos = bins_below<7>(bin, key) + rank;  // keys up to kKeyFirst = 26
#endif
    if (t < 32u) s_bin[(s + 1) & 1][t] = 0u;  // read for the last time in step s - 1
    s_a[pos] = ra;
    s_b[pos] = rb;
    s_meta[pos] = lane | (key << kO);
    COUP_TRAJ_STAMP(1);
    __syncthreads();
    COUP_TRAJ_STAMP(2);
    const uint32_t m = s_meta[t];
    lane = m & (T - 1u);
    key = (m >> kO) & 31u;
    ra = s_a[t];
    rb = s_b[t];
    L = unpack<N>(ra, rb);
    const int64_t li = base + lane;
    if (li >= a.n) continue;  // past the batch
    const int64_t o = s * a.ostride + li;
    rng.env_id = lane_stream_id(a.env_id_base, li);
    rng.blk_tag = 0u;
    // every output of step s goes through out(): staged by lane (STAGE > 0)
    // or stored at once
    auto out = [&](uint32_t w, uint32_t legal) {
      if (STAGE != 0) {
        s_out[lane] = w;
        s_olegal[lane] = legal;
      } else {
        store_staged<N>(a, o, w, legal);
      }
    };
    // a new episode and a non-terminal state after resolve_chance are
    // decision nodes: LegalActionsMask is decision_mask, the player L.M
    if (key == kKeyFirst) {  // step() after LAST (rl_environment.py:310-311)
      L = new_episode<N>(L.episode + 1u, rng);
      const uint32_t legal = decision_mask(L);
      out(stage_head(-1, 0u, 0u, 0u) | stage_player((int)L.M), legal);
      key = ahead_key(L, sample_action(legal, rng.draw(L.episode, L.move)));
      pack(L, ra, rb);
      continue;
    }
    if (key == kKeyReset) {  // finished in step s - 1 with auto-reset (vector_env.py:62-65)
      // step s - 1's legal mask and player, after the new deal: its staged
      // head is already stored (above), so these two go out directly
      L = new_episode<N>(L.episode + 1u, rng);
      const uint32_t legal = decision_mask(L);
      store_legal_player(a, o - a.ostride, legal, (int)L.M);
      key = ahead_key(L, sample_action(legal, rng.draw(L.episode, L.move)));
    }
    if (key == kKeyDead) {  // no legal decision: coup_step's rejected step
      errs += 1u;
      out(stage_head(-1, 1u, 0u, 0u) | stage_player(current_player(L)), legal_mask(L));
      pack(L, ra, rb);
      continue;
    }
    COUP_TRAJ_STAMP(3);
    const uint32_t x = key_action(key);
    const uint32_t err_before = L.err;
    apply_decision(L, x);
    L.move += 1u;
    resolve_chance(L, rng);
    errs += (L.err && !err_before) ? 1u : 0u;
    COUP_TRAJ_STAMP(4);
    const bool term = is_terminal(L);
    const uint32_t head = stage_head((int)x, term ? 2u : 1u, L.rloser, L.rcount);
    if (term) {
      s_eps[lane] += 1;
      s_ret[lane] += returns(L, 0u);
      if (ar) {
        out(head, 0u);  // legal mask and player once the next episode is dealt
        key = kKeyReset;
        pack(L, ra, rb);
        continue;
      }
      key = kKeyFirst;
      out(head | stage_player(-4), 0u);  // terminal: no legal actions, kTerminalPlayerId
      pack(L, ra, rb);
      continue;
    }
    const uint32_t legal = decision_mask(L);
    out(head | stage_player((int)L.M), legal);
    if (s + 1 < steps) key = ahead_key(L, sample_action(legal, rng.draw(L.episode, L.move)));
    pack(L, ra, rb);
    COUP_TRAJ_STAMP(5);
  }
  __syncthreads();  // the last step's staged outputs are complete
  if (STAGE == 1 && steps > 0 && t < nvalid)
    store_staged<N>(a, (steps - 1) * a.ostride + base + t, s_out[t], s_olegal[t]);
  if (steps > 0 && key == kKeyReset && base + lane < a.n) {  // finished on the last step
    L = new_episode<N>(unpack<N>(ra, rb).episode + 1u, rng);
    store_legal_player(a, (steps - 1) * a.ostride + base + lane, decision_mask(L), (int)L.M);
    pack(L, ra, rb);
  }
  __syncthreads();
  s_a[lane] = ra;
  s_b[lane] = rb;
  __syncthreads();
  if (base + t < a.n) {
    const int64_t i = base + t;
    a.sa[i] = s_a[t];
    a.sb[i] = s_b[t];
    a.ep.add(i, s_eps[t], s_ret[t]);
  }
  if (errs) atomicAdd(a.err_count, errs);
  COUP_TRAJ_STAMP_FLUSH(g_np_traj_phases, steps);
}

template <int N>
__global__ __launch_bounds__(kThreads) void k_reset(uint4* sa, uint4* sb, int64_t n, const uint8_t* mask, int mode,
                                                  int deal, uint32_t seed_lo, uint32_t seed_hi,
                                                  uint32_t env_id_base) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  if (mask && mask[i] == 0) return;
  const uint32_t ep = mode == 0 ? 0u : plane_episode(sb[i]) + 1u;
  NLane<N> L = initial_lane<N>(ep);
  L.err = (mode != 0 && L.episode == 0u) ? 1u : 0u;  // counter wrap (coup_nlane.h kNpEpisodeMask)
  if (deal) {
    NRng rng{seed_lo, seed_hi, lane_stream_id(env_id_base, i), 0u, make_uint4(0, 0, 0, 0)};
    resolve_chance(L, rng);
  }
  uint4 wa, wb;
  pack(L, wa, wb);
  sa[i] = wa;
  sb[i] = wb;
}

template <int N>
__global__ __launch_bounds__(kThreads) void k_apply(uint4* sa, uint4* sb, int64_t n, const int8_t* actions,
                                                  uint32_t* err_count) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const int x = actions[i];
  if (x < 0) return;
  NLane<N> L = unpack<N>(sa[i], sb[i]);
  const uint32_t err_before = L.err;
  if (!apply_action(L, (uint32_t)x)) {
    count_error(err_count);
    return;
  }
  if (L.err && !err_before) count_error(err_count);
  uint4 wa, wb;
  pack(L, wa, wb);
  sa[i] = wa;
  sb[i] = wb;
}

struct QueryArgs {
  const uint4* sa;
  const uint4* sb;
  int64_t n;
  uint32_t* legal;
  int8_t* cur_player;
  uint8_t* terminal;
  int8_t* rewards;  // [B][N]
  int8_t* returns;  // [B][N]
};

template <int N>
__global__ __launch_bounds__(kThreads) void k_query(QueryArgs a) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= a.n) return;
  const NLane<N> L = unpack<N>(a.sa[i], a.sb[i]);
  if (a.legal) a.legal[i] = legal_mask(L);
  if (a.cur_player) a.cur_player[i] = (int8_t)current_player(L);
  if (a.terminal) a.terminal[i] = is_terminal(L) ? 1 : 0;
#pragma unroll
  for (int p = 0; p < N; ++p) {
    if (a.rewards) a.rewards[i * N + p] = (int8_t)reward(L, (uint32_t)p);
    if (a.returns) a.returns[i * N + p] = (int8_t)returns(L, (uint32_t)p);
  }
}

// ------------------------------------------------------ observation tensor
//
// CoupObserver::WriteTensor (coup.cc:248-287) with num_players_ = N; one
// observer row is
//   [observer N | cards 20N | cur_move N | cards_state 8N | coins N | last_action 18N]
// and a lane's N rows are contiguous.  A block expands kObsLanes lanes: the
// records go to LDS (hands, coins, last actions, mover or 7 when terminal),
// then the block's kObsLanes x N x 49N floats are stored as one stream of
// float4 (the span starts 16-byte aligned since kObsLanes x N x 49N x 4 is a
// multiple of 16).
constexpr int kObsLanes = 32;

template <int N>
__global__ __launch_bounds__(kThreads) void k_obs(const uint4* sa, const uint4* sb, int64_t n, float* obs) {
  constexpr uint32_t kRow = 49u * N, kLane = N * kRow;
  typedef float v4f __attribute__((ext_vector_type(4)));
  __shared__ uint32_t rec[kObsLanes][8];
  const int64_t lane0 = (int64_t)blockIdx.x * kObsLanes;
  const int64_t left = n - lane0;
  const uint32_t nv = left >= kObsLanes ? (uint32_t)kObsLanes : (uint32_t)left;
  if (threadIdx.x < nv) {
    const uint4 wa = sa[lane0 + threadIdx.x], wb = sb[lane0 + threadIdx.x];
    const NLane<N> L = unpack<N>(wa, wb);
    obs_record(L, rec[threadIdx.x]);
  }
  __syncthreads();
  float* base = obs + lane0 * kLane;
  const uint32_t total = nv * kLane, nf4 = total / 4u;
  for (uint32_t j = threadIdx.x; j < nf4; j += kThreads) {
    const uint32_t e = 4u * j;
    uint32_t lane = e / kLane, rem = e - lane * kLane;
    uint32_t o = rem / kRow, pos = rem - o * kRow;
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[k] = obs_elem<N>(rec[lane], o, pos);
      if (++pos == kRow) {
        pos = 0;
        if (++o == (uint32_t)N) {
          o = 0;
          ++lane;
        }
      }
    }
    v4f w = {v[0], v[1], v[2], v[3]};
    __builtin_nontemporal_store(w, reinterpret_cast<v4f*>(base) + j);
  }
  if (threadIdx.x == 0) {
    for (uint32_t e = 4u * nf4; e < total; ++e) {
      const uint32_t lane = e / kLane, rem = e - lane * kLane, o = rem / kRow;
      base[e] = obs_elem<N>(rec[lane], o, rem - o * kRow);
    }
  }
}

__global__ __launch_bounds__(kThreads) void k_export(const uint4* sa, const uint4* sb, int64_t n, uint4* dst) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  dst[2 * i] = sa[i];
  uint4 b = sb[i];
  b.w &= kNpEpisodeLo;  // a parked decision (k_step_sorted) is not state
  dst[2 * i + 1] = b;
}

__global__ __launch_bounds__(kThreads) void k_import(uint4* sa, uint4* sb, int64_t n, const uint4* src) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  sa[i] = src[2 * i];
  uint4 b = src[2 * i + 1];
  b.w &= kNpEpisodeLo;
  sb[i] = b;
}

// ------------------------------------------------------------ launchers

namespace {

unsigned grid_for(int64_t n, int per_block) { return (unsigned)((n + per_block - 1) / per_block); }

// calls f(std::integral_constant<int, N>) for the env's player count
template <class F>
hipError_t dispatch(int players, F&& f) {
  switch (players) {
    case 2: f(std::integral_constant<int, 2>()); break;
    case 3: f(std::integral_constant<int, 3>()); break;
    case 4: f(std::integral_constant<int, 4>()); break;
    case 5: f(std::integral_constant<int, 5>()); break;
    case 6: f(std::integral_constant<int, 6>()); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace

hipError_t launch_reset(const Env& e, const uint8_t* mask, int mode, int deal) {
  if (e.n == 0) return hipSuccess;
  return dispatch(e.players, [&](auto np) {
    constexpr int N = decltype(np)::value;
    k_reset<N><<<grid_for(e.n, kThreads), kThreads, 0, e.stream>>>(e.sa, e.sb, e.n, mask, mode, deal, e.seed_lo,
                                                                    e.seed_hi, e.env_id_base);
  });
}

// Lanes per regrouping block.  Larger blocks give each wave of the rules
// phase lanes with fewer distinct decisions, at the price of longer
// barrier waits: the 6-player uniform step measured 39.5 / 35.9 / 36.4 us
// per 2^20-lane step at 256 / 512 / 1024 lanes, the 6-player rollout 29.3 /
// 25.7 / 22.7 us per step (3 and 4 players: 512 best for the step;
// profiles/r02/ab/np_sort_block_size.log).  The step keeps its auto-resets
// on one wave behind a barrier, which 1024-lane blocks make the longer
// wait; the rollout sorts its resets like a decision.  After the step's
// phase 2 stopped testing terminal / chance at known decision nodes, the
// 6-player step prefers 1024-lane blocks: 34.1 vs 34.7 / 35.2 us in two
// interleaved processes (profiles/r02/ab/np_step_block_size_final.jsonl).
// COUP_NP_SORT_THREADS = 256 / 512 / 1024 overrides both (A/B runs; 128
// measured 47.4 us; every size gives the same results,
// test_regrouped_*_block_size_invariant).
constexpr int step_sort_lanes(int players) { return players >= 6 ? 1024 : 512; }
constexpr int kRolloutSortLanes = 1024;

hipError_t launch_step(const Env& e, const int8_t* actions, const coup_step_outputs* out) {
  if (e.n == 0) return hipSuccess;
  StepArgs a{};
  a.sa = e.sa;
  a.sb = e.sb;
  a.n = e.n;
  a.seed_lo = e.seed_lo;
  a.seed_hi = e.seed_hi;
  a.env_id_base = e.env_id_base;
  a.auto_reset = e.auto_reset;
  a.actions_in = actions;
  a.err_count = e.err_count;
#ifdef COUP_WAVE_TRACE
  a.trace = coup_debug_get_trace();
#endif
  float* obs = nullptr;
  if (out) {
    a.actions = out->actions;
    a.rewards = out->rewards;
    a.step_type = out->step_type;
    a.legal = out->legal_mask;
    a.cur_player = out->cur_player;
    (void)ep_acc_of(out, a.ep);  // checked by the C ABI
    obs = out->obs;
  }
  return dispatch(e.players, [&](auto np) {
    constexpr int N = decltype(np)::value;
    const unsigned grid = grid_for(e.n, kThreads);
    if (regroup_lanes(e.knobs, e.n)) {
#ifdef COUP_AB_VARIANTS
      // measurement builds: the rejected schedules of DESIGN.md section 5
      // (no decision drawn ahead; COUP_NP_RESET_INLINE=1, resets dealt where
      // the game ends, 34.07 vs 35.01 us per 2^20-lane step in one process,
      // profiles/r03/ab/np_reset_inline.jsonl; COUP_NP_RESET_GROUP=1, one
      // thread per reset) and block sizes (COUP_NP_SORT_THREADS)
      const bool ahead = e.knobs.np_ahead != 0, inl = e.knobs.np_reset_inline != 0;
      const bool single = e.knobs.np_reset_group == 1;
      auto go = [&](auto lanes) {
        constexpr int TB = decltype(lanes)::value;
        const unsigned g = grid_for(e.n, TB);
        if (actions)
          note_launch("coup::np::k_step_sorted<{}, false, false, {}>", N, TB),
              k_step_sorted<N, false, false, TB><<<g, TB, 0, e.stream>>>(a);
        else if (ahead && inl)
          note_launch("coup::np::k_step_sorted<{}, true, true, {}, true>", N, TB),
              k_step_sorted<N, true, true, TB, true><<<g, TB, 0, e.stream>>>(a);
        else if (ahead && single)
          note_launch("coup::np::k_step_sorted<{}, true, true, {}, false, 1>", N, TB),
              k_step_sorted<N, true, true, TB, false, 1><<<g, TB, 0, e.stream>>>(a);
        else if (ahead)
          note_launch("coup::np::k_step_sorted<{}, true, true, {}>", N, TB),
              k_step_sorted<N, true, true, TB><<<g, TB, 0, e.stream>>>(a);
        else
          note_launch("coup::np::k_step_sorted<{}, true, false, {}>", N, TB),
              k_step_sorted<N, true, false, TB><<<g, TB, 0, e.stream>>>(a);
      };
      switch (sort_lanes(e.knobs.np_sort_lanes, step_sort_lanes(N))) {
        case 256: go(std::integral_constant<int, 256>()); break;
        case 1024: go(std::integral_constant<int, 1024>()); break;
        default: go(std::integral_constant<int, 512>()); break;
      }
#else
      // the shipped schedule: decision drawn ahead, resets dealt by 4-thread
      // groups, step_sort_lanes(N) lanes per block
      constexpr int TB = step_sort_lanes(N);
      const unsigned g = grid_for(e.n, TB);
      note_launch("coup::np::k_step_sorted<{}, {b}, {b}, {}>", N, !actions, !actions, TB);
      if (actions)
        k_step_sorted<N, false, false, TB><<<g, TB, 0, e.stream>>>(a);
      else
        k_step_sorted<N, true, true, TB><<<g, TB, 0, e.stream>>>(a);
#endif
    } else if (actions) {
      note_launch("coup::np::k_step<{}, false>", N);
      k_step<N, false><<<grid, kThreads, 0, e.stream>>>(a);
    } else {
      note_launch("coup::np::k_step<{}, true>", N);
      k_step<N, true><<<grid, kThreads, 0, e.stream>>>(a);
    }
    if (obs) {
      note_launch("coup::np::k_obs<{}>", N);
      k_obs<N><<<grid_for(e.n, kObsLanes), kThreads, 0, e.stream>>>(e.sa, e.sb, e.n, obs);
    }
  });
}

hipError_t launch_trajectory(const Env& e, int64_t steps, const coup_step_outputs* out, bool slices) {
  StepArgs a{};
  a.ostride = slices ? e.n : 0;
  a.sa = e.sa;
  a.sb = e.sb;
  a.n = e.n;
  a.seed_lo = e.seed_lo;
  a.seed_hi = e.seed_hi;
  a.env_id_base = e.env_id_base;
  a.auto_reset = e.auto_reset;
  a.err_count = e.err_count;
  if (out) {
    a.actions = out->actions;
    a.rewards = out->rewards;
    a.step_type = out->step_type;
    a.legal = out->legal_mask;
    a.cur_player = out->cur_player;
    (void)ep_acc_of(out, a.ep);  // checked by the C ABI
  }
  return dispatch(e.players, [&](auto np) {
    constexpr int N = decltype(np)::value;
    if (regroup_lanes(e.knobs, e.n)) {
#ifdef COUP_AB_VARIANTS
      switch (sort_lanes(e.knobs.np_sort_lanes, kRolloutSortLanes)) {
        case 256:
          note_launch("coup::np::k_trajectory_sorted<{}, 256>", N);
          k_trajectory_sorted<N, 256><<<grid_for(e.n, 256), 256, 0, e.stream>>>(a, steps);
          break;
        case 512:
          note_launch("coup::np::k_trajectory_sorted<{}, 512>", N);
          k_trajectory_sorted<N, 512><<<grid_for(e.n, 512), 512, 0, e.stream>>>(a, steps);
          break;
        default:
          // COUP_TRAJ_STAGE=0: the round-2 stores (1024-lane blocks)
          if (e.knobs.np_traj_stage == 0)
            note_launch("coup::np::k_trajectory_sorted<{}, 1024, 0>", N),
                k_trajectory_sorted<N, 1024, 0><<<grid_for(e.n, 1024), 1024, 0, e.stream>>>(a, steps);
          else
            note_launch("coup::np::k_trajectory_sorted<{}, 1024>", N),
                k_trajectory_sorted<N, 1024><<<grid_for(e.n, 1024), 1024, 0, e.stream>>>(a, steps);
          break;
      }
#else
      note_launch("coup::np::k_trajectory_sorted<{}, {}>", N, kRolloutSortLanes);
      k_trajectory_sorted<N, kRolloutSortLanes><<<grid_for(e.n, kRolloutSortLanes), kRolloutSortLanes, 0, e.stream>>>(
          a, steps);
#endif
    } else {
      note_launch("coup::np::k_step_trajectory<{}>", N);
      k_step_trajectory<N><<<grid_for(e.n, kThreads), kThreads, 0, e.stream>>>(a, steps);
    }
  });
}

hipError_t launch_rollout(const Env& e, int64_t steps, const coup_rollout_stats* stats) {
  if (e.n == 0 || steps == 0) return hipSuccess;
  RolloutArgs a{};
  a.sa = e.sa;
  a.sb = e.sb;
  a.n = e.n;
  a.seed_lo = e.seed_lo;
  a.seed_hi = e.seed_hi;
  a.env_id_base = e.env_id_base;
  a.steps = steps;
  a.err_count = e.err_count;
  if (stats) {
    (void)ep_acc_of(stats, a.ep);  // checked by the C ABI
    a.length_sum = stats->length_sum;
  }
  return dispatch(e.players, [&](auto np) {
    constexpr int N = decltype(np)::value;
    const unsigned grid = grid_for(e.n, kThreads);
    if (regroup_lanes(e.knobs, e.n)) {
#ifdef COUP_AB_VARIANTS
      switch (sort_lanes(e.knobs.np_sort_lanes, kRolloutSortLanes)) {
        case 512:
          note_launch("coup::np::k_rollout_sorted<{}, 512>", N);
          k_rollout_sorted<N, 512><<<grid_for(e.n, 512), 512, 0, e.stream>>>(a);
          break;
        case 256:
          note_launch("coup::np::k_rollout_sorted<{}, 256>", N);
          k_rollout_sorted<N, 256><<<grid, 256, 0, e.stream>>>(a);
          break;
        default:
          if (!e.knobs.np_scan)  // COUP_NP_SCAN=0: the per-lane bin prefix
            note_launch("coup::np::k_rollout_sorted<{}, 1024, false>", N),
                k_rollout_sorted<N, 1024, false><<<grid_for(e.n, 1024), 1024, 0, e.stream>>>(a);
          else
            note_launch("coup::np::k_rollout_sorted<{}, 1024>", N),
                k_rollout_sorted<N, 1024><<<grid_for(e.n, 1024), 1024, 0, e.stream>>>(a);
          break;
      }
#else
      note_launch("coup::np::k_rollout_sorted<{}, {}>", N, kRolloutSortLanes);
      k_rollout_sorted<N, kRolloutSortLanes><<<grid_for(e.n, kRolloutSortLanes), kRolloutSortLanes, 0, e.stream>>>(a);
#endif
    } else {
      note_launch("coup::np::k_rollout<{}>", N);
      k_rollout<N><<<grid, kThreads, 0, e.stream>>>(a);
    }
  });
}

hipError_t launch_apply(const Env& e, const int8_t* actions) {
  if (e.n == 0) return hipSuccess;
  return dispatch(e.players, [&](auto np) {
    constexpr int N = decltype(np)::value;
    k_apply<N><<<grid_for(e.n, kThreads), kThreads, 0, e.stream>>>(e.sa, e.sb, e.n, actions, e.err_count);
  });
}

hipError_t launch_query(const Env& e, const coup_query_outputs* out) {
  if (e.n == 0) return hipSuccess;
  QueryArgs a{};
  a.sa = e.sa;
  a.sb = e.sb;
  a.n = e.n;
  a.legal = out->legal_mask;
  a.cur_player = out->cur_player;
  a.terminal = out->terminal;
  a.rewards = out->rewards;
  a.returns = out->returns;
  return dispatch(e.players, [&](auto np) {
    constexpr int N = decltype(np)::value;
    k_query<N><<<grid_for(e.n, kThreads), kThreads, 0, e.stream>>>(a);
    if (out->obs) k_obs<N><<<grid_for(e.n, kObsLanes), kThreads, 0, e.stream>>>(e.sa, e.sb, e.n, out->obs);
  });
}

hipError_t launch_export(const Env& e, uint32_t* dst) {
  if (e.n == 0) return hipSuccess;
  k_export<<<grid_for(e.n, kThreads), kThreads, 0, e.stream>>>(e.sa, e.sb, e.n, reinterpret_cast<uint4*>(dst));
  return hipGetLastError();
}

hipError_t launch_import(const Env& e, const uint32_t* src) {
  if (e.n == 0) return hipSuccess;
  k_import<<<grid_for(e.n, kThreads), kThreads, 0, e.stream>>>(e.sa, e.sb, e.n,
                                                                reinterpret_cast<const uint4*>(src));
  return hipGetLastError();
}

}  // namespace np
}  // namespace coup

#ifdef COUP_TRAJ_PHASES
// Measurement builds (-DCOUP_TRAJ_PHASES): np::k_trajectory_sorted's
// per-phase shader cycles summed over waves, then wave-steps.
extern "C" int coup_debug_np_traj_phases(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_np_traj_phases), sizeof(g_np_traj_phases)) != hipSuccess) return 2;
  if (reset) {
    const unsigned long long z[kTrajPhases + 1] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_np_traj_phases), z, sizeof(z)) != hipSuccess) return 2;
  }
  return 0;
}
#endif
#ifdef COUP_COUNT_PHILOX
extern "C" int coup_debug_philox_counts_np(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_philox_counts), sizeof(unsigned long long) * 2) != hipSuccess) return 2;
  if (reset) {
    const unsigned long long z[2] = {0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_philox_counts), z, sizeof(z)) != hipSuccess) return 2;
  }
  return 0;
}
#endif
