/*
 * coup_mi355x.h -- C ABI of the MI355X-native batched Coup environment.
 *
 * One env handle = B independent 2-player Coup games ("lanes") whose state
 * lives in HBM as one 16-byte record per lane (layout: DESIGN.md section 3).
 * Every compute entry point runs on the GPU (gfx950 HIP kernels, one lane
 * per thread); there is no CPU fallback.  All array arguments are DEVICE
 * pointers owned by the caller (e.g. torch tensors' data_ptr()), laid out
 * lane-major ([B] or [B][...]).  Any output pointer may be NULL to skip it.
 * Work is enqueued on the env's HIP stream (coup_set_stream); calls are
 * asynchronous unless stated otherwise.  Return value: 0 on success,
 * otherwise a COUP_E_* code with a message in coup_last_error().
 *
 * Reference interfaces replaced (BStarcheus/open_spiel_coup):
 *   open_spiel::Game / State virtual API     open_spiel/spiel.h:210-1035
 *   CoupGame / CoupState                     open_spiel/games/coup.h:111-231
 *   pure C ABI pattern for Game/State        open_spiel/rust/src/rust_open_spiel.h:24-84
 *   rl_environment.Environment reset/step    open_spiel/python/rl_environment.py:282-367
 *   SyncVectorEnv step(reset_if_done)        open_spiel/python/vector_env.py:40-78
 */
#ifndef COUP_MI355X_H_
#define COUP_MI355X_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define COUP_ABI_VERSION 14

#define COUP_NUM_PLAYERS 2          /* coup.h:42 */
#define COUP_MAX_PLAYERS 6          /* N-player extension */
#define COUP_NUM_ACTIONS 18         /* coup.h:203 NumDistinctActions */
#define COUP_NUM_CARD_TYPES 5       /* coup.h:44, MaxChanceOutcomes */
#define COUP_OBS_SIZE 98            /* coup.cc:1118-1130 ObservationTensorShape */
#define COUP_INFO_STATE_SIZE 2492   /* coup.cc:1104-1116 InformationStateTensorShape */
#define COUP_MAX_GAME_LENGTH 90     /* coup.h:219 */
#define COUP_STATE_BYTES 16         /* packed lane record */
#define COUP_HISTORY_BYTES 96       /* per-lane history: one byte per history index */
#define COUP_NP_STATE_BYTES 32      /* N-player engine lane record */

/* coup_create flags */
#define COUP_FLAG_AUTO_RESET 1      /* SyncVectorEnv(reset_if_done=True) semantics */
#define COUP_FLAG_HISTORY 2         /* keep per-lane histories (InformationStateTensor, strings) */
#define COUP_FLAG_GENERIC 4         /* use the N-player engine also at N = 2 (cross-checks) */
#define COUP_FLAG_UNCHECKED 8       /* caller actions (coup_step, coup_step_host, coup_apply_action) outside
                                       LegalActions() are applied as pyspiel's apply_action does (no legality
                                       check, DoApplyAction's own checks decide; COUP_SLOT_UNCHECKED); 2 players */

/* rl_environment.StepType (rl_environment.py:96-103) */
#define COUP_STEP_FIRST 0
#define COUP_STEP_MID 1
#define COUP_STEP_LAST 2
#define COUP_STEP_SKIPPED 3        /* coup_step with actions[i] < 0: lane i left untouched */

/* open_spiel player ids (spiel_globals.h:28,34) */
#define COUP_CHANCE_PLAYER (-1)
#define COUP_TERMINAL_PLAYER (-4)

/* Bit set in coup_query's legal mask at chance nodes: bits 0..4 are then the
 * card types with a non-zero deck count (LegalActionsMask(kChancePlayerId),
 * spiel.cc:371-377). */
#define COUP_MASK_CHANCE_FLAG (1u << 31)

/* error codes */
#define COUP_OK 0
#define COUP_E_INVALID 1    /* bad argument (null env, bad batch, ...) */
#define COUP_E_HIP 2        /* HIP runtime error */
#define COUP_E_LANES 3      /* one or more lanes rejected an action (see coup_error_count) */

typedef struct coup_env coup_env;

/* Shapes below are for the 2-player game.  An env of N players
 * (coup_create_ex) has rewards / returns [B][N] and obs [B][N][49N]
 * (the N-player ObservationTensor); its records are
 * COUP_NP_STATE_BYTES long and it has no history / info_state. */

/* Outputs of one batched env step; every pointer optional (NULL = skip). */
typedef struct {
  int8_t* actions;      /* [B]  decision action applied this step (-1: lane was reset) */
  int8_t* rewards;      /* [B][2] Rewards() after the step (coup.cc:1012) */
  uint8_t* step_type;   /* [B]  COUP_STEP_* */
  uint32_t* legal_mask; /* [B]  bit a set iff a in LegalActions() of the current player */
  int8_t* cur_player;   /* [B]  CurrentPlayer() of the (post-reset) state */
  float* obs;           /* [B][2][98] ObservationTensor(p) for p = 0, 1 */
  float* info_state;    /* [B][2][2492] InformationStateTensor(p) (needs COUP_FLAG_HISTORY) */
  /* Per-episode accumulators: for a lane whose episode ends in this step
   * (step type LAST), episodes[i] += 1 and return_sum[i] += Returns()[0] of
   * the finished game (coup.cc:1016-1032), read before an auto-reset; other
   * lanes keep their values.  The multi-GPU bench all-gathers them
   * (SURVEY.md 8(e)).  Both or neither. */
  int32_t* episodes;    /* [B] */
  int32_t* return_sum;  /* [B] */
  /* The same accumulators packed into ONE word per lane (instead of
   * episodes / return_sum, not with them): return_sum << 8 | episodes as
   * int16 (episode_word_bytes = 2) or return_sum << 16 | episodes as int32
   * (4), two's complement, updated by adding (return << S) + 1 at each
   * finished episode.  The word is the all-gather payload as it stands
   * (2 bytes per lane each way at 2 bytes).  Fields do not saturate: the
   * caller bounds the steps between clears (int16: <= 255 episodes and
   * |return_sum| <= 127, i.e. 2 (N - 1) K <= 127). */
  void* episode_word;          /* [B] int16 or int32 */
  int32_t episode_word_bytes;  /* 2 or 4 when episode_word != NULL */
} coup_step_outputs;

/* Per-lane query of the current state (State accessors); all optional. */
typedef struct {
  uint32_t* legal_mask; /* [B] decision mask, or chance mask | COUP_MASK_CHANCE_FLAG */
  int8_t* cur_player;   /* [B] CurrentPlayer() (coup.cc:458-466) */
  uint8_t* terminal;    /* [B] IsTerminal() (coup.cc:989-1010) */
  int8_t* rewards;      /* [B][2] Rewards() (coup.cc:1012-1014) */
  int8_t* returns;      /* [B][2] Returns() (coup.cc:1016-1032) */
  float* obs;           /* [B][2][98] ObservationTensor (coup.cc:1051-1056) */
  float* info_state;    /* [B][2][2492] InformationStateTensor (coup.cc:1044-1049); needs COUP_FLAG_HISTORY */
} coup_query_outputs;

/* Result of coup_slot_op for its lane (128 bytes, host memory). */
typedef struct {
  uint32_t record[4];    /* packed lane record (coup_export_state layout) */
  uint8_t history[96];   /* history bytes (coup_export_history layout) */
  uint32_t legal_mask;   /* as coup_query_outputs.legal_mask */
  int8_t cur_player;     /* CurrentPlayer() (coup.cc:458-466) */
  uint8_t terminal;      /* IsTerminal() (coup.cc:989-1010) */
  uint8_t ok;            /* 0: the action was rejected (lane left unchanged) */
  uint8_t unrepresentable; /* with ok = 0 under COUP_SLOT_UNCHECKED: the reference's DoApplyAction ACCEPTS the
                              action, but its result leaves the packed record's fields (a 16th coin, an unsorted
                              3-4 card hand) -- a known parity gap, not a reference raise */
  int8_t rewards[2];     /* Rewards() (coup.cc:1012-1014) */
  int8_t returns[2];     /* Returns() (coup.cc:1016-1032) */
  uint8_t pad[4];
} coup_slot_result;

/* coup_slot_op flags */
#define COUP_SLOT_INIT 1       /* put the lane in NewInitialState() first (coup.cc:393-428) */
#define COUP_SLOT_OBS 2        /* append ObservationTensor [2][98] float to the result */
#define COUP_SLOT_INFO 4       /* append InformationStateTensor [2][2492] float (after obs if both) */
#define COUP_SLOT_NO_RESULT 8  /* asynchronous: no result, host_out may be NULL */
#define COUP_SLOT_RESET 16     /* first, start the lane's next episode (coup_reset on the lane: episode + 1,
                                  NewInitialState); not with src_env or COUP_SLOT_INIT */
#define COUP_SLOT_DEAL 32      /* last, resolve the pending chance deals under the sampling contract of the
                                  lane's stream (seed, env_id_base + lane): rl_environment's chance sampling
                                  until a decision node (rl_environment.py:369-382); entries to the history */
#define COUP_SLOT_UNCHECKED 64 /* apply `action` as pyspiel's apply_action (pyspiel.cc:266, spiel.cc:322-331): no
                                  LegalActions() check, DoApplyAction's own checks decide (coup.cc:490-809);
                                  result.ok = 0, the lane untouched, where the reference raises, on a terminal
                                  state, or where the result leaves the record's fields (then
                                  result.unrepresentable = 1) */

/* One request of coup_slot_ops (24 bytes): the op coup_slot_op would run on
 * lane `lane` with src_lane (< 0: no copy), action (< 0: none) and flags
 * (COUP_SLOT_INIT / COUP_SLOT_UNCHECKED; the output flags are per call). */
typedef struct {
  int64_t lane;
  int64_t src_lane;
  int32_t action;
  int32_t flags;
} coup_slot_req;

/* Per-lane rollout statistics accumulated by coup_rollout (device, [B]). */
typedef struct {
  int32_t* episodes;    /* [B] episodes finished */
  int32_t* return_sum;  /* [B] sum over finished episodes of player 0's return */
  int32_t* length_sum;  /* [B] sum over finished episodes of decisions taken */
  /* episodes / return_sum packed as coup_step_outputs.episode_word (instead
   * of the pair, not with it) */
  void* episode_word;
  int32_t episode_word_bytes;
} coup_rollout_stats;

/* ABI version of the loaded library (== COUP_ABI_VERSION). */
int coup_abi_version(void);
/* Message of the last failing call on this thread ("" if none). */
const char* coup_last_error(void);

/* Create an env of `batch` lanes on the current HIP device.  Lane i uses the
 * global env id env_id_base + i for its random streams, so a batch split over
 * ranks by id range reproduces the single-GPU trajectories bit for bit.
 * Ids are 32-bit: env_id_base + batch must not exceed 2^32 (COUP_E_INVALID
 * otherwise, instead of lanes silently sharing streams).
 * flags: COUP_FLAG_AUTO_RESET -- SyncVectorEnv(reset_if_done=True) semantics
 * (a finished lane restarts inside the same step); without it rl_environment
 * semantics (LAST, then the next step resets).  COUP_FLAG_HISTORY -- keep a
 * [B][96]-byte history (entry i = history index i: bits [4:0] action or card
 * type, [5] chance deal, [6] acting / receiving player), needed for the
 * InformationStateTensor.  The env starts with every lane reset and dealt
 * (rl_environment.reset, rl_environment.py:324-367).  Synchronous. */
int coup_create(int64_t batch, uint64_t seed, uint32_t env_id_base, int flags, coup_env** out);
/* coup_create with a player count: 2 is the reference game; 3..6 (and 2
 * with COUP_FLAG_GENERIC) run the N-player extension, whose rules reduce to
 * the reference's at N = 2 (the reference game is 2-player only, coup.h:42;
 * DESIGN.md section 11 has the extension's rules).  Synchronous. */
int coup_create_ex(int64_t batch, uint64_t seed, uint32_t env_id_base, int flags, int num_players, coup_env** out);
int coup_destroy(coup_env* env);
/* Re-read the env's dispatch knobs from the environment variables
 * coup_create reads them from (COUP_OBS_SPLIT, COUP_INFO_SPLIT,
 * COUP_REGROUP, COUP_PIPE, COUP_TRAJ_CHUNK; in a measurement build also the
 * A/B variant knobs): for tests and A/B runs that switch one existing env
 * between forms.  Launches never read the environment themselves.  (The
 * rules-trajectory record buffer keeps the size coup_create gave it: a larger
 * COUP_TRAJ_CHUNK is capped to it.) */
int coup_reload_knobs(coup_env* env);
/* Use this HIP stream (hipStream_t, may be NULL = default) for later calls. */
int coup_set_stream(coup_env* env, void* hip_stream);
int64_t coup_batch(const coup_env* env);
/* NumPlayers() (coup.h:205) of the env, and its lane record size in bytes. */
int coup_num_players(const coup_env* env);
int coup_state_bytes(const coup_env* env);

/* Reset lanes (all if lane_mask == NULL, else lanes with lane_mask[i] != 0):
 * next episode, fresh CoupState, chance deals resolved (FIRST step). */
int coup_reset(coup_env* env, const uint8_t* lane_mask);

/* One batched rl_environment step.  actions: [B] decision actions (int8),
 * or NULL to draw each lane's action uniformly from its legal set under the
 * sampling contract (random_agent.py:29-42).  Per lane: apply the action
 * (State::ApplyAction, spiel.cc:322-331), resolve the chance deals that
 * follow (rl_environment.py:369-382), report rewards / step type, reset a
 * finished lane (see auto_reset) and write the post-step legal mask and
 * observations.  An illegal action leaves the lane unchanged and counts in
 * coup_error_count.  A negative action skips the lane: it is left untouched
 * (no reset, no deals, no error), reports action -1, rewards 0 and step type
 * COUP_STEP_SKIPPED, and its legal mask / observations describe its current
 * state -- so one launch steps any subset of the lanes (SyncVectorEnv over
 * per-game environments, vector_env.py:40-67). */
int coup_step(coup_env* env, const int8_t* actions, const coup_step_outputs* out);

/* coup_step_host flags */
#define COUP_HOST_OBS 1   /* also return ObservationTensor [B][P][49P] */
#define COUP_HOST_INFO 2  /* also return InformationStateTensor [B][2][2492] (COUP_FLAG_HISTORY) */
#define COUP_HOST_ACTIVE 4  /* tensors only for the lanes whose action is >= 0 (2 players, actions
                               not NULL): m rows in lane order, obs [m][2][98] at off[5], then info
                               [m][2][2492] at off[5] + align16(m * 784) -- one env of a shared
                               SyncVectorEnv env stepping alone copies its own rows, not B */

/* coup_step for small batches that want the answers on the host (the
 * per-game rl_environment.Environment and SyncVectorEnv, rl_environment.py:
 * 282-322): `actions` is a HOST [B] int8 array (or NULL: uniform policy;
 * negative entries skip lanes as in coup_step).  The step kernel writes its
 * outputs straight into mapped pinned host memory and the call synchronises
 * the env's stream -- one launch, no query kernel (with COUP_HOST_INFO the
 * outputs are staged in device memory and brought over by one copy, which
 * beats stores over the host link for 19,936 bytes per lane).  host_out
 * receives, in sections starting at the offsets coup_step_host_layout
 * returns (16-byte aligned): legal_mask uint32 [B], cur_player int8 [B],
 * step_type uint8 [B], rewards int8 [B][P], actions int8 [B], then the
 * tensors `want` asks for (obs before info_state). */
int coup_step_host(coup_env* env, const int8_t* actions, int want, void* host_out);
/* Section offsets off[0..5] of coup_step_host's output and its total size in
 * bytes, for `batch` lanes of `num_players` players. */
size_t coup_step_host_layout(int64_t batch, int num_players, int want, size_t* off);

/* `steps` uniform-random env steps per lane (the coup_step of actions ==
 * NULL, with the env's auto-reset setting), every step's outputs stored:
 * out's actions / rewards / step_type / legal_mask / cur_player (and obs /
 * info_state) point to [steps][B][...] buffers (slice t = step t, laid out
 * as coup_step's [B][...]); episodes / return_sum / episode_word are [B]
 * accumulators as in coup_step.  Results equal `steps` coup_step calls --
 * the trajectory a learner collects (rl_environment.py:282-322 per step).
 * Without tensors: ONE launch, the state kept in registers (the env must not
 * keep histories, COUP_E_INVALID), lanes regrouped by decision every step
 * from 2^18 lanes.  With obs: coup_step_many's
 * rules-trajectory split step where it applies (from 2^20 lanes), else one
 * coup_step per slice; info_state needs COUP_FLAG_HISTORY and takes
 * coup_step per slice. */
int coup_step_trajectory(coup_env* env, int64_t steps, const coup_step_outputs* out);

/* `steps` calls of coup_step(env, NULL, out) -- uniform-random policy, every
 * step writing the same output buffers -- as one call, with the same results
 * (outputs of the last step, records, accumulators, error count), every
 * step's outputs stored (over the same buffers).  Forms (DESIGN.md
 * section 5):
 * - without tensors or history (2 and N players): ONE trajectory launch for
 *   the steps (coup_step_trajectory's kernels, output stride 0);
 * - the split observation step (2-player lanes with obs and no history, from
 *   2^20 lanes: coup_obs_split_variant): chunks of up to COUP_TRAJ_CHUNK
 *   (default 8) steps as one regrouped rules-trajectory launch that stores
 *   every step's records to a per-env buffer, then the address-order writer
 *   once per step from them;
 * - otherwise one coup_step per step.
 * COUP_PIPE=0 at coup_create keeps one coup_step per step (A/B).  May be
 * captured into a HIP graph (no allocation, no synchronisation). */
int coup_step_many(coup_env* env, int64_t steps, const coup_step_outputs* out);

/* `steps` uniform-random env steps per lane in one launch, state kept in
 * registers (auto-reset always on); per-lane statistics are accumulated
 * into `stats` (optional).  Not available with COUP_FLAG_HISTORY. */
int coup_rollout(coup_env* env, int64_t steps, const coup_rollout_stats* stats);

/* --- open_spiel::State surface, one action per lane -------------------- */

/* Put lanes (mask as in coup_reset) in NewInitialState() (coup.cc:393-428):
 * a chance node with four deals pending, episode counter advanced. */
int coup_new_initial_state(coup_env* env, const uint8_t* lane_mask);
/* State::ApplyAction (spiel.cc:322-331) per lane, decision or chance outcome;
 * actions[i] < 0 leaves lane i untouched.  No chance auto-resolution. */
int coup_apply_action(coup_env* env, const int8_t* actions);
/* Per-lane accessors of the current state. */
int coup_query(coup_env* env, const coup_query_outputs* out);

/* Lane-pool op of the per-game State facade: one launch on one lane of a
 * 2-player COUP_FLAG_HISTORY env, the lane standing for one open_spiel
 * State.  In order: if src_env is not NULL, lane `lane` becomes a copy of
 * src_env's lane `src_lane` (State::Clone, spiel.h:822; src_env may be env);
 * COUP_SLOT_INIT resets it to NewInitialState (coup.cc:393-428, history
 * cleared); action >= 0 applies State::ApplyAction (spiel.cc:322-331) --
 * an illegal action leaves the lane unchanged and sets result.ok = 0, the
 * SpielError of coup.cc:492-495 & co; then, unless COUP_SLOT_NO_RESULT,
 * the lane's coup_slot_result (followed by the tensors the flags ask for)
 * is copied to host_out and the call synchronises the env's stream.
 * Replaces the per-state calls of the reference's C ABI
 * (rust_open_spiel.h:34-73: StateClone, StateApplyAction,
 * StateLegalActions, StateCurrentPlayer, StateIsTerminal, StateReturns,
 * StateObservationTensor, StateInformationStateTensor) with one round trip. */
int coup_slot_op(coup_env* env, int64_t lane, const coup_env* src_env, int64_t src_lane, int action, int flags,
                 void* host_out);

/* n independent coup_slot_op requests (host array `reqs`) in one launch --
 * e.g. all children of a Deep CFR traverser node (deep_cfr.py:440-471:
 * state.child(a) for every legal a) or one action on each state of a
 * frontier.  Copies read src_env (may be env; NULL only if no request
 * copies).  Requests must be independent: destination lanes distinct, and
 * no destination lane the source of another request when src_env == env
 * (COUP_E_INVALID otherwise).  flags: COUP_SLOT_OBS / COUP_SLOT_INFO /
 * COUP_SLOT_NO_RESULT for every request.  Unless COUP_SLOT_NO_RESULT,
 * host_out receives n coup_slot_result, then (COUP_SLOT_OBS) n x [2][98]
 * floats, then (COUP_SLOT_INFO) n x [2][2492] floats, and the call
 * synchronises the env's stream. */
int coup_slot_ops(coup_env* env, int64_t n, const coup_slot_req* reqs, const coup_env* src_env, int flags,
                  void* host_out);

/* --- host-resident per-game states --------------------------------------- */

/* A single State op is ~0.1 us of integer code; a device round trip is a
 * PCIe crossing each way (the op server above: ~7 us).  For the per-state
 * callers of rust_open_spiel.h:34-73 / pyspiel.cc:263-345 (one op per node:
 * outcome_sampling_mccfr.py:81-87, deep_cfr.py:440-444) the library also
 * runs the SAME rules (coup_lane.h) and tensor decoders (coup_tensor.h) on
 * the host, over a coup_slot_result as the state (record, history bytes and
 * the answers), so a host state and a device lane convert with one copy
 * (coup_slot_op's result one way, coup_write_lane the other).  Batched work
 * stays on the device.  These run on the calling thread; no HIP call. */
int coup_host_state_init(coup_slot_result* out);                    /* NewInitialState (coup.cc:393-428) */
/* State::ApplyAction on `in` into `out` (may alias): flags COUP_SLOT_UNCHECKED
 * as pyspiel's apply_action (spiel.cc:322-331, no legality check), else with
 * it; ok / unrepresentable exactly as coup_slot_op reports them. */
int coup_host_state_apply(const coup_slot_result* in, int action, int flags, coup_slot_result* out);
/* ObservationTensor [2][98] and / or InformationStateTensor [2][2492] of
 * both players (either pointer may be NULL; coup.cc:1044-1056). */
int coup_host_state_tensors(const coup_slot_result* st, float* obs, float* info);
/* rl_environment's lane ops on a host state (coup_slot_op's COUP_SLOT_RESET /
 * COUP_SLOT_DEAL semantics): mode COUP_SLOT_INIT starts from the lane
 * coup_create leaves (in may be NULL), COUP_SLOT_RESET the next episode,
 * then `action` (< 0: none; COUP_SLOT_UNCHECKED as pyspiel's apply_action),
 * then COUP_SLOT_DEAL the pending chance deals under the sampling contract of
 * stream (seed, env_id) -- the draws the env's device lane would use. */
int coup_host_state_step(const coup_slot_result* in, int action, int mode, uint64_t seed, uint32_t env_id,
                         coup_slot_result* out);
/* ObservationString(player) (kind 0), InformationStateString(player) (1) --
 * CoupObserver::StringFrom, coup.cc:290-373 -- or ToString() (2, coup.cc:
 * 945-987) of st into buf (cap bytes, NUL-terminated when it fits).  Returns
 * the length (>= cap: truncated), -1 for a bad argument. */
int64_t coup_host_state_string(const coup_slot_result* st, int kind, int player, char* buf, int64_t cap);
/* Write host state `src` (its record and history bytes) into lane `lane` of
 * a 2-player COUP_FLAG_HISTORY env (State::SetState-style migration to the
 * device), ordered after the env's pending stream and server work. */
int coup_write_lane(coup_env* env, int64_t lane, const coup_slot_result* src);

/* --- device-resident op server ------------------------------------------ */

/* A resident wave that runs coup_slot_op requests without kernel launches
 * (DESIGN.md section 12).  It runs on its own non-blocking HIP stream of the
 * current device and polls a ring of requests in mapped, coherent pinned host
 * memory; an answered op is one host write the wave sees, the op, and one
 * device->host write the host sees.  coup_slot_op on an env attached to a
 * server (coup_attach_server), whose src_env is NULL or attached to the same
 * server, goes through it; other entry points on such an env first wait for
 * the server's pending requests, and the server waits for (synchronises) work
 * enqueued on the env's stream before it reads the env's lanes, so the two
 * paths stay ordered.  The wave leaves after idle_us microseconds without a
 * request, on coup_server_destroy, on coup_destroy of any env (freeing
 * memory synchronises the device, which would otherwise wait out the idle
 * time), or when the host finds it idle; the next request relaunches it.
 * While a wave idles, a device-wide synchronisation (hipDeviceSynchronize,
 * torch.cuda.synchronize) waits for it to leave: at most idle_us (the Python
 * pool's default is 2000, COUP_SERVER_IDLE_US).  The server's host side is
 * serialised by a lock of its own (a post, its wait and the copy of its
 * result are one section), so ops on envs sharing a server may come from
 * several threads; calls on one env are still not reentrant.  Each request
 * carries a checksum the wave verifies, so a torn read of its ring slot is
 * polled again instead of served.  Replaces, for the per-state callers of
 * rust_open_spiel.h:34-73 / pyspiel.cc:263-345, the launch-and-synchronise
 * round trip of each State op. */
typedef struct coup_server coup_server;
int coup_server_create(int64_t idle_us, coup_server** out);
/* Serves the pending requests, stops the wave and frees the server.  Detach
 * (or destroy) its envs first. */
int coup_server_destroy(coup_server* srv);
/* Route env's coup_slot_op through srv (NULL detaches).  env: 2-player,
 * COUP_FLAG_HISTORY. */
int coup_attach_server(coup_env* env, coup_server* srv);
/* out[0] requests served, out[1] wave launches, out[2] a wave may be running,
 * out[3] idle_us. */
int coup_server_stats(const coup_server* srv, uint64_t* out);

/* Copy the packed lane records ([B][coup_state_bytes / 4] uint32, device)
 * out of / into the env. */
int coup_export_state(coup_env* env, uint32_t* dst);
int coup_import_state(coup_env* env, const uint32_t* src);
/* Copy the per-lane histories ([B][96] bytes, device; COUP_FLAG_HISTORY). */
int coup_export_history(coup_env* env, uint8_t* dst);
int coup_import_history(coup_env* env, const uint8_t* src);

/* Number of lanes that rejected an action since the last call (resets the
 * counter).  Synchronises the env's stream. */
int coup_error_count(coup_env* env, int64_t* out);

/* --- measurement ------------------------------------------------------- */

/* The memory traffic of one observation-writing 2-player step over `batch`
 * lanes with no rules in between: every lane's 16-byte record is loaded and
 * stored back unchanged, and the action, rewards, step type, legal mask,
 * current player and [B][2][98] float observation buffers are written in the
 * step kernel's order (same grid, same XCD-aware block -> lane-group
 * mapping, same wave-cooperative sc1 buffer stores).  Timing it beside
 * coup_step in one process gives that step's store-pattern ceiling on the
 * box at hand (bench.py: roofline.store_ceiling_ms).  `records` is a device
 * buffer of batch x 16 bytes; the output pointers are as in
 * coup_step_outputs (any may be NULL).  Asynchronous on `hip_stream`. */
int coup_measure_step_traffic(int64_t batch, uint32_t* records, const coup_step_outputs* out, void* hip_stream);

/* Measurement helper: the split writers' store pattern with no decode --
 * n_float4 float4 of the device buffer dst written in address order by
 * blocks of `threads` threads, `passes` float4 per thread (the grid of
 * k_obs_sweep_rows<512, 2> / k_info_sweep<1024, 2>: threads x passes =
 * 512 x 2 or 1024 x 2; a measurement build takes more shapes, and with
 * COUP_SWEEP_RESIDENT in `mode` a grid-stride form from a resident grid),
 * non-temporal.  Its duration is those writers' store ceiling on the box at
 * hand (bench.py: roofline.store_ceiling_ms of the split steps).  The data:
 * tensor-like (0.0 with a 1.0 in one float of 32), or with
 * COUP_SWEEP_INDEX_BITS every float the float4's index bits (HBM store time
 * depends on the data).  Asynchronous on `hip_stream`. */
#define COUP_SWEEP_RESIDENT 1
#define COUP_SWEEP_INDEX_BITS 2
int coup_measure_store_sweep(float* dst, int64_t n_float4, int threads, int passes, int mode, void* hip_stream);

/* Measurement helper: the observation-step form coup_step uses for a batch
 * of `batch` 2-player lanes with observations and no information state --
 * 0 the fused step kernel, > 0 the split form's writer variant (the rules
 * step without tensors, then the observations in address order; DESIGN.md
 * section 5).  COUP_OBS_SPLIT overrides it. */
int coup_obs_split_variant(int64_t batch);

/* The same for the InformationStateTensor step (2-player lanes with the
 * information state and no observations): 0 the fused step kernel, > 0 the
 * split form's k_info_sweep shape.  COUP_INFO_SPLIT overrides it. */
int coup_info_split_variant(int64_t batch);

/* What this build of the library holds: 0 the product (the shipped kernels
 * only), COUP_BUILD_AB_VARIANTS a measurement build that also instantiates
 * every measured-and-rejected kernel variant, selected by environment
 * variables read at coup_create (build.py writes it to
 * build/ab/libcoup_mi355x.so for A/B runs and their equality tests). */
#define COUP_BUILD_AB_VARIANTS 1
/* Bits 3:1: how the 2-player rules trajectories store each step's outputs
 * (their STAGE template argument): 0 from the thread
 * that played the lane, 2 staged by lane in LDS and stored by the lane's
 * home thread behind the next step's count barrier (a measurement build). */
#define COUP_BUILD_TRAJ_STAGE_SHIFT 1
#define COUP_BUILD_TRAJ_STAGE_MASK 0x7
int coup_build_flags(void);

/* The kernels this thread's library calls have launched -- enqueued, or
 * recorded into a HIP graph being captured -- since the log was last reset:
 * in first-launch order, repeats collapsed, joined by " + ", spelled as
 * bench.py's roofline.kernel spells them (rocprofv3 prints the same kernels
 * with their defaulted template arguments written out).  The step, step_many,
 * trajectory and rollout paths of both engines note their launches.  Writes
 * up to cap - 1 bytes and a NUL to buf (may be null), returns the full
 * length; reset != 0 clears the log after reading it.  Host bookkeeping only
 * (ABI 14: the every-lane parity tests assert with it that they ran the
 * kernels the bench line names). */
int coup_launch_log(char* buf, int cap, int reset);

#ifdef __cplusplus
}
#endif
#endif /* COUP_MI355X_H_ */
