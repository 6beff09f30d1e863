/*
 * coup_oracle.h -- CPU restatement of the reference Coup rules engine.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle for the MI355X
 * Coup environment.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it, and only as the checker / the timed CPU
 * baseline.  The product library (open_spiel_coup_amd/libcoup_mi355x.so)
 * never links, loads or calls anything in oracle/.
 *
 * What it restates (reference = BStarcheus/open_spiel_coup @ 2025-01-17):
 *   open_spiel/games/coup.h            constants, enums, state fields
 *   open_spiel/games/coup.cc           CoupState / CoupObserver / CoupGame
 *   open_spiel/spiel.cc:322-331        State::ApplyAction bookkeeping
 *   open_spiel/spiel.cc:371-377        State::LegalActionsMask
 *   open_spiel/observer.h:173-176      ContiguousAllocator zero-fill + offsets
 *   open_spiel/observer.h:287-297      kDefaultObsType / kInfoStateObsType
 * Pinning: the reference's own golden vectors (coup_test.cc known-answer
 * scenarios, integration_tests/playthroughs/coup.txt) -- see tests/golden/.
 * The reference C++ itself is NOT buildable here (abseil is not vendored),
 * so there is no oracle/_ref.
 *
 * The sampling contract (Philox4x32-10 keyed by seed/env id, one 32-bit
 * draw per history slot) is this project's own; see DESIGN.md section 4.
 */
#ifndef COUP_ORACLE_H_
#define COUP_ORACLE_H_

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OC_NUM_PLAYERS 2
#define OC_MAX_CARDS 4
#define OC_NUM_TYPES 5
#define OC_NUM_ACTIONS 18
#define OC_MAX_GAME_LENGTH 90
#define OC_MAX_CHANCE_IN_HISTORY 45
#define OC_MAX_MOVE_NUMBER (OC_MAX_GAME_LENGTH + OC_MAX_CHANCE_IN_HISTORY)
#define OC_OBS_SIZE 98
#define OC_INFO_SIZE 2492
#define OC_NONE (-1)

/* Card types (coup.h:50-57) */
enum { OC_ASSASSIN = 0, OC_AMBASSADOR, OC_CAPTAIN, OC_CONTESSA, OC_DUKE };
/* Card states (coup.h:59-63) */
enum { OC_FACEDOWN = 0, OC_FACEUP = 1 };
/* Actions (coup.h:65-85) */
enum {
  OC_INCOME = 0, OC_FOREIGN_AID, OC_COUP, OC_TAX, OC_ASSASSINATE, OC_EXCHANGE,
  OC_STEAL, OC_LOSE1, OC_LOSE2, OC_PASS, OC_BLOCK, OC_CHALLENGE,
  OC_XR12, OC_XR13, OC_XR14, OC_XR23, OC_XR24, OC_XR34
};

/* Error codes raised where the reference calls SpielFatalError / SPIEL_CHECK */
enum { OC_OK = 0, OC_ERR_ILLEGAL = 1, OC_ERR_PROGRESSION = 2, OC_ERR_TERMINAL = 3,
       OC_ERR_UNREPRESENTABLE = 4 /* valid in the reference, outside the packed record's fields */ };

typedef struct {
  int value; /* card type */
  int state; /* face down / up */
} oc_card;

typedef struct {
  oc_card cards[OC_MAX_CARDS];
  int ncards;
  int coins;
  int last_action; /* OC_NONE or action id */
  int lost_challenge;
} oc_player;

typedef struct {
  int deck[OC_NUM_TYPES];
  oc_player pl[OC_NUM_PLAYERS];
  int queue[8];
  int qlen;
  int turn_player;  /* cur_player_turn_ */
  int move_player;  /* cur_player_move_ */
  int opp_player;   /* opp_player_ */
  int turn_begin;
  int turn_number;
  int is_chance;
  int rewards[OC_NUM_PLAYERS];
  int move_number;
  int hist_len;
  int hist_player[OC_MAX_MOVE_NUMBER + 1];
  int hist_action[OC_MAX_MOVE_NUMBER + 1];
  int hist_deal_to[OC_MAX_MOVE_NUMBER + 1]; /* -1 unless a chance deal */
  int error;
} oc_state;

/* --- State API (one game) ------------------------------------------------ */
void oc_init(oc_state* s);
int oc_is_terminal(const oc_state* s);
int oc_current_player(const oc_state* s); /* -4 terminal, -1 chance */
int oc_legal_actions(const oc_state* s, int* out); /* returns count */
uint32_t oc_legal_mask(const oc_state* s);        /* bit a set if legal */
int oc_apply_action(oc_state* s, int action);      /* returns error code */
/* pyspiel's apply_action (no legality check); the state is unchanged on error */
int oc_apply_action_unchecked(oc_state* s, int action);
void oc_returns(const oc_state* s, int* out2);
void oc_rewards(const oc_state* s, int* out2);
int oc_chance_outcomes(const oc_state* s, int* actions, double* probs);
void oc_observation_tensor(const oc_state* s, int player, float* out98);
void oc_info_state_tensor(const oc_state* s, int player, float* out2492);
/* strings; return needed length (excl. NUL), write up to cap bytes */
int oc_observation_string(const oc_state* s, int player, char* buf, int cap);
int oc_info_state_string(const oc_state* s, int player, char* buf, int cap);
int oc_to_string(const oc_state* s, char* buf, int cap);
/* canonical 16-byte packed record, layout in DESIGN.md section 3 */
void oc_pack(const oc_state* s, uint32_t episode, uint32_t err, uint32_t* out4);
/* history as the product's 96 history bytes (entry i: [4:0] action / card,
 * [5] chance deal, [6] acting / receiving player; 0xFF past the end) */
void oc_history_bytes(const oc_state* s, uint8_t* out96);

/* --- Sampling contract --------------------------------------------------- */
void oc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
/* `episode` enters the counter as given; callers pass it masked to the
 * record's width (OC_EPISODE_MASK: 28 bits for 2 players; the N-player
 * record keeps 30, NP_EPISODE_MASK) */
uint32_t oc_draw(uint64_t seed, uint32_t env_id, uint32_t episode, uint32_t draw_idx);
#define OC_EPISODE_MASK 0xFFFFFFFu

/* --- Batched rollout driver (uniform random policy) ----------------------
 * Mirrors the batched step of the product: per lane and per step, sample a
 * legal action uniformly, apply it, resolve chance deals, and (auto_reset)
 * restart finished episodes.  Any output pointer may be NULL.
 *   actions[steps][n], rewards[steps][n][2], step_type[steps][n],
 *   legal[steps][n], obs[steps][n][2][98], final_state[n][4]
 * obs_overwrite: write obs at every step into the same obs[n][2][98] buffer
 * (the GPU env overwrites its obs buffer the same way).
 */
typedef struct {
  uint64_t seed;
  uint32_t env_id_base;
  int64_t n;
  int64_t steps;
  int auto_reset;
  int obs_overwrite;
  int8_t* actions;
  int8_t* rewards;
  uint8_t* step_type;
  uint32_t* legal;
  float* obs;
  float* info;             /* InformationStateTensor x2: [steps][n][2][2492] */
  uint32_t* final_state;
  uint8_t* final_hist;     /* [n][96] */
  int64_t* decisions;      /* total decisions applied (scalar) */
  int64_t* episodes_done;  /* total finished episodes (scalar) */
  int64_t* return_sum_p0;  /* sum of final returns of player 0 */
  int32_t* lane_episodes;  /* [n] episodes finished per lane (optional) */
  int32_t* lane_return_sum; /* [n] per lane: sum of player 0's final returns (optional) */
} oc_rollout_args;
int oc_rollout(const oc_rollout_args* a);

/* --- Every-lane window driver (the bench-size parity tests) ---------------
 * The same uniform rollout as oc_rollout (2 players) / np_rollout (N), with
 * only the steps [from, steps) recorded, in rows of `stride` lanes, so a
 * caller can split the lanes of one [steps - from][B] array over threads
 * (every pointer pre-offset to the chunk's first lane; n <= stride).
 * Tensors are not stored but reduced per lane and step to two linear hashes
 * of their fp32 bit patterns, h_j = sum_i bits(x_i) * w_j[i] (exact in 64
 * bits: w < 2^18, at most 2 x 2492 terms), which the GPU side computes the
 * same way.  Snapshots: the packed records and the per-lane episode counts /
 * player-0 return sums (counted from step stats_from) after snap_at[k] steps.
 */
#define OC_WINDOW_SNAPS 4
typedef struct {
  uint64_t seed;
  uint32_t env_id_base;   /* of this chunk's first lane */
  int players;            /* 2: coup_oracle.c; 3..6: the written N-player spec */
  int64_t n, steps, from, stride;
  int auto_reset;
  int8_t* actions;        /* [steps - from][stride] */
  int8_t* rewards;        /* [steps - from][stride][players] */
  uint8_t* step_type;     /* [steps - from][stride] */
  uint32_t* legal;        /* [steps - from][stride] */
  int8_t* cur_player;     /* [steps - from][stride] */
  const uint32_t* obs_w;  /* [2][2 * 98] (2 players) */
  uint64_t* obs_hash;     /* [steps - from][stride][2] */
  const uint32_t* info_w; /* [2][2 * 2492] */
  uint64_t* info_hash;    /* [steps - from][stride][2] */
  int64_t stats_from;
  int nsnap;
  int64_t snap_at[OC_WINDOW_SNAPS];
  uint32_t* snap_state[OC_WINDOW_SNAPS]; /* [stride][4] (2 players) or [stride][8] */
  int32_t* snap_eps[OC_WINDOW_SNAPS];    /* [stride] */
  int32_t* snap_ret[OC_WINDOW_SNAPS];    /* [stride] */
} oc_window_args;
int oc_rollout_window(const oc_window_args* a); /* players == 2 */

#ifdef __cplusplus
}
#endif
#endif /* COUP_ORACLE_H_ */
