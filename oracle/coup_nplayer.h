/*
 * coup_nplayer.h -- CPU specification of the N-player Coup extension (2..6).
 *
 * TEST INFRASTRUCTURE ONLY (same rules as coup_oracle.h).  The reference is
 * 2-player only (open_spiel/games/coup.h:42; coup.cc:45-46), so N > 2 has no
 * reference semantics: this file is the written specification of this
 * project's extension, and the GPU's N-player kernels
 * are checked against it ("parity unpinned" with respect to the reference).
 * At N = 2 the rules reduce to the reference's exactly, which the tests
 * check against the 2-player oracle and the reference's golden data.
 *
 * Generalisation (each rule reduces to the 2-player one):
 *   - seats 0..N-1; "next alive after p" skips eliminated players;
 *   - Coup, Assassinate and Steal target the next alive player after the
 *     turn player (the 18-action space has no target argument);
 *   - Foreign Aid, Tax and Exchange are answered by every other alive player
 *     in seat order after the turn player until one blocks / challenges;
 *     targeted actions are answered by the target only;
 *   - the counterpart O of the player to move M is explicit: NextPlayerMove
 *     swaps M and O; NextPlayerTurn moves the turn to the next alive seat;
 *   - a lost card gives -(N-1) to its owner and +1 to every other player;
 *     returns_p = sum_{q != p} faceup_q - (N-1) faceup_p (zero-sum);
 *   - starting coins: 1 and 2 at N = 2 (coup.cc:407-420), 2 each otherwise;
 *   - MaxGameLength = 45 N (90 at N = 2, coup.h:219);
 *   - initial deals go round the table twice (0,1,..,N-1,0,1,..).
 */
#ifndef COUP_NPLAYER_H_
#define COUP_NPLAYER_H_

#include <stdint.h>

#include "coup_oracle.h" /* oc_window_args */

#ifdef __cplusplus
extern "C" {
#endif

#define NP_MAX_PLAYERS 6
#define NP_MAX_HIST 300
#define NP_EPISODE_MASK 0x3FFFFFFFu /* 30-bit episode counter of the N-player record */

typedef struct {
  int value, state;
} np_card;

typedef struct {
  np_card cards[4];
  int ncards, coins, last_action, lost_challenge;
} np_player;

typedef struct {
  int n;
  int deck[5];
  np_player pl[NP_MAX_PLAYERS];
  int queue[8], qlen;
  int init_left;  /* initial deals still to make */
  int T, M, O, begin, turn, move;
  int rewards[NP_MAX_PLAYERS];
  int error;
} np_state;

void np_init(np_state* s, int n);
int np_is_terminal(const np_state* s);
int np_current_player(const np_state* s);
uint32_t np_legal_mask(const np_state* s); /* chance: card mask | 1u<<31 */
int np_apply_action(np_state* s, int a);    /* 0 ok, else error code */
void np_returns(const np_state* s, int* out);
int np_obs_size(int n);                     /* 49 n */
void np_observation_tensor(const np_state* s, int player, float* out);
/* 32-byte record (8 x u32), layout in DESIGN.md section 11 */
void np_pack(const np_state* s, uint32_t episode, uint32_t* out8);

/* uniform-random rollout under the sampling contract (coup_oracle.h) */
typedef struct {
  int n_players;
  uint64_t seed;
  uint32_t env_id_base;
  int64_t n, steps;
  int auto_reset;
  int8_t* actions;     /* [steps][n] */
  int8_t* rewards;     /* [steps][n][P] */
  uint8_t* step_type;  /* [steps][n] */
  uint32_t* legal;     /* [steps][n] */
  float* obs;          /* [steps][n][P][49P] or NULL */
  uint32_t* final_state; /* [n][8] */
  int64_t* episodes_done;
  int64_t* return_sum_p0;
  int32_t* lane_episodes;   /* [n] per lane (optional) */
  int32_t* lane_return_sum; /* [n] per lane (optional) */
  int8_t* cur_player;       /* [steps][n] CurrentPlayer() after the step (optional) */
} np_rollout_args;
int np_rollout(const np_rollout_args* a);
/* the every-lane window driver (oc_window_args, coup_oracle.h) for 3..6
 * players (no tensor hashes: the N-player benches write no tensors) */
int np_rollout_window(const oc_window_args* a);

#ifdef __cplusplus
}
#endif
#endif /* COUP_NPLAYER_H_ */
