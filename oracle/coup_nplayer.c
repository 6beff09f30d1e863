/*
 * coup_nplayer.c -- CPU specification of the N-player Coup extension.
 * TEST INFRASTRUCTURE ONLY; see coup_nplayer.h for the rules and scope.
 * The structure follows coup_oracle.c (itself a restatement of coup.cc);
 * comments cite the reference line each generalised rule comes from.
 */
#include "coup_nplayer.h"

#include <string.h>

#include "coup_oracle.h" /* action / card ids, oc_draw */

static int max_len(const np_state* s) { return 45 * s->n; }

static void sort_hand(np_player* p) {
  for (int i = 1; i < p->ncards; ++i) {
    np_card c = p->cards[i];
    int j = i - 1;
    while (j >= 0 && (c.value < p->cards[j].value ||
                      (c.value == p->cards[j].value && c.state < p->cards[j].state))) {
      p->cards[j + 1] = p->cards[j];
      --j;
    }
    p->cards[j + 1] = c;
  }
}

static void erase_card(np_player* p, int idx) {
  for (int i = idx; i + 1 < p->ncards; ++i) p->cards[i] = p->cards[i + 1];
  p->ncards--;
}

static int has_face_down(const np_player* p, int v) {
  for (int i = 0; i < p->ncards; ++i)
    if (p->cards[i].value == v && p->cards[i].state == OC_FACEDOWN) return 1;
  return 0;
}

static int alive(const np_state* s, int p) {
  /* coup.cc:994-1006 */
  const np_player* pl = &s->pl[p];
  if (pl->ncards < 2) return 1;
  for (int i = 0; i < pl->ncards; ++i)
    if (pl->cards[i].state == OC_FACEDOWN) return 1;
  return 0;
}

/* next alive seat after p; the next seat if nobody else is alive */
static int next_alive(const np_state* s, int p) {
  for (int k = 1; k < s->n; ++k) {
    int q = (p + k) % s->n;
    if (alive(s, q)) return q;
  }
  return (p + 1) % s->n;
}

static void next_turn(np_state* s) {
  /* NextPlayerTurn (coup.cc:1079-1086) */
  s->T = next_alive(s, s->T);
  s->M = s->T;
  s->O = next_alive(s, s->T);
  s->turn++;
  s->begin = 1;
}

static void next_move(np_state* s) {
  /* NextPlayerMove (coup.cc:1088-1092): M and O change roles */
  int m = s->M;
  s->M = s->O;
  s->O = m;
  s->begin = 0;
}

static void lose_reward(np_state* s, int p) {
  for (int q = 0; q < s->n; ++q) s->rewards[q] += (q == p) ? -(s->n - 1) : 1;
}

void np_init(np_state* s, int n) {
  /* CoupState::CoupState (coup.cc:393-428) */
  memset(s, 0, sizeof(*s));
  s->n = n;
  for (int t = 0; t < 5; ++t) s->deck[t] = 3;
  for (int p = 0; p < n; ++p) {
    s->pl[p].coins = (n == 2 && p == 0) ? 1 : 2;
    s->pl[p].last_action = OC_NONE;
  }
  s->init_left = 2 * n;
  s->T = 0;
  s->M = 0;
  s->O = 1;
  s->begin = 1;
}

int np_is_terminal(const np_state* s) {
  /* coup.cc:989-1010 */
  if (s->move > max_len(s)) return 1;
  int a = 0;
  for (int p = 0; p < s->n; ++p) a += alive(s, p);
  return a <= 1;
}

static int is_chance(const np_state* s) { return s->init_left > 0 || s->qlen > 0; }

int np_current_player(const np_state* s) {
  if (np_is_terminal(s)) return -4;
  if (is_chance(s)) return -1;
  return s->M;
}

static uint32_t lose_mask(const np_state* s) {
  const np_player* p = &s->pl[s->M];
  uint32_t m = 0;
  if (p->cards[0].state == OC_FACEDOWN) m |= 1u << OC_LOSE1;
  if (p->cards[1].state == OC_FACEDOWN) m |= 1u << OC_LOSE2;
  return m;
}

/* 0 where the reference would raise "Invalid action progression" */
uint32_t np_legal_mask(const np_state* s) {
  /* LegalActions (coup.cc:824-938), op = O */
  if (np_is_terminal(s)) return 0;
  if (is_chance(s)) {
    uint32_t m = 1u << 31;
    for (int t = 0; t < 5; ++t)
      if (s->deck[t] > 0) m |= 1u << t;
    return m;
  }
  const np_player* cp = &s->pl[s->M];
  const np_player* op = &s->pl[s->O];
  if (s->begin) {
    if (cp->coins >= 10) return 1u << OC_COUP;
    uint32_t m = (1u << OC_INCOME) | (1u << OC_FOREIGN_AID) | (1u << OC_TAX) | (1u << OC_EXCHANGE);
    if (cp->coins >= 7) m |= 1u << OC_COUP;
    if (cp->coins >= 3) m |= 1u << OC_ASSASSINATE;
    if (s->pl[next_alive(s, s->T)].coins > 0) m |= 1u << OC_STEAL;
    return m;
  }
  if (cp->lost_challenge) return lose_mask(s);
  if (s->M != s->T) {
    switch (op->last_action) {
      case OC_FOREIGN_AID: return (1u << OC_PASS) | (1u << OC_BLOCK);
      case OC_TAX:
      case OC_EXCHANGE: return (1u << OC_PASS) | (1u << OC_CHALLENGE);
      case OC_STEAL: return (1u << OC_PASS) | (1u << OC_BLOCK) | (1u << OC_CHALLENGE);
      case OC_ASSASSINATE: return lose_mask(s) | (1u << OC_BLOCK) | (1u << OC_CHALLENGE);
      case OC_COUP: return lose_mask(s);
      default: return 0;
    }
  }
  if (cp->last_action == OC_EXCHANGE) {
    if (cp->ncards < 4) return 0;
    int up = -1;
    for (int i = 0; i < cp->ncards; ++i)
      if (cp->cards[i].state == OC_FACEUP) {
        up = i;
        break;
      }
    static const int pi[6] = {0, 0, 0, 1, 1, 2}, pj[6] = {1, 2, 3, 2, 3, 3};
    uint32_t m = 0;
    for (int k = 0; k < 6; ++k)
      if (pi[k] != up && pj[k] != up) m |= 1u << (OC_XR12 + k);
    return m;
  }
  if (op->last_action == OC_BLOCK) return (1u << OC_PASS) | (1u << OC_CHALLENGE);
  return 0;
}

static void replace_card(np_state* s, int v) {
  /* ChallengeFailReplaceCard (coup.cc:468-486) on O */
  np_player* op = &s->pl[s->O];
  for (int i = 0; i < op->ncards; ++i) {
    if (op->cards[i].value == v && op->cards[i].state == OC_FACEDOWN) {
      s->deck[v] += 1;
      erase_card(op, i);
      s->queue[s->qlen++] = s->O;
      return;
    }
  }
  s->error = 2;
}

/* second half of a claim (coup.cc:542-603 via the Pass recursion) with the
 * claimant to move (M) and O = the last player who answered */
static void complete_claim(np_state* s, int a) {
  np_player* cp = &s->pl[s->M];
  np_player* op = &s->pl[s->O];
  switch (a) {
    case OC_FOREIGN_AID:
      cp->coins += 2;
      next_turn(s);
      return;
    case OC_TAX:
      cp->coins += 3;
      next_turn(s);
      return;
    case OC_EXCHANGE:
      s->queue[s->qlen++] = s->M;
      s->queue[s->qlen++] = s->M;
      return;
    case OC_STEAL: {
      int k = op->coins > 1 ? 2 : 1;
      cp->coins += k;
      op->coins -= k;
      next_turn(s);
      return;
    }
    default:
      s->error = 2;
  }
}

/* the turn ends after a double flip unless the game is over (at N = 2 it
 * always is: coup.cc:660-669, 733-742 do not change the turn) */
static void flip_two(np_state* s, int p) {
  np_player* pl = &s->pl[p];
  for (int i = 0; i < 2; ++i) {
    if (pl->cards[i].state == OC_FACEDOWN) {
      pl->cards[i].state = OC_FACEUP;
      lose_reward(s, p);
    }
  }
  if (!np_is_terminal(s)) next_turn(s);
}

static void do_challenge(np_state* s) {
  /* coup.cc:635-771 with op = O */
  np_player* cp = &s->pl[s->M];
  np_player* op = &s->pl[s->O];
  int cl = cp->last_action;
  if (op->last_action == OC_BLOCK) {
    if (cl == OC_FOREIGN_AID) {
      cp->last_action = OC_CHALLENGE;
      if (has_face_down(op, OC_DUKE)) {
        cp->lost_challenge = 1;
        replace_card(s, OC_DUKE);
      } else {
        op->lost_challenge = 1;
        cp->coins += 2;
        next_move(s);
      }
    } else if (cl == OC_ASSASSINATE) {
      cp->last_action = OC_CHALLENGE;
      if (has_face_down(op, OC_CONTESSA)) {
        cp->lost_challenge = 1;
        replace_card(s, OC_CONTESSA);
      } else {
        flip_two(s, s->O);
      }
    } else if (cl == OC_STEAL) {
      cp->last_action = OC_CHALLENGE;
      if (has_face_down(op, OC_CAPTAIN)) {
        cp->lost_challenge = 1;
        replace_card(s, OC_CAPTAIN);
      } else if (has_face_down(op, OC_AMBASSADOR)) {
        cp->lost_challenge = 1;
        replace_card(s, OC_AMBASSADOR);
      } else {
        op->lost_challenge = 1;
        int k = op->coins > 1 ? 2 : 1;
        cp->coins += k;
        op->coins -= k;
        next_move(s);
      }
    } else {
      s->error = 2;
    }
    return;
  }
  switch (op->last_action) {
    case OC_TAX:
      cp->last_action = OC_CHALLENGE;
      if (has_face_down(op, OC_DUKE)) {
        cp->lost_challenge = 1;
        replace_card(s, OC_DUKE);
        op->coins += 3;
      } else {
        op->lost_challenge = 1;
        next_move(s);
      }
      return;
    case OC_EXCHANGE:
      cp->last_action = OC_CHALLENGE;
      if (has_face_down(op, OC_AMBASSADOR)) {
        cp->lost_challenge = 1;
        replace_card(s, OC_AMBASSADOR);
        next_move(s);
        complete_claim(s, OC_EXCHANGE);
      } else {
        op->lost_challenge = 1;
        next_move(s);
      }
      return;
    case OC_ASSASSINATE:
      cp->last_action = OC_CHALLENGE;
      if (has_face_down(op, OC_ASSASSIN)) {
        flip_two(s, s->M);
      } else {
        op->lost_challenge = 1;
        op->coins += 3;
        next_move(s);
      }
      return;
    case OC_STEAL:
      cp->last_action = OC_CHALLENGE;
      if (has_face_down(op, OC_CAPTAIN)) {
        cp->lost_challenge = 1;
        replace_card(s, OC_CAPTAIN);
        int k = cp->coins > 1 ? 2 : 1;
        op->coins += k;
        cp->coins -= k;
      } else {
        op->lost_challenge = 1;
        next_move(s);
      }
      return;
    default:
      s->error = 2;
  }
}

/* next alive seat after M, before wrapping round to the turn player T */
static int next_responder(const np_state* s) {
  for (int k = 1; k < s->n; ++k) {
    int q = (s->M + k) % s->n;
    if (q == s->T) return -1;
    if (alive(s, q)) return q;
  }
  return -1;
}

static void do_decision(np_state* s, int a) {
  np_player* cp = &s->pl[s->M];
  for (int p = 0; p < s->n; ++p) s->rewards[p] = 0; /* coup.cc:527 */
  switch (a) {
    case OC_INCOME:
      cp->last_action = a;
      cp->coins += 1;
      next_turn(s);
      return;
    case OC_FOREIGN_AID:
    case OC_TAX:
    case OC_EXCHANGE:
    case OC_STEAL:
    case OC_COUP:
    case OC_ASSASSINATE:
      /* announce: the first responder (the target for targeted actions) */
      cp->last_action = a;
      if (a == OC_COUP) cp->coins -= 7;
      if (a == OC_ASSASSINATE) cp->coins -= 3;
      s->O = s->T;
      s->M = next_alive(s, s->T);
      s->begin = 0;
      return;
    case OC_LOSE1:
    case OC_LOSE2: {
      int idx = a - OC_LOSE1;
      cp->last_action = a;
      cp->cards[idx].state = OC_FACEUP;
      cp->lost_challenge = 0;
      sort_hand(cp);
      lose_reward(s, s->M);
      next_turn(s);
      return;
    }
    case OC_PASS: {
      cp->last_action = a;
      int pending = s->pl[s->O].last_action;
      if (pending == OC_BLOCK) {
        next_turn(s);
        return;
      }
      int r = (pending == OC_STEAL) ? -1 : next_responder(s);
      if (r >= 0) {
        s->M = r; /* the next player may answer the claim */
        return;
      }
      next_move(s);
      complete_claim(s, pending);
      return;
    }
    case OC_BLOCK:
      cp->last_action = a;
      next_move(s);
      return;
    case OC_CHALLENGE:
      do_challenge(s);
      return;
    default:
      break;
  }
  if (a >= OC_XR12 && a <= OC_XR34) {
    static const int pi[6] = {0, 0, 0, 1, 1, 2}, pj[6] = {1, 2, 3, 2, 3, 3};
    int k = a - OC_XR12;
    cp->last_action = a;
    erase_card(cp, pj[k]);
    s->deck[pj[k]] += 1; /* coup.cc:794: the slot index (reference quirk) */
    erase_card(cp, pi[k]);
    s->deck[pi[k]] += 1;
    if (s->pl[s->O].lost_challenge)
      next_move(s);
    else
      next_turn(s);
    return;
  }
  s->error = 1;
}

int np_apply_action(np_state* s, int a) {
  if (np_is_terminal(s)) return s->error = 3;
  uint32_t m = np_legal_mask(s);
  if (a < 0 || a > 17 || !((m >> a) & 1u)) return s->error = 1;
  if (m & (1u << 31)) {
    int to;
    if (s->init_left > 0) {
      to = (2 * s->n - s->init_left) % s->n;
      s->init_left--;
    } else {
      to = s->queue[0];
      for (int i = 1; i < s->qlen; ++i) s->queue[i - 1] = s->queue[i];
      s->qlen--;
    }
    s->deck[a] -= 1;
    np_player* p = &s->pl[to];
    p->cards[p->ncards].value = a;
    p->cards[p->ncards].state = OC_FACEDOWN;
    p->ncards++;
    sort_hand(p);
  } else {
    do_decision(s, a);
    for (int i = 1; i < s->qlen; ++i)
      if (s->queue[i] != s->queue[0]) s->error = 4; /* the packed queue is (player, length) */
  }
  s->move++;
  return s->error;
}

void np_returns(const np_state* s, int* out) {
  int up[NP_MAX_PLAYERS] = {0}, total = 0;
  for (int p = 0; p < s->n; ++p) {
    for (int i = 0; i < s->pl[p].ncards; ++i) up[p] += s->pl[p].cards[i].state == OC_FACEUP;
    total += up[p];
  }
  for (int p = 0; p < s->n; ++p) out[p] = (total - up[p]) - (s->n - 1) * up[p];
}

int np_obs_size(int n) { return 49 * n; }

void np_observation_tensor(const np_state* s, int player, float* out) {
  /* CoupObserver::WriteTensor (coup.cc:248-287) with num_players_ = N */
  const int n = s->n;
  for (int i = 0; i < 49 * n; ++i) out[i] = 0.0f;
  int off = 0;
  out[player] = 1.0f;
  off += n;
  for (int p = 0; p < n; ++p) {
    for (int i = 0; i < s->pl[p].ncards; ++i) {
      np_card c = s->pl[p].cards[i];
      if ((p == player && c.state == OC_FACEDOWN) || c.state == OC_FACEUP) out[off + i * 5 + c.value] = 1.0f;
    }
    off += 20;
  }
  if (!np_is_terminal(s)) out[off + s->M] = 1.0f;
  off += n;
  for (int p = 0; p < n; ++p)
    for (int i = 0; i < s->pl[p].ncards; ++i) out[off + p * 8 + i * 2 + s->pl[p].cards[i].state] = 1.0f;
  off += 8 * n;
  for (int p = 0; p < n; ++p) out[off + p] = (float)s->pl[p].coins;
  off += n;
  for (int p = 0; p < n; ++p)
    if (s->pl[p].last_action != OC_NONE) out[off + p * 18 + s->pl[p].last_action] = 1.0f;
}

void np_pack(const np_state* s, uint32_t episode, uint32_t* w) {
  /* 32-byte record: a step has at most one card
   * loser, so Rewards() is (loser, count); deals pending after the initial
   * ones all go to one player, so the queue is (player, length) */
  memset(w, 0, 8 * sizeof(uint32_t));
  uint32_t hands[6];
  for (int p = 0; p < 6; ++p) {
    hands[p] = 0xFFFFu;
    if (p >= s->n) continue;
    for (int i = 0; i < s->pl[p].ncards; ++i) {
      hands[p] &= ~(0xFu << (4 * i));
      hands[p] |= (uint32_t)(s->pl[p].cards[i].value * 2 + s->pl[p].cards[i].state) << (4 * i);
    }
  }
  w[0] = hands[0] | (hands[1] << 16);
  w[1] = hands[2] | (hands[3] << 16);
  w[2] = hands[4] | (hands[5] << 16);
  uint32_t coins = 0, last = 0, lost = 0, rloser = 0, rcount = 0, deck = 0;
  for (int p = 0; p < 6; ++p) {
    if (p >= s->n) {
      last |= 31u << (5 * p);
      continue;
    }
    coins |= (uint32_t)s->pl[p].coins << (4 * p);
    last |= (uint32_t)(s->pl[p].last_action == OC_NONE ? 31 : s->pl[p].last_action) << (5 * p);
    lost |= (uint32_t)s->pl[p].lost_challenge << p;
    if (s->rewards[p] < 0) {
      rloser = (uint32_t)p;
      rcount = (uint32_t)(-s->rewards[p] / (s->n - 1));
    }
  }
  for (int t = 0; t < 5; ++t) deck |= (uint32_t)s->deck[t] << (4 * t);
  const uint32_t qp = s->qlen ? (uint32_t)s->queue[0] : 0u;
  w[3] = coins | (lost << 24) | ((uint32_t)s->begin << 30) | ((uint32_t)(s->error ? 1 : 0) << 31);
  w[4] = last | (rcount << 30);
  w[5] = deck | ((uint32_t)s->init_left << 20) | ((uint32_t)s->qlen << 24) | (qp << 26) | ((uint32_t)s->T << 29);
  w[6] = (uint32_t)s->move | ((uint32_t)s->turn << 9) | ((uint32_t)s->M << 18) | ((uint32_t)s->O << 21) |
         (rloser << 24) | (((episode >> 25) & 31u) << 27);
  w[7] = episode & 0x1FFFFFFu; /* 30-bit episode: bits 24..0 here, 29..25 in w[6] */
}

/* ------------------------------------------------------------- rollouts */

static void resolve(np_state* s, uint64_t seed, uint32_t env, uint32_t ep) {
  while (np_current_player(s) == -1) {
    uint32_t u = oc_draw(seed, env, ep & NP_EPISODE_MASK, (uint32_t)s->move);
    int total = 0;
    for (int t = 0; t < 5; ++t) total += s->deck[t];
    uint32_t r = (uint32_t)(((uint64_t)u * (uint32_t)total) >> 32), cum = 0;
    int pick = 4;
    for (int t = 0; t < 4; ++t) {
      cum += (uint32_t)s->deck[t];
      if (cum > r) {
        pick = t;
        break;
      }
    }
    np_apply_action(s, pick);
  }
}

int np_rollout(const np_rollout_args* a) {
  const int P = a->n_players;
  int64_t done = 0, ret_sum = 0;
  for (int64_t lane = 0; lane < a->n; ++lane) {
    uint32_t env = a->env_id_base + (uint32_t)lane, ep = 0;
    np_state s;
    np_init(&s, P);
    resolve(&s, a->seed, env, ep);
    int pending = 0;
    for (int64_t t = 0; t < a->steps; ++t) {
      int act = -1, rw[NP_MAX_PLAYERS] = {0};
      uint8_t st;
      if (pending) {
        ep++;
        np_init(&s, P);
        resolve(&s, a->seed, env, ep);
        pending = 0;
        st = 0;
      } else {
        uint32_t m = np_legal_mask(&s);
        uint32_t u = oc_draw(a->seed, env, ep & NP_EPISODE_MASK, (uint32_t)s.move);
        uint32_t idx = (uint32_t)(((uint64_t)u * (uint32_t)__builtin_popcount(m)) >> 32);
        for (uint32_t k = 0; k < idx; ++k) m &= m - 1;
        act = __builtin_ctz(m);
        np_apply_action(&s, act);
        resolve(&s, a->seed, env, ep);
        for (int p = 0; p < P; ++p) rw[p] = s.rewards[p];
        if (np_is_terminal(&s)) {
          int ret[NP_MAX_PLAYERS];
          np_returns(&s, ret);
          done++;
          ret_sum += ret[0];
          if (a->lane_episodes) a->lane_episodes[lane] += 1;
          if (a->lane_return_sum) a->lane_return_sum[lane] += ret[0];
          st = 2;
          if (a->auto_reset) {
            ep++;
            np_init(&s, P);
            resolve(&s, a->seed, env, ep);
          } else {
            pending = 1;
          }
        } else {
          st = 1;
        }
      }
      int64_t o = t * a->n + lane;
      if (a->actions) a->actions[o] = (int8_t)act;
      if (a->rewards)
        for (int p = 0; p < P; ++p) a->rewards[o * P + p] = (int8_t)rw[p];
      if (a->step_type) a->step_type[o] = st;
      if (a->legal) a->legal[o] = np_legal_mask(&s);
      if (a->cur_player) a->cur_player[o] = (int8_t)np_current_player(&s);
      if (a->obs)
        for (int p = 0; p < P; ++p) np_observation_tensor(&s, p, a->obs + (o * P + p) * 49 * P);
    }
    if (a->final_state) np_pack(&s, ep, a->final_state + 8 * lane);
  }
  if (a->episodes_done) *a->episodes_done = done;
  if (a->return_sum_p0) *a->return_sum_p0 = ret_sum;
  return 0;
}

/* np_rollout's per-lane loop recording only steps [from, steps) into rows of
 * `stride` lanes, with record / accumulator snapshots (coup_oracle.h). */
int np_rollout_window(const oc_window_args* a) {
  const int P = a->players;
  if (P < 2 || P > NP_MAX_PLAYERS || a->n > a->stride || a->from < 0 || a->from > a->steps || a->obs_hash ||
      a->info_hash)
    return 1;
  for (int64_t lane = 0; lane < a->n; ++lane) {
    uint32_t env = a->env_id_base + (uint32_t)lane, ep = 0;
    int32_t eps = 0, ret_sum = 0;
    np_state s;
    np_init(&s, P);
    resolve(&s, a->seed, env, ep);
    int pending = 0;
    for (int64_t t = 0; t < a->steps; ++t) {
      int act = -1, rw[NP_MAX_PLAYERS] = {0};
      uint8_t st;
      if (pending) {
        ep++;
        np_init(&s, P);
        resolve(&s, a->seed, env, ep);
        pending = 0;
        st = 0;
      } else {
        uint32_t m = np_legal_mask(&s);
        uint32_t u = oc_draw(a->seed, env, ep & NP_EPISODE_MASK, (uint32_t)s.move);
        uint32_t idx = (uint32_t)(((uint64_t)u * (uint32_t)__builtin_popcount(m)) >> 32);
        for (uint32_t k = 0; k < idx; ++k) m &= m - 1;
        act = __builtin_ctz(m);
        np_apply_action(&s, act);
        resolve(&s, a->seed, env, ep);
        for (int p = 0; p < P; ++p) rw[p] = s.rewards[p];
        if (np_is_terminal(&s)) {
          int ret[NP_MAX_PLAYERS];
          np_returns(&s, ret);
          if (t >= a->stats_from) {
            eps += 1;
            ret_sum += ret[0];
          }
          st = 2;
          if (a->auto_reset) {
            ep++;
            np_init(&s, P);
            resolve(&s, a->seed, env, ep);
          } else {
            pending = 1;
          }
        } else {
          st = 1;
        }
      }
      if (t >= a->from) {
        int64_t o = (t - a->from) * a->stride + lane;
        if (a->actions) a->actions[o] = (int8_t)act;
        if (a->rewards)
          for (int p = 0; p < P; ++p) a->rewards[o * P + p] = (int8_t)rw[p];
        if (a->step_type) a->step_type[o] = st;
        if (a->legal) a->legal[o] = np_legal_mask(&s);
        if (a->cur_player) a->cur_player[o] = (int8_t)np_current_player(&s);
      }
      for (int k = 0; k < a->nsnap; ++k) {
        if (a->snap_at[k] != t + 1) continue;
        if (a->snap_state[k]) np_pack(&s, ep, a->snap_state[k] + 8 * lane);
        if (a->snap_eps[k]) a->snap_eps[k][lane] = eps;
        if (a->snap_ret[k]) a->snap_ret[k][lane] = ret_sum;
      }
    }
  }
  return 0;
}
