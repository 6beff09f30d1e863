/*
 * coup_oracle.c -- CPU restatement of the reference Coup rules engine.
 *
 * TEST INFRASTRUCTURE ONLY (see coup_oracle.h).  Each function cites the
 * reference file:line it restates.  The structure deliberately follows the
 * reference's object model (hand arrays kept sorted, a FIFO deal queue,
 * recursion for Pass / lost Exchange challenge) rather than the packed
 * register layout the HIP kernel uses, so the two implementations are
 * independent.
 */
#include "coup_oracle.h"

#include <stdio.h>
#include <string.h>

/* ---------------------------------------------------------------- helpers */

static int card_less(oc_card a, oc_card b) {
  /* CoupCard::operator< (coup.h:91-94): by value, then state */
  return a.value < b.value || (a.value == b.value && a.state < b.state);
}

static void sort_hand(oc_player* p) {
  /* CoupPlayer::SortCards (coup.cc:389-391); insertion sort is fine for <=4 */
  for (int i = 1; i < p->ncards; ++i) {
    oc_card c = p->cards[i];
    int j = i - 1;
    while (j >= 0 && card_less(c, p->cards[j])) {
      p->cards[j + 1] = p->cards[j];
      --j;
    }
    p->cards[j + 1] = c;
  }
}

static void erase_card(oc_player* p, int idx) {
  for (int i = idx; i + 1 < p->ncards; ++i) p->cards[i] = p->cards[i + 1];
  p->ncards--;
}

static int has_face_down(const oc_player* p, int value) {
  /* CoupPlayer::HasFaceDownCard (coup.cc:379-387) */
  for (int i = 0; i < p->ncards; ++i)
    if (p->cards[i].value == value && p->cards[i].state == OC_FACEDOWN) return 1;
  return 0;
}

static void queue_push(oc_state* s, int p) { s->queue[s->qlen++] = p; }

static int queue_pop(oc_state* s) {
  int front = s->queue[0];
  for (int i = 1; i < s->qlen; ++i) s->queue[i - 1] = s->queue[i];
  s->qlen--;
  return front;
}

static void next_turn(oc_state* s) {
  /* CoupState::NextPlayerTurn (coup.cc:1079-1086) */
  s->turn_player = 1 - s->turn_player;
  s->move_player = s->turn_player;
  s->opp_player = 1 - s->move_player;
  s->turn_number++;
  s->turn_begin = 1;
}

static void next_move(oc_state* s) {
  /* CoupState::NextPlayerMove (coup.cc:1088-1092) */
  s->move_player = 1 - s->move_player;
  s->opp_player = 1 - s->move_player;
  s->turn_begin = 0;
}

/* ------------------------------------------------------------- state API */

void oc_init(oc_state* s) {
  /* CoupState::CoupState (coup.cc:393-428) */
  memset(s, 0, sizeof(*s));
  for (int t = 0; t < OC_NUM_TYPES; ++t) s->deck[t] = 3;
  for (int p = 0; p < OC_NUM_PLAYERS; ++p) {
    s->pl[p].ncards = 0;
    s->pl[p].coins = p == 0 ? 1 : 2;
    s->pl[p].last_action = OC_NONE;
    s->pl[p].lost_challenge = 0;
  }
  s->turn_player = 0;
  s->move_player = 0;
  s->opp_player = 1;
  s->turn_begin = 1;
  s->turn_number = 0;
  s->is_chance = 1;
  queue_push(s, 0);
  queue_push(s, 1);
  queue_push(s, 0);
  queue_push(s, 1);
}

int oc_is_terminal(const oc_state* s) {
  /* CoupState::IsTerminal (coup.cc:989-1010) */
  if (s->move_number > OC_MAX_GAME_LENGTH) return 1;
  int alive = 0;
  for (int p = 0; p < OC_NUM_PLAYERS; ++p) {
    const oc_player* pl = &s->pl[p];
    if (pl->ncards < 2) {
      alive++;
      continue;
    }
    for (int i = 0; i < pl->ncards; ++i) {
      if (pl->cards[i].state == OC_FACEDOWN) {
        alive++;
        break;
      }
    }
  }
  return alive <= 1;
}

int oc_current_player(const oc_state* s) {
  /* CoupState::CurrentPlayer (coup.cc:458-466) */
  if (oc_is_terminal(s)) return -4;
  if (s->is_chance) return -1;
  return s->move_player;
}

static int lose_card_actions(const oc_state* s, int* out, int n) {
  /* CoupState::LegalLoseCardActions (coup.cc:811-822): slots 0 and 1 only */
  const oc_player* p = &s->pl[s->move_player];
  if (p->cards[0].state == OC_FACEDOWN) out[n++] = OC_LOSE1;
  if (p->cards[1].state == OC_FACEDOWN) out[n++] = OC_LOSE2;
  return n;
}

/* returns count, or -1 where the reference raises SpielFatalError */
static int legal_actions_impl(const oc_state* s, int* out) {
  /* CoupState::LegalActions (coup.cc:824-938) */
  int n = 0;
  if (oc_is_terminal(s)) return 0;
  if (s->is_chance) {
    for (int t = 0; t < OC_NUM_TYPES; ++t)
      if (s->deck[t] > 0) out[n++] = t;
    return n;
  }
  const oc_player* cp = &s->pl[s->move_player];
  const oc_player* op = &s->pl[s->opp_player];
  if (s->turn_begin) {
    if (cp->coins >= 10) {
      out[n++] = OC_COUP;
      return n;
    }
    out[n++] = OC_INCOME;
    out[n++] = OC_FOREIGN_AID;
    if (cp->coins >= 7) out[n++] = OC_COUP;
    out[n++] = OC_TAX;
    if (cp->coins >= 3) out[n++] = OC_ASSASSINATE;
    out[n++] = OC_EXCHANGE;
    if (op->coins > 0) out[n++] = OC_STEAL;
    return n;
  }
  if (cp->lost_challenge) return lose_card_actions(s, out, 0);
  if (s->move_player != s->turn_player) {
    switch (op->last_action) {
      case OC_FOREIGN_AID:
        out[n++] = OC_PASS;
        out[n++] = OC_BLOCK;
        return n;
      case OC_TAX:
      case OC_EXCHANGE:
        out[n++] = OC_PASS;
        out[n++] = OC_CHALLENGE;
        return n;
      case OC_STEAL:
        out[n++] = OC_PASS;
        out[n++] = OC_BLOCK;
        out[n++] = OC_CHALLENGE;
        return n;
      case OC_ASSASSINATE:
        n = lose_card_actions(s, out, 0);
        out[n++] = OC_BLOCK;
        out[n++] = OC_CHALLENGE;
        return n;
      case OC_COUP:
        return lose_card_actions(s, out, 0);
      default:
        return -1;
    }
  }
  if (cp->last_action == OC_EXCHANGE) {
    if (cp->ncards < 4) return -1;
    int up = -1;
    for (int i = 0; i < cp->ncards; ++i)
      if (cp->cards[i].state == OC_FACEUP) {
        up = i;
        break;
      }
    /* pairs (i,j) of slots to return that do not include the face-up slot */
    static const int pair_i[6] = {0, 0, 0, 1, 1, 2};
    static const int pair_j[6] = {1, 2, 3, 2, 3, 3};
    for (int k = 0; k < 6; ++k)
      if (pair_i[k] != up && pair_j[k] != up) out[n++] = OC_XR12 + k;
    return n;
  }
  if (op->last_action == OC_BLOCK) {
    out[n++] = OC_PASS;
    out[n++] = OC_CHALLENGE;
    return n;
  }
  return -1;
}

int oc_legal_actions(const oc_state* s, int* out) {
  int n = legal_actions_impl(s, out);
  return n < 0 ? 0 : n;
}

uint32_t oc_legal_mask(const oc_state* s) {
  int acts[OC_NUM_ACTIONS];
  int n = oc_legal_actions(s, acts);
  uint32_t m = 0;
  for (int i = 0; i < n; ++i) m |= 1u << acts[i];
  return m;
}

static void challenge_fail_replace(oc_state* s, int value) {
  /* CoupState::ChallengeFailReplaceCard (coup.cc:468-486) */
  oc_player* op = &s->pl[s->opp_player];
  for (int i = 0; i < op->ncards; ++i) {
    if (op->cards[i].value == value && op->cards[i].state == OC_FACEDOWN) {
      s->deck[value] += 1;
      erase_card(op, i);
      queue_push(s, s->opp_player);
      s->is_chance = 1;
      return;
    }
  }
  s->error = OC_ERR_PROGRESSION;
}

static void reward_to_mover(oc_state* s, int delta) {
  s->rewards[s->move_player] += delta;
  s->rewards[s->opp_player] -= delta;
}

static void do_apply_d(oc_state* s, int a, int depth);

static void do_apply(oc_state* s, int a) { do_apply_d(s, a, 0); }

static void do_challenge(oc_state* s) {
  /* Challenge branch of DoApplyAction (coup.cc:635-771) */
  oc_player* cp = &s->pl[s->move_player];
  oc_player* op = &s->pl[s->opp_player];
  if (op->last_action == OC_BLOCK) {
    /* cp is the turn player challenging a block of cp's own action */
    if (cp->last_action == OC_FOREIGN_AID) {
      cp->last_action = OC_CHALLENGE;
      if (has_face_down(op, OC_DUKE)) {
        cp->lost_challenge = 1;
        challenge_fail_replace(s, OC_DUKE);
      } else {
        op->lost_challenge = 1;
        cp->coins += 2;
        next_move(s);
      }
    } else if (cp->last_action == OC_ASSASSINATE) {
      cp->last_action = OC_CHALLENGE;
      if (has_face_down(op, OC_CONTESSA)) {
        cp->lost_challenge = 1;
        challenge_fail_replace(s, OC_CONTESSA);
      } else {
        for (int i = 0; i < 2; ++i) {
          if (op->cards[i].state == OC_FACEDOWN) {
            op->cards[i].state = OC_FACEUP;
            reward_to_mover(s, +1);
          }
        }
      }
    } else if (cp->last_action == OC_STEAL) {
      cp->last_action = OC_CHALLENGE;
      if (has_face_down(op, OC_CAPTAIN)) {
        cp->lost_challenge = 1;
        challenge_fail_replace(s, OC_CAPTAIN);
      } else if (has_face_down(op, OC_AMBASSADOR)) {
        cp->lost_challenge = 1;
        challenge_fail_replace(s, OC_AMBASSADOR);
      } else {
        op->lost_challenge = 1;
        int k = op->coins > 1 ? 2 : 1;
        cp->coins += k;
        op->coins -= k;
        next_move(s);
      }
    } else {
      s->error = OC_ERR_PROGRESSION;
    }
    return;
  }
  switch (op->last_action) {
    case OC_TAX:
      cp->last_action = OC_CHALLENGE;
      if (has_face_down(op, OC_DUKE)) {
        cp->lost_challenge = 1;
        challenge_fail_replace(s, OC_DUKE);
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
        challenge_fail_replace(s, OC_AMBASSADOR);
        s->is_chance = 0; /* coup.cc:715: lets the recursive Exchange run */
        next_move(s);
        do_apply(s, OC_EXCHANGE);
      } else {
        op->lost_challenge = 1;
        next_move(s);
      }
      return;
    case OC_ASSASSINATE:
      cp->last_action = OC_CHALLENGE;
      if (has_face_down(op, OC_ASSASSIN)) {
        for (int i = 0; i < 2; ++i) {
          if (cp->cards[i].state == OC_FACEDOWN) {
            cp->cards[i].state = OC_FACEUP;
            reward_to_mover(s, -1);
          }
        }
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
        challenge_fail_replace(s, OC_CAPTAIN);
        int k = cp->coins > 1 ? 2 : 1;
        op->coins += k;
        cp->coins -= k;
      } else {
        op->lost_challenge = 1;
        next_move(s);
      }
      return;
    default:
      s->error = OC_ERR_PROGRESSION;
      return;
  }
}

static void do_apply_d(oc_state* s, int a, int depth) {
  /* CoupState::DoApplyAction (coup.cc:490-809).  `depth` counts the Pass
   * recursion (coup.cc:628): legal play recurses once; an unchecked Pass
   * answering a Pass recurses without end in the reference (a crash), which
   * this restatement reports as an error instead. */
  if (oc_current_player(s) == -1) {
    /* chance branch (coup.cc:491-520) */
    if (a < 0 || a >= OC_NUM_TYPES || s->deck[a] <= 0 || s->qlen <= 0) {
      s->error = OC_ERR_ILLEGAL;
      return;
    }
    int to = queue_pop(s);
    s->hist_deal_to[s->hist_len] = to;
    s->deck[a] -= 1;
    oc_player* p = &s->pl[to];
    p->cards[p->ncards].value = a;
    p->cards[p->ncards].state = OC_FACEDOWN;
    p->ncards++;
    sort_hand(p);
    if (s->qlen == 0) s->is_chance = 0;
    return;
  }

  oc_player* cp = &s->pl[s->move_player];
  oc_player* op = &s->pl[s->opp_player];
  s->rewards[0] = s->rewards[1] = 0; /* coup.cc:527 */

  switch (a) {
    case OC_INCOME:
      cp->last_action = a;
      cp->coins += 1;
      next_turn(s);
      return;
    case OC_FOREIGN_AID:
      if (s->turn_begin) {
        cp->last_action = a;
        next_move(s);
      } else {
        cp->coins += 2;
        next_turn(s);
      }
      return;
    case OC_COUP:
      if (cp->coins < 7) { s->error = OC_ERR_ILLEGAL; return; }
      cp->last_action = a;
      cp->coins -= 7;
      next_move(s);
      return;
    case OC_TAX:
      if (s->turn_begin) {
        cp->last_action = a;
        next_move(s);
      } else {
        cp->coins += 3;
        next_turn(s);
      }
      return;
    case OC_ASSASSINATE:
      if (cp->coins < 3) { s->error = OC_ERR_ILLEGAL; return; }
      cp->last_action = a;
      cp->coins -= 3;
      next_move(s);
      return;
    case OC_EXCHANGE:
      if (s->turn_begin) {
        cp->last_action = a;
        next_move(s);
      } else {
        queue_push(s, s->move_player);
        queue_push(s, s->move_player);
        s->is_chance = 1;
      }
      return;
    case OC_STEAL:
      if (op->coins < 1) { s->error = OC_ERR_ILLEGAL; return; }
      if (s->turn_begin) {
        cp->last_action = a;
        next_move(s);
      } else {
        int k = op->coins > 1 ? 2 : 1;
        cp->coins += k;
        op->coins -= k;
        next_turn(s);
      }
      return;
    case OC_LOSE1:
    case OC_LOSE2: {
      int idx = a - OC_LOSE1;
      if (idx >= cp->ncards || cp->cards[idx].state != OC_FACEDOWN) {
        s->error = OC_ERR_ILLEGAL;
        return;
      }
      cp->last_action = a;
      cp->cards[idx].state = OC_FACEUP;
      cp->lost_challenge = 0;
      sort_hand(cp);
      reward_to_mover(s, -1);
      next_turn(s);
      return;
    }
    case OC_PASS: {
      cp->last_action = a;
      int pending = op->last_action;
      if (pending == OC_BLOCK) {
        next_turn(s);
      } else if (depth >= 4) {
        s->error = OC_ERR_PROGRESSION; /* unbounded recursion in the reference */
      } else {
        next_move(s);
        do_apply_d(s, pending, depth + 1); /* coup.cc:628: completes the original action */
      }
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
    /* ExchangeReturnXY (coup.cc:773-804) */
    static const int pair_i[6] = {0, 0, 0, 1, 1, 2};
    static const int pair_j[6] = {1, 2, 3, 2, 3, 3};
    int k = a - OC_XR12;
    int lo = pair_i[k], hi = pair_j[k];
    if (cp->ncards != 4) { s->error = OC_ERR_ILLEGAL; return; }
    cp->last_action = a;
    erase_card(cp, hi);
    s->deck[hi] += 1; /* coup.cc:794 credits the hand SLOT index (reference quirk) */
    erase_card(cp, lo);
    s->deck[lo] += 1;
    if (op->lost_challenge)
      next_move(s);
    else
      next_turn(s);
    return;
  }
  s->error = OC_ERR_ILLEGAL;
}

int oc_apply_action(oc_state* s, int a) {
  /* State::ApplyAction (spiel.cc:322-331), with a legality check in front
   * (State::ApplyActionWithLegalityCheck semantics).  */
  if (oc_is_terminal(s)) return s->error = OC_ERR_TERMINAL;
  int acts[OC_NUM_ACTIONS];
  int n = legal_actions_impl(s, acts);
  if (n < 0) return s->error = OC_ERR_PROGRESSION;
  int ok = 0;
  for (int i = 0; i < n; ++i) ok |= acts[i] == a;
  if (!ok) return s->error = OC_ERR_ILLEGAL;
  int player = oc_current_player(s);
  s->hist_deal_to[s->hist_len] = -1;
  do_apply(s, a);
  s->hist_player[s->hist_len] = player;
  s->hist_action[s->hist_len] = a;
  s->hist_len++;
  s->move_number++;
  return s->error;
}

/* Field widths of the product's 16-byte record:
 * coins 0..15, at most 4 queued deals, at most 4 cards per hand counting
 * the deals queued for it, cur_rewards_[0] in -2..5, hands in SortCards
 * order.  Legal play stays far inside them; unchecked actions can leave
 * them (a hand stays unsorted after the double flip of coup.cc:660-669 /
 * 733-742 on 3 or 4 cards, which has no SortCards). */
static int representable(const oc_state* s) {
  if (s->qlen > 4) return 0;
  for (int p = 0; p < OC_NUM_PLAYERS; ++p) {
    int pending = 0;
    for (int i = 0; i < s->qlen; ++i) pending += s->queue[i] == p;
    if (s->pl[p].coins < 0 || s->pl[p].coins > 15) return 0;
    if (s->pl[p].ncards + pending > OC_MAX_CARDS) return 0;
    for (int i = 1; i < s->pl[p].ncards; ++i)
      if (card_less(s->pl[p].cards[i], s->pl[p].cards[i - 1])) return 0;
  }
  return s->rewards[0] >= -2 && s->rewards[0] <= 5;
}

int oc_apply_action_unchecked(oc_state* s, int a) {
  /* State::ApplyAction (spiel.cc:322-331) as pyspiel binds apply_action
   * (pyspiel.cc:266): no LegalActions() check; DoApplyAction's own checks
   * decide (coup.cc:492-495, 549, 568, 590, 608, 685-692, 770, 787, 796,
   * 806).  On any error the state is left as it was. */
  if (oc_is_terminal(s)) return OC_ERR_TERMINAL;
  if (a < 0 || a >= OC_NUM_ACTIONS) return OC_ERR_ILLEGAL; /* coup.cc:493 / 806 */
  if (s->error) return s->error;
  oc_state t = *s;
  int player = oc_current_player(&t);
  t.hist_deal_to[t.hist_len] = -1;
  do_apply(&t, a); /* ExchangeReturn needs 4 cards: coup.cc:793 erases past the end or :796 fails */
  if (t.error) return t.error;
  if (!representable(&t)) return OC_ERR_UNREPRESENTABLE;
  t.hist_player[t.hist_len] = player;
  t.hist_action[t.hist_len] = a;
  t.hist_len++;
  t.move_number++;
  *s = t;
  return OC_OK;
}

void oc_returns(const oc_state* s, int* out2) {
  /* CoupState::Returns (coup.cc:1016-1032) */
  int up[2] = {0, 0};
  for (int p = 0; p < 2; ++p)
    for (int i = 0; i < s->pl[p].ncards; ++i) up[p] += s->pl[p].cards[i].state == OC_FACEUP;
  out2[0] = up[1] - up[0];
  out2[1] = up[0] - up[1];
}

void oc_rewards(const oc_state* s, int* out2) {
  /* CoupState::Rewards (coup.cc:1012-1014) */
  out2[0] = s->rewards[0];
  out2[1] = s->rewards[1];
}

int oc_chance_outcomes(const oc_state* s, int* actions, double* probs) {
  /* CoupState::ChanceOutcomes (coup.cc:1062-1077) */
  double total = 0;
  for (int t = 0; t < OC_NUM_TYPES; ++t) total += s->deck[t];
  int n = 0;
  for (int t = 0; t < OC_NUM_TYPES; ++t) {
    if (s->deck[t] > 0) {
      actions[n] = t;
      probs[n] = s->deck[t] / total;
      n++;
    }
  }
  return n;
}

/* -------------------------------------------------------------- tensors */

/* CoupObserver::WriteTensor (coup.cc:248-287) through a ContiguousAllocator
 * (observer.h:173-176, observer.cc:28-35): zero-fill, then consecutive
 * blocks.  perfect_recall selects the info-state variant (history block
 * instead of last_action). */
static void write_tensor(const oc_state* s, int player, int perfect_recall, float* out) {
  int size = perfect_recall ? OC_INFO_SIZE : OC_OBS_SIZE;
  for (int i = 0; i < size; ++i) out[i] = 0.0f;
  int off = 0;
  /* player one-hot [2] */
  out[off + player] = 1.0f;
  off += 2;
  /* p1_cards, p2_cards [4][5]: own face-down cards + all face-up cards */
  for (int p = 0; p < 2; ++p) {
    for (int i = 0; i < s->pl[p].ncards; ++i) {
      oc_card c = s->pl[p].cards[i];
      int visible = (p == player && c.state == OC_FACEDOWN) || c.state == OC_FACEUP;
      if (visible) out[off + i * OC_NUM_TYPES + c.value] = 1.0f;
    }
    off += OC_MAX_CARDS * OC_NUM_TYPES;
  }
  /* cur_move_player [2], zeros when terminal */
  if (!oc_is_terminal(s)) out[off + s->move_player] = 1.0f;
  off += 2;
  /* cards_state [2][4][2] */
  for (int p = 0; p < 2; ++p)
    for (int i = 0; i < s->pl[p].ncards; ++i)
      out[off + p * 8 + i * 2 + s->pl[p].cards[i].state] = 1.0f;
  off += 16;
  /* coins [2] */
  out[off + 0] = (float)s->pl[0].coins;
  out[off + 1] = (float)s->pl[1].coins;
  off += 2;
  if (!perfect_recall) {
    /* last_action [2][18] */
    for (int p = 0; p < 2; ++p)
      if (s->pl[p].last_action != OC_NONE) out[off + p * OC_NUM_ACTIONS + s->pl[p].last_action] = 1.0f;
  } else {
    /* history [135][18] (coup.cc:230-245): player actions, and chance deals
     * only when dealt to the observing player */
    for (int i = 0; i < s->hist_len; ++i) {
      int hp = s->hist_player[i];
      if (hp >= 0 || (hp == -1 && s->hist_deal_to[i] == player))
        out[off + i * OC_NUM_ACTIONS + s->hist_action[i]] = 1.0f;
    }
  }
}

void oc_observation_tensor(const oc_state* s, int player, float* out98) {
  write_tensor(s, player, 0, out98);
}

void oc_info_state_tensor(const oc_state* s, int player, float* out2492) {
  write_tensor(s, player, 1, out2492);
}

/* -------------------------------------------------------------- strings */

static const char* kCardNames[5] = {"Assassin", "Ambassador", "Captain", "Contessa", "Duke"};
static const char* kActionNames[18] = {
    "Income", "ForeignAid", "Coup", "Tax", "Assassinate", "Exchange",
    "Steal", "LoseCard1", "LoseCard2", "Pass", "Block", "Challenge",
    "ExchangeReturn12", "ExchangeReturn13", "ExchangeReturn14",
    "ExchangeReturn23", "ExchangeReturn24", "ExchangeReturn34"};

typedef struct {
  char* buf;
  int cap;
  int len;
} sbuf;

static void sb_put(sbuf* b, const char* str) {
  for (const char* c = str; *c; ++c) {
    if (b->len + 1 < b->cap) b->buf[b->len] = *c;
    b->len++;
  }
  if (b->cap > 0) b->buf[b->len < b->cap ? b->len : b->cap - 1] = '\0';
}

static void sb_int(sbuf* b, int v) {
  char tmp[16];
  snprintf(tmp, sizeof(tmp), "%d", v);
  sb_put(b, tmp);
}

static void sb_card_row(sbuf* b, int slot, const char* val, const char* state) {
  /* "Card N: <value padded to 11>| <state>\n" (coup.cc:312-337, 956-964) */
  char pad[16];
  int n = 11 - (int)strlen(val);
  if (n < 0) n = 0;
  memset(pad, ' ', (size_t)n);
  pad[n] = '\0';
  sb_put(b, "Card ");
  sb_int(b, slot + 1);
  sb_put(b, ": ");
  sb_put(b, val);
  sb_put(b, pad);
  sb_put(b, "| ");
  sb_put(b, state);
  sb_put(b, "\n");
}

/* CoupObserver::StringFrom (coup.cc:290-373) for the two built-in observer
 * types: public + single-player private, without / with perfect recall. */
static int string_from(const oc_state* s, int player, int perfect_recall, char* buf, int cap) {
  sbuf b = {buf, cap, 0};
  if (cap > 0) buf[0] = '\0';
  sb_put(&b, "Observer: P");
  sb_int(&b, player + 1);
  sb_put(&b, "\nTurn: ");
  sb_int(&b, s->turn_number);
  sb_put(&b, "\nMove: P");
  sb_int(&b, s->move_player + 1);
  sb_put(&b, "\n");
  for (int p = 0; p < 2; ++p) {
    sb_put(&b, "P");
    sb_int(&b, p + 1);
    sb_put(&b, "\n        Card         State\n");
    for (int i = 0; i < s->pl[p].ncards; ++i) {
      oc_card c = s->pl[p].cards[i];
      int show = c.state == OC_FACEUP || (p == player && c.state == OC_FACEDOWN);
      sb_card_row(&b, i, show ? kCardNames[c.value] : "-", c.state ? "FaceUp" : "FaceDown");
    }
    sb_put(&b, "Coins: ");
    sb_int(&b, s->pl[p].coins);
    sb_put(&b, "\n");
    if (!perfect_recall) {
      sb_put(&b, "Last Action: ");
      sb_put(&b, s->pl[p].last_action == OC_NONE ? "None" : kActionNames[s->pl[p].last_action]);
      sb_put(&b, "\n\n");
    } else {
      sb_put(&b, "\n");
    }
  }
  if (perfect_recall) {
    sb_put(&b, "Action Sequence: ");
    for (int i = 0; i < s->hist_len; ++i) {
      int last = i == s->hist_len - 1;
      if (s->hist_player[i] == -1) {
        if (s->hist_deal_to[i] == player) {
          sb_put(&b, "PC-");
          sb_put(&b, kCardNames[s->hist_action[i]]);
          if (!last) sb_put(&b, ", ");
        }
      } else {
        sb_put(&b, "P");
        sb_int(&b, s->hist_player[i] + 1);
        sb_put(&b, "-");
        sb_put(&b, kActionNames[s->hist_action[i]]);
        if (!last) sb_put(&b, ", ");
      }
    }
    sb_put(&b, "\n");
  }
  return b.len;
}

int oc_observation_string(const oc_state* s, int player, char* buf, int cap) {
  return string_from(s, player, 0, buf, cap);
}

int oc_info_state_string(const oc_state* s, int player, char* buf, int cap) {
  return string_from(s, player, 1, buf, cap);
}

int oc_to_string(const oc_state* s, char* buf, int cap) {
  /* CoupState::ToString (coup.cc:945-987) */
  sbuf b = {buf, cap, 0};
  if (cap > 0) buf[0] = '\0';
  sb_put(&b, "Turn: ");
  sb_int(&b, s->turn_number);
  sb_put(&b, "\nMove: P");
  sb_int(&b, s->move_player + 1);
  sb_put(&b, "\n");
  for (int p = 0; p < 2; ++p) {
    sb_put(&b, "P");
    sb_int(&b, p + 1);
    sb_put(&b, "\n        Card         State\n");
    for (int i = 0; i < s->pl[p].ncards; ++i) {
      oc_card c = s->pl[p].cards[i];
      sb_card_row(&b, i, kCardNames[c.value], c.state ? "FaceUp" : "FaceDown");
    }
    sb_put(&b, "Coins: ");
    sb_int(&b, s->pl[p].coins);
    sb_put(&b, "\nLast Action: ");
    sb_put(&b, s->pl[p].last_action == OC_NONE ? "None" : kActionNames[s->pl[p].last_action]);
    sb_put(&b, "\n\n");
  }
  sb_put(&b, "Action Sequence: ");
  for (int i = 0; i < s->hist_len; ++i) {
    if (s->hist_player[i] == -1) {
      sb_put(&b, "PC-");
      sb_put(&b, kCardNames[s->hist_action[i]]);
    } else {
      sb_put(&b, "P");
      sb_int(&b, s->hist_player[i] + 1);
      sb_put(&b, "-");
      sb_put(&b, kActionNames[s->hist_action[i]]);
    }
    if (i < s->hist_len - 1) sb_put(&b, ", ");
  }
  sb_put(&b, "\n");
  return b.len;
}

/* ------------------------------------------------------------ packing */

void oc_pack(const oc_state* s, uint32_t episode, uint32_t err, uint32_t* w) {
  /* Canonical 16-byte record. */
  uint32_t hand[2];
  for (int p = 0; p < 2; ++p) {
    hand[p] = 0xFFFFu;
    for (int i = 0; i < s->pl[p].ncards; ++i) {
      uint32_t kind = (uint32_t)(s->pl[p].cards[i].value * 2 + s->pl[p].cards[i].state);
      hand[p] &= ~(0xFu << (4 * i));
      hand[p] |= kind << (4 * i);
    }
  }
  uint32_t deck = 0;
  for (int t = 0; t < 5; ++t) deck |= (uint32_t)s->deck[t] << (4 * t);
  uint32_t q = 0;
  for (int i = 0; i < s->qlen; ++i) q |= (uint32_t)s->queue[i] << i;
  uint32_t last0 = s->pl[0].last_action == OC_NONE ? 31u : (uint32_t)s->pl[0].last_action;
  uint32_t last1 = s->pl[1].last_action == OC_NONE ? 31u : (uint32_t)s->pl[1].last_action;
  w[0] = hand[0] | (hand[1] << 16);
  w[1] = deck | ((uint32_t)s->pl[0].coins << 20) | ((uint32_t)s->pl[1].coins << 24) |
         ((uint32_t)(s->rewards[0] + 2) << 28) | ((err & 1u) << 31);
  w[2] = last0 | (last1 << 5) | ((uint32_t)s->pl[0].lost_challenge << 10) |
         ((uint32_t)s->pl[1].lost_challenge << 11) | ((uint32_t)s->qlen << 12) | (q << 15) |
         ((uint32_t)s->turn_player << 19) | ((uint32_t)s->move_player << 20) |
         ((uint32_t)s->turn_begin << 21) | ((uint32_t)s->move_number << 22) | (((episode >> 25) & 7u) << 29);
  w[3] = (uint32_t)s->turn_number | ((episode & 0x1FFFFFFu) << 7); /* 28-bit episode: bits 24..0 here */
}

void oc_history_bytes(const oc_state* s, uint8_t* out) {
  memset(out, 0xFF, 96);
  for (int i = 0; i < s->hist_len && i < 96; ++i) {
    int chance = s->hist_player[i] == -1;
    int who = chance ? s->hist_deal_to[i] : s->hist_player[i];
    out[i] = (uint8_t)(s->hist_action[i] | (chance << 5) | (who << 6));
  }
}

/* ------------------------------------------------------ sampling contract */

void oc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  /* Philox4x32 with 10 rounds (Salmon et al., SC'11 "Parallel random numbers:
   * as easy as 1, 2, 3"); multipliers and Weyl constants of Random123. */
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
  uint32_t k0 = key[0], k1 = key[1];
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0;
    uint32_t n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0;
  out[1] = c1;
  out[2] = c2;
  out[3] = c3;
}

uint32_t oc_draw(uint64_t seed, uint32_t env_id, uint32_t episode, uint32_t draw_idx) {
  /* One 32-bit draw per history slot: key = (env id, seed lo),
   * counter = (slot / 4, episode, seed hi, 'Coup'), word = slot % 4. */
  uint32_t key[2] = {env_id, (uint32_t)seed};
  uint32_t ctr[4] = {draw_idx >> 2, episode, (uint32_t)(seed >> 32), 0x436F7570u}; /* episode as stored */
  uint32_t out[4];
  oc_philox4x32_10(ctr, key, out);
  return out[draw_idx & 3];
}

static int sample_chance(const oc_state* s, uint32_t u) {
  int total = 0;
  for (int t = 0; t < 5; ++t) total += s->deck[t];
  uint32_t r = (uint32_t)(((uint64_t)u * (uint32_t)total) >> 32);
  uint32_t cum = 0;
  for (int t = 0; t < 5; ++t) {
    cum += (uint32_t)s->deck[t];
    if (cum > r) return t;
  }
  return -1;
}

static int sample_uniform(const oc_state* s, uint32_t u) {
  int acts[OC_NUM_ACTIONS];
  int n = oc_legal_actions(s, acts);
  if (n <= 0) return -1;
  uint32_t idx = (uint32_t)(((uint64_t)u * (uint32_t)n) >> 32);
  return acts[idx]; /* acts ascending == idx-th set bit of the legal mask */
}

static void resolve_chance(oc_state* s, uint64_t seed, uint32_t env_id, uint32_t episode) {
  /* rl_environment._sample_external_events (rl_environment.py:369-382) */
  while (oc_current_player(s) == -1) {
    uint32_t u = oc_draw(seed, env_id, episode & OC_EPISODE_MASK, (uint32_t)s->move_number);
    oc_apply_action(s, sample_chance(s, u));
  }
}

int oc_rollout(const oc_rollout_args* a) {
  int64_t decisions = 0, done_eps = 0, ret_sum = 0;
  for (int64_t lane = 0; lane < a->n; ++lane) {
    uint32_t env_id = a->env_id_base + (uint32_t)lane;
    uint32_t episode = 0;
    oc_state s;
    oc_init(&s);
    resolve_chance(&s, a->seed, env_id, episode);
    int pending_reset = 0;
    for (int64_t t = 0; t < a->steps; ++t) {
      int8_t act = -1;
      int rw[2] = {0, 0};
      uint8_t st;
      if (pending_reset) {
        /* rl_environment.step after LAST -> reset (rl_environment.py:310-311) */
        episode++;
        oc_init(&s);
        resolve_chance(&s, a->seed, env_id, episode);
        pending_reset = 0;
        st = 0; /* FIRST */
      } else {
        uint32_t u = oc_draw(a->seed, env_id, episode & OC_EPISODE_MASK, (uint32_t)s.move_number);
        int action = sample_uniform(&s, u);
        act = (int8_t)action;
        oc_apply_action(&s, action);
        resolve_chance(&s, a->seed, env_id, episode);
        decisions++;
        oc_rewards(&s, rw);
        if (oc_is_terminal(&s)) {
          int ret[2];
          oc_returns(&s, ret);
          done_eps++;
          ret_sum += ret[0];
          if (a->lane_episodes) a->lane_episodes[lane] += 1;
          if (a->lane_return_sum) a->lane_return_sum[lane] += ret[0];
          st = 2; /* LAST */
          if (a->auto_reset) {
            /* SyncVectorEnv.step(reset_if_done=True) (vector_env.py:62-65) */
            episode++;
            oc_init(&s);
            resolve_chance(&s, a->seed, env_id, episode);
          } else {
            pending_reset = 1;
          }
        } else {
          st = 1; /* MID */
        }
      }
      int64_t o = t * a->n + lane;
      if (a->actions) a->actions[o] = act;
      if (a->rewards) {
        a->rewards[2 * o] = (int8_t)rw[0];
        a->rewards[2 * o + 1] = (int8_t)rw[1];
      }
      if (a->step_type) a->step_type[o] = st;
      if (a->legal) a->legal[o] = oc_legal_mask(&s);
      if (a->obs) {
        float* dst = a->obs + (a->obs_overwrite ? lane : o) * 2 * OC_OBS_SIZE;
        oc_observation_tensor(&s, 0, dst);
        oc_observation_tensor(&s, 1, dst + OC_OBS_SIZE);
      }
      if (a->info) {
        float* dst = a->info + o * 2 * OC_INFO_SIZE;
        oc_info_state_tensor(&s, 0, dst);
        oc_info_state_tensor(&s, 1, dst + OC_INFO_SIZE);
      }
    }
    if (a->final_state) oc_pack(&s, episode, s.error ? 1u : 0u, a->final_state + 4 * lane);
    if (a->final_hist) oc_history_bytes(&s, a->final_hist + 96 * lane);
  }
  if (a->decisions) *a->decisions = decisions;
  if (a->episodes_done) *a->episodes_done = done_eps;
  if (a->return_sum_p0) *a->return_sum_p0 = ret_sum;
  return 0;
}

/* The every-lane window driver (coup_oracle.h): oc_rollout's per-lane loop,
 * recording only steps [from, steps) and hashing the tensors. */
static void window_hash(const float* x, int len, const uint32_t* w, uint64_t* out2) {
  uint64_t h0 = 0, h1 = 0;
  for (int i = 0; i < len; ++i) {
    uint32_t b;
    memcpy(&b, x + i, 4);
    h0 += (uint64_t)b * w[i];
    h1 += (uint64_t)b * w[len + i];
  }
  out2[0] = h0;
  out2[1] = h1;
}

int oc_rollout_window(const oc_window_args* a) {
  if (a->players != 2 || a->n > a->stride || a->from < 0 || a->from > a->steps) return OC_ERR_ILLEGAL;
  float obs[2 * OC_OBS_SIZE];
  float info[2 * OC_INFO_SIZE]; /* 20 KB of stack */
  for (int64_t lane = 0; lane < a->n; ++lane) {
    uint32_t env_id = a->env_id_base + (uint32_t)lane;
    uint32_t episode = 0;
    int32_t eps = 0, ret_sum = 0;
    oc_state s;
    oc_init(&s);
    resolve_chance(&s, a->seed, env_id, episode);
    int pending_reset = 0;
    for (int64_t t = 0; t < a->steps; ++t) {
      int8_t act = -1;
      int rw[2] = {0, 0};
      uint8_t st;
      if (pending_reset) {
        episode++;
        oc_init(&s);
        resolve_chance(&s, a->seed, env_id, episode);
        pending_reset = 0;
        st = 0;
      } else {
        uint32_t u = oc_draw(a->seed, env_id, episode & OC_EPISODE_MASK, (uint32_t)s.move_number);
        int action = sample_uniform(&s, u);
        act = (int8_t)action;
        oc_apply_action(&s, action);
        resolve_chance(&s, a->seed, env_id, episode);
        oc_rewards(&s, rw);
        if (oc_is_terminal(&s)) {
          int ret[2];
          oc_returns(&s, ret);
          if (t >= a->stats_from) {
            eps += 1;
            ret_sum += ret[0];
          }
          st = 2;
          if (a->auto_reset) {
            episode++;
            oc_init(&s);
            resolve_chance(&s, a->seed, env_id, episode);
          } else {
            pending_reset = 1;
          }
        } else {
          st = 1;
        }
      }
      if (t >= a->from) {
        int64_t o = (t - a->from) * a->stride + lane;
        if (a->actions) a->actions[o] = act;
        if (a->rewards) {
          a->rewards[2 * o] = (int8_t)rw[0];
          a->rewards[2 * o + 1] = (int8_t)rw[1];
        }
        if (a->step_type) a->step_type[o] = st;
        if (a->legal) a->legal[o] = oc_legal_mask(&s);
        if (a->cur_player) a->cur_player[o] = (int8_t)oc_current_player(&s);
        if (a->obs_hash) {
          oc_observation_tensor(&s, 0, obs);
          oc_observation_tensor(&s, 1, obs + OC_OBS_SIZE);
          window_hash(obs, 2 * OC_OBS_SIZE, a->obs_w, a->obs_hash + 2 * o);
        }
        if (a->info_hash) {
          oc_info_state_tensor(&s, 0, info);
          oc_info_state_tensor(&s, 1, info + OC_INFO_SIZE);
          window_hash(info, 2 * OC_INFO_SIZE, a->info_w, a->info_hash + 2 * o);
        }
      }
      for (int k = 0; k < a->nsnap; ++k) {
        if (a->snap_at[k] != t + 1) continue;
        if (a->snap_state[k]) oc_pack(&s, episode, s.error ? 1u : 0u, a->snap_state[k] + 4 * lane);
        if (a->snap_eps[k]) a->snap_eps[k][lane] = eps;
        if (a->snap_ret[k]) a->snap_ret[k][lane] = ret_sum;
      }
    }
  }
  return 0;
}
