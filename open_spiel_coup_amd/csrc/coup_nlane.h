// coup_nlane.h -- the N-player Coup extension (N = 2..6) on a register lane.
//
// The reference game is 2-player only (coup.h:42, coup.cc:45-46); the
// extension's rules are written down in oracle/coup_nplayer.h and the GPU
// is checked against that specification (parity unpinned for N > 2).  At
// N = 2 the rules are the reference's, which the GPU tests check against
// the 2-player engine and the reference's golden data.
//
// A lane is a 32-byte record (8 x u32), stored as two
// uint4 planes so each plane loads and stores fully coalesced:
//   w0..w2  hands of seats (0,1) (2,3) (4,5): 16-bit nibble strings (coup_lane.h)
//   w3      coins 4 bits/seat [23:0] | lost_challenge [29:24] | begin [30] | err [31]
//   w4      last action 5 bits/seat [29:0] (31 = None) | reward count [31:30]
//   w5      deck [19:0] | initial deals left [23:20] | queue length [25:24] |
//           queue player [28:26] | turn player T [31:29]
//   w6      move [8:0] | turn [17:9] | mover M [20:18] | counterpart O [23:21] |
//           reward loser [26:24] | episode bits 29..25 [31:27]
//   w7      episode bits 24..0 [24:0] (30-bit counter; [29:25] park the
//           regrouped step's next decision, coup_nplayer.hip)
// Rewards() is (loser, count): one decision makes at most one player lose
// cards, -(N-1) per card to the loser and +1 to everybody else.  Deals
// queued after the initial ones always go to one player (replacement card
// and/or Exchange draws), so the queue is (player, length).
//
// Per-seat fields are bit fields indexed with a run-time shift (no arrays,
// so nothing spills to scratch); N is a template parameter, so seat loops
// unroll and "mod N" is a compare.
#pragma once

#include "coup_lane.h"

namespace coup {
namespace np {

// 30-bit episode counter (the Philox counter word of the lane's draws);
// past 2^30 episodes a lane would replay its first games, so the wrap sets
// the record's error flag (new_episode).  kNpEpisodeLo: its bits in w7.
constexpr uint32_t kNpEpisodeMask = 0x3FFFFFFFu;
constexpr uint32_t kNpEpisodeLo = 0x1FFFFFFu;

// episode of a packed record's second plane
__device__ __forceinline__ uint32_t plane_episode(const uint4& b) { return (b.w & kNpEpisodeLo) | ((b.z >> 27) << 25); }

constexpr uint32_t kMaxSeats = 6;

template <int N>
struct NLane {
  uint32_t hA, hB, hC;  // hands of seats (0,1), (2,3), (4,5)
  uint32_t coins;       // 4 bits per seat
  uint32_t last;        // 5 bits per seat
  uint32_t lost;        // 1 bit per seat
  uint32_t deck, init_left, qlen, qp;
  uint32_t T, M, O, begin, err;
  uint32_t move, turn, episode;
  uint32_t rloser, rcount;
};

template <int N>
__device__ __forceinline__ NLane<N> unpack(uint4 a, uint4 b) {
  NLane<N> L;
  L.hA = a.x;
  L.hB = a.y;
  L.hC = a.z;
  L.coins = a.w & 0xFFFFFFu;
  L.lost = (a.w >> 24) & 0x3Fu;
  L.begin = (a.w >> 30) & 1u;
  L.err = a.w >> 31;
  L.last = b.x & 0x3FFFFFFFu;
  L.rcount = b.x >> 30;
  L.deck = b.y & 0xFFFFFu;
  L.init_left = (b.y >> 20) & 0xFu;
  L.qlen = (b.y >> 24) & 3u;
  L.qp = (b.y >> 26) & 7u;
  L.T = b.y >> 29;
  L.move = b.z & 0x1FFu;
  L.turn = (b.z >> 9) & 0x1FFu;
  L.M = (b.z >> 18) & 7u;
  L.O = (b.z >> 21) & 7u;
  L.rloser = (b.z >> 24) & 7u;
  L.episode = plane_episode(b);
  return L;
}

template <int N>
__device__ __forceinline__ void pack(const NLane<N>& L, uint4& a, uint4& b) {
  a.x = L.hA;
  a.y = L.hB;
  a.z = L.hC;
  a.w = L.coins | (L.lost << 24) | (L.begin << 30) | (L.err << 31);
  b.x = L.last | (L.rcount << 30);
  b.y = L.deck | (L.init_left << 20) | (L.qlen << 24) | ((L.qlen ? L.qp : 0u) << 26) | (L.T << 29);
  b.z = L.move | (L.turn << 9) | (L.M << 18) | (L.O << 21) | (L.rloser << 24) | (((L.episode >> 25) & 31u) << 27);
  b.w = L.episode & kNpEpisodeLo;
}

// NewInitialState: deck 3 of each, no cards dealt yet (2N initial deals go
// round the table twice), 1 and 2 coins at N = 2 (coup.cc:407-420), 2 each
// otherwise; seat 0 to move.
template <int N>
__device__ __forceinline__ NLane<N> initial_lane(uint32_t episode) {
  NLane<N> L;
  L.hA = 0xFFFFFFFFu;
  L.hB = 0xFFFFFFFFu;
  L.hC = 0xFFFFFFFFu;
  L.coins = N == 2 ? 0x21u : (0x222222u & ((1u << (4 * N)) - 1u));
  L.last = 0x3FFFFFFFu;
  L.lost = 0;
  L.deck = kInitialDeck;
  L.init_left = 2u * N;
  L.qlen = 0;
  L.qp = 0;
  L.T = 0;
  L.M = 0;
  L.O = 1;
  L.begin = 1;
  L.err = 0;
  L.move = 0;
  L.turn = 0;
  L.episode = episode & kNpEpisodeMask;
  L.rloser = 0;
  L.rcount = 0;
  return L;
}

// ------------------------------------------------------ per-seat fields

// Seat p's hand.  Written as arithmetic on the three words (no select
// between struct fields): LLVM turns a select of two fields of the lane
// into an indexed load, which puts the whole lane in scratch memory.
template <int N>
__device__ __forceinline__ uint32_t hand(const NLane<N>& L, uint32_t p) {
  if (N <= 2) return (L.hA >> (16u * p)) & 0xFFFFu;
  const uint64_t lo = ((uint64_t)L.hB << 32) | L.hA;  // seats 0..3
  const uint32_t a = (uint32_t)(lo >> (16u * (p & 3u)));
  if (N <= 4) return a & 0xFFFFu;
  const uint32_t c = L.hC >> (16u * (p & 1u));  // seats 4, 5
  const uint32_t hi = 0u - (uint32_t)(p >= 4u);  // all ones for seats 4, 5
  return ((a & ~hi) | (c & hi)) & 0xFFFFu;
}

template <int N>
__device__ __forceinline__ void set_hand(NLane<N>& L, uint32_t p, uint32_t h) {
  const uint32_t sh = 16u * (p & 1u);
  const uint32_t field = 0xFFFFu << sh, v = h << sh;
  // all-ones masks of the word that holds seat p
  const uint32_t inA = 0u - (uint32_t)(p < 2u);
  const uint32_t inB = 0u - (uint32_t)(p - 2u < 2u);
  const uint32_t inC = 0u - (uint32_t)(p >= 4u);
  L.hA = (L.hA & ~(field & inA)) | (v & inA);
  if (N > 2) L.hB = (L.hB & ~(field & inB)) | (v & inB);
  if (N > 4) L.hC = (L.hC & ~(field & inC)) | (v & inC);
}

template <int N>
__device__ __forceinline__ uint32_t coins(const NLane<N>& L, uint32_t p) { return (L.coins >> (4u * p)) & 0xFu; }
// coins never leave 0..12, so a field add / subtract never carries out
template <int N>
__device__ __forceinline__ void add_coins(NLane<N>& L, uint32_t p, int32_t k) {
  L.coins += (uint32_t)k << (4u * p);
}
template <int N>
__device__ __forceinline__ uint32_t last(const NLane<N>& L, uint32_t p) { return (L.last >> (5u * p)) & 31u; }
template <int N>
__device__ __forceinline__ void set_last(NLane<N>& L, uint32_t p, uint32_t a) {
  L.last = (L.last & ~(31u << (5u * p))) | (a << (5u * p));
}
template <int N>
__device__ __forceinline__ uint32_t lost(const NLane<N>& L, uint32_t p) { return (L.lost >> p) & 1u; }
template <int N>
__device__ __forceinline__ void set_lost(NLane<N>& L, uint32_t p, uint32_t v) {
  L.lost = (L.lost & ~(1u << p)) | (v << p);
}

// -------------------------------------------------------- seat order

// bit p set iff seat p is alive (coup.cc:994-1006 per player)
template <int N>
__device__ __forceinline__ uint32_t alive_mask(const NLane<N>& L) {
  uint32_t m = 0;
#pragma unroll
  for (int p = 0; p < N; ++p) m |= (alive(hand(L, (uint32_t)p)) ? 1u : 0u) << p;
  return m;
}

// seats p+1, p+2, ..., p+N-1 (mod N) as bits 0..N-2
template <int N>
__device__ __forceinline__ uint32_t after(uint32_t m, uint32_t p) {
  return ((m >> (p + 1u)) | (m << (N - 1u - p))) & ((1u << (N - 1)) - 1u);
}

template <int N>
__device__ __forceinline__ uint32_t seat_plus(uint32_t p, uint32_t k) {
  const uint32_t q = p + k;
  return q >= (uint32_t)N ? q - N : q;
}

// the next alive seat after p; the next seat if nobody else is alive
template <int N>
__device__ __forceinline__ uint32_t next_alive(uint32_t am, uint32_t p) {
  const uint32_t r = after<N>(am, p);
  return seat_plus<N>(p, r ? 1u + (uint32_t)__builtin_ctz(r) : 1u);
}

template <int N>
__device__ __forceinline__ bool is_terminal(const NLane<N>& L) {
  // IsTerminal (coup.cc:989-1010) with MaxGameLength = 45 N
  return L.move > 45u * N || __popc(alive_mask(L)) <= 1;
}

template <int N>
__device__ __forceinline__ bool is_chance(const NLane<N>& L) { return (L.init_left | L.qlen) != 0u; }

template <int N>
__device__ __forceinline__ int current_player(const NLane<N>& L) {
  return is_terminal(L) ? -4 : (is_chance(L) ? -1 : (int)L.M);
}

template <int N>
__device__ __forceinline__ int32_t reward(const NLane<N>& L, uint32_t p) {
  return p == L.rloser ? -(int32_t)((N - 1) * L.rcount) : (int32_t)L.rcount;
}

// Returns: sum over the others' face-up cards - (N-1) x own face-up cards
template <int N>
__device__ __forceinline__ int32_t returns(const NLane<N>& L, uint32_t p) {
  int32_t total = 0;
#pragma unroll
  for (int q = 0; q < N; ++q) total += (int32_t)face_up_count(hand(L, (uint32_t)q));
  return total - N * (int32_t)face_up_count(hand(L, p));
}

// ------------------------------------------------------------ legal mask

template <int N>
__device__ __forceinline__ uint32_t decision_mask(const NLane<N>& L) {
  const uint32_t M = L.M, O = L.O;
  const uint32_t cp_coins = coins(L, M);
  const uint32_t cp_last = last(L, M), op_last = last(L, O);
  const uint32_t cp_hand = hand(L, M);
  if (L.begin) {
    if (cp_coins >= 10) return 1u << kCoup;
    uint32_t m = (1u << kIncome) | (1u << kForeignAid) | (1u << kTax) | (1u << kExchange);
    m |= (cp_coins >= 7) ? (1u << kCoup) : 0u;
    m |= (cp_coins >= 3) ? (1u << kAssassinate) : 0u;
    m |= coins(L, next_alive<N>(alive_mask(L), L.T)) > 0 ? (1u << kSteal) : 0u;
    return m;
  }
  if (lost(L, M)) return lose_card_mask(cp_hand);
  if (M != L.T) {
    switch (op_last) {
      case kForeignAid: return (1u << kPass) | (1u << kBlock);
      case kTax:
      case kExchange: return (1u << kPass) | (1u << kChallenge);
      case kSteal: return (1u << kPass) | (1u << kBlock) | (1u << kChallenge);
      case kAssassinate: return lose_card_mask(cp_hand) | (1u << kBlock) | (1u << kChallenge);
      case kCoup: return lose_card_mask(cp_hand);
      default: return 0u;
    }
  }
  if (cp_last == kExchange) {
    if (nib(cp_hand, 3) == 0xFu) return 0u;
    const uint32_t up = cp_hand & 0x1111u;
    if (up == 0) return 0x3Fu << kExchangeReturn12;
    const uint32_t s = (uint32_t)__builtin_ctz(up) >> 2;
    const uint32_t excl = (0x07u | (0x19u << 6) | (0x2Au << 12) | (0x34u << 18)) >> (6u * s);
    return ((~excl) & 0x3Fu) << kExchangeReturn12;
  }
  if (op_last == kBlock) return (1u << kPass) | (1u << kChallenge);
  return 0u;
}

template <int N>
__device__ __forceinline__ uint32_t legal_mask(const NLane<N>& L) {
  if (is_terminal(L)) return 0u;
  if (is_chance(L)) return chance_mask(L.deck) | kChanceFlag;
  return decision_mask(L);
}

// ----------------------------------------------------------- transitions

template <int N>
__device__ __forceinline__ void next_turn(NLane<N>& L) {
  const uint32_t am = alive_mask(L);
  L.T = next_alive<N>(am, L.T);
  L.M = L.T;
  L.O = next_alive<N>(am, L.T);
  L.turn += 1u;
  L.begin = 1u;
}

template <int N>
__device__ __forceinline__ void next_move(NLane<N>& L) {
  const uint32_t m = L.M;
  L.M = L.O;
  L.O = m;
  L.begin = 0u;
}

template <int N>
__device__ __forceinline__ void lose_reward(NLane<N>& L, uint32_t p) {
  L.rloser = p;
  L.rcount += 1u;
}

template <int N>
__device__ __forceinline__ void queue_push(NLane<N>& L, uint32_t p) {
  L.qp = p;
  L.qlen += 1u;
}

// ChallengeFailReplaceCard (coup.cc:468-486) on O
template <int N>
__device__ __forceinline__ void replace_card(NLane<N>& L, uint32_t type) {
  const uint32_t h = hand(L, L.O);
  const uint32_t hit = nib_eq(h, 2u * type);
  if (hit == 0) {
    L.err = 1u;
    return;
  }
  L.deck += 1u << (4u * type);
  set_hand(L, L.O, hand_remove(h, (uint32_t)__builtin_ctz(hit) >> 2));
  queue_push(L, L.O);
}

template <int N>
__device__ __forceinline__ void steal_coins(NLane<N>& L, uint32_t to, uint32_t from) {
  const int32_t k = coins(L, from) > 1u ? 2 : 1;
  add_coins(L, to, k);
  add_coins(L, from, -k);
}

// second half of a claim, claimant to move (coup.cc:542-603)
template <int N>
__device__ __forceinline__ void complete_claim(NLane<N>& L, uint32_t a) {
  switch (a) {
    case kForeignAid:
      add_coins(L, L.M, 2);
      next_turn(L);
      break;
    case kTax:
      add_coins(L, L.M, 3);
      next_turn(L);
      break;
    case kExchange:
      queue_push(L, L.M);
      queue_push(L, L.M);
      break;
    case kSteal:
      steal_coins(L, L.M, L.O);
      next_turn(L);
      break;
    default:
      L.err = 1u;
  }
}

// flip slots 0 and 1 of seat p; the turn moves on unless the game is over
// (at N = 2 it always is: coup.cc:660-669, 733-742)
template <int N>
__device__ __forceinline__ void flip_two(NLane<N>& L, uint32_t p) {
  uint32_t h = hand(L, p);
#pragma unroll
  for (uint32_t i = 0; i < 2; ++i) {
    if ((nib(h, i) & 1u) == 0) {
      h |= 1u << (4u * i);
      lose_reward(L, p);
    }
  }
  set_hand(L, p, h);
  if (!is_terminal(L)) next_turn(L);
}

// Challenge (coup.cc:635-771) with op = O
template <int N>
__device__ __forceinline__ void apply_challenge(NLane<N>& L) {
  const uint32_t M = L.M, O = L.O;
  const uint32_t op_last = last(L, O), cp_last = last(L, M);
  const uint32_t op_hand = hand(L, O);
  set_last(L, M, kChallenge);
  if (op_last == kBlock) {
    if (cp_last == kForeignAid) {
      if (has_face_down(op_hand, kDuke)) {
        set_lost(L, M, 1u);
        replace_card(L, kDuke);
      } else {
        set_lost(L, O, 1u);
        add_coins(L, M, 2);
        next_move(L);
      }
    } else if (cp_last == kAssassinate) {
      if (has_face_down(op_hand, kContessa)) {
        set_lost(L, M, 1u);
        replace_card(L, kContessa);
      } else {
        flip_two(L, O);
      }
    } else if (cp_last == kSteal) {
      if (has_face_down(op_hand, kCaptain)) {
        set_lost(L, M, 1u);
        replace_card(L, kCaptain);
      } else if (has_face_down(op_hand, kAmbassador)) {
        set_lost(L, M, 1u);
        replace_card(L, kAmbassador);
      } else {
        set_lost(L, O, 1u);
        steal_coins(L, M, O);
        next_move(L);
      }
    } else {
      set_last(L, M, cp_last);
      L.err = 1u;
    }
    return;
  }
  switch (op_last) {
    case kTax:
      if (has_face_down(op_hand, kDuke)) {
        set_lost(L, M, 1u);
        replace_card(L, kDuke);
        add_coins(L, O, 3);
      } else {
        set_lost(L, O, 1u);
        next_move(L);
      }
      break;
    case kExchange:
      if (has_face_down(op_hand, kAmbassador)) {
        set_lost(L, M, 1u);
        replace_card(L, kAmbassador);
        next_move(L);
        complete_claim(L, kExchange);
      } else {
        set_lost(L, O, 1u);
        next_move(L);
      }
      break;
    case kAssassinate:
      if (has_face_down(op_hand, kAssassin)) {
        flip_two(L, M);
      } else {
        set_lost(L, O, 1u);
        add_coins(L, O, 3);
        next_move(L);
      }
      break;
    case kSteal:
      if (has_face_down(op_hand, kCaptain)) {
        set_lost(L, M, 1u);
        replace_card(L, kCaptain);
        steal_coins(L, O, M);
      } else {
        set_lost(L, O, 1u);
        next_move(L);
      }
      break;
    default:
      set_last(L, M, cp_last);
      L.err = 1u;
  }
}

// the first alive seat after M before the turn player T, or N if none
template <int N>
__device__ __forceinline__ uint32_t next_responder(const NLane<N>& L) {
  const uint32_t r = after<N>(alive_mask(L), L.M);
  const uint32_t dist = L.T >= L.M ? L.T - L.M : L.T + N - L.M;  // seats from M to T
  const uint32_t k = r ? 1u + (uint32_t)__builtin_ctz(r) : (uint32_t)N;
  return k < dist ? seat_plus<N>(L.M, k) : (uint32_t)N;
}

template <int N>
__device__ __forceinline__ void apply_decision(NLane<N>& L, uint32_t a) {
  const uint32_t M = L.M;
  L.rloser = 0u;  // cur_rewards_ cleared (coup.cc:527)
  L.rcount = 0u;
  if (a == kChallenge) {
    apply_challenge(L);
    return;
  }
  if (a >= kExchangeReturn12) {
    const uint32_t k = a - kExchangeReturn12;
    const uint32_t lo = (0x211000u >> (4u * k)) & 0xFu;
    const uint32_t hi = (0x332321u >> (4u * k)) & 0xFu;
    set_hand(L, M, hand_remove(hand_remove(hand(L, M), hi), lo));
    L.deck += (1u << (4u * hi)) + (1u << (4u * lo));  // coup.cc:794 slot-index quirk
    set_last(L, M, a);
    if (lost(L, L.O))
      next_move(L);
    else
      next_turn(L);
    return;
  }
  if (a == kLoseCard1 || a == kLoseCard2) {
    const uint32_t slot = a - kLoseCard1;
    const uint32_t h = hand(L, M);
    set_hand(L, M, hand_insert(hand_remove(h, slot), nib(h, slot) | 1u));
    set_last(L, M, a);
    set_lost(L, M, 0u);
    lose_reward(L, M);
    next_turn(L);
    return;
  }
  if (a == kPass) {
    const uint32_t pending = last(L, L.O);
    set_last(L, M, kPass);
    if (pending == kBlock) {
      next_turn(L);
      return;
    }
    const uint32_t r = pending == kSteal ? (uint32_t)N : next_responder(L);
    if (r < (uint32_t)N) {
      L.M = r;  // the next seat answers the claim
      return;
    }
    next_move(L);
    complete_claim(L, pending);
    return;
  }
  set_last(L, M, a);
  switch (a) {
    case kIncome:
      add_coins(L, M, 1);
      next_turn(L);
      break;
    case kBlock:
      next_move(L);
      break;
    default: {
      // claims and attacks: the first responder (the target of Coup /
      // Assassinate / Steal) answers, the claimant becomes the counterpart
      if (a == kCoup) add_coins(L, M, -7);
      if (a == kAssassinate) add_coins(L, M, -3);
      L.O = L.T;
      L.M = next_alive<N>(alive_mask(L), L.T);
      L.begin = 0u;
      break;
    }
  }
}

// Regrouping key of decision x at L (coup_regroup.h, the sorted step and
// rollout): Pass split by what it ends, Challenge by its outcome.
template <int N>
__device__ __forceinline__ uint32_t refine_key(const NLane<N>& L, uint32_t x) {
  if (x == kPass) {
    const uint32_t pending = last(L, L.O);
    if (pending == kBlock) return kKeyPassBlock;
    if (pending != kSteal && next_responder(L) < (uint32_t)N) return kPass;
    switch (pending) {
      case kForeignAid: return kKeyPassComplete + 0u;
      case kTax: return kKeyPassComplete + 1u;
      case kExchange: return kKeyPassComplete + 2u;
      case kSteal: return kKeyPassComplete + 3u;
      default: return kPass;
    }
  }
  if (x == kChallenge)
    return challenge_holds(last(L, L.O), last(L, L.M), hand(L, L.O)) ? kKeyChallengeLost : (uint32_t)kChallenge;
  return x;
}

// chance outcome: the initial deals go round the table twice, later deals
// to the queued player
template <int N>
__device__ __forceinline__ uint32_t deal_target(const NLane<N>& L) {
  if (L.init_left) {
    const uint32_t v = 2u * N - L.init_left;
    return v >= (uint32_t)N ? v - N : v;
  }
  return L.qp;
}

template <int N>
__device__ __forceinline__ void apply_deal(NLane<N>& L, uint32_t type) {
  const uint32_t p = deal_target(L);
  if (L.init_left)
    L.init_left -= 1u;
  else
    L.qlen -= 1u;
  L.deck -= 1u << (4u * type);
  set_hand(L, p, hand_insert(hand(L, p), 2u * type));
}

template <int N>
__device__ __forceinline__ bool apply_action(NLane<N>& L, uint32_t a) {
  if (a > 17u) return false;
  const uint32_t m = legal_mask(L);
  if (((m >> a) & 1u) == 0u) return false;
  if (m & kChanceFlag)
    apply_deal(L, a);
  else
    apply_decision(L, a);
  L.move += 1u;
  return true;
}

// Sampling contract as in coup_lane.h; the block cache tag has 7 bits of
// block index (moves up to 45 x 6 + deals < 512).
struct NRng {
  uint32_t seed_lo, seed_hi, env_id;
  uint32_t blk_tag;
  uint4 blk;

  __device__ __forceinline__ uint32_t draw(uint32_t ep, uint32_t idx) {
    const uint32_t tag = ((ep << 7) | (idx >> 2)) + 1u;
    if (tag != blk_tag) {
      blk = philox4x32_10(make_uint4(idx >> 2, ep, seed_hi, 0x436F7570u), env_id, seed_lo);
      blk_tag = tag;
    }
    const uint32_t j = idx & 3u;
    return j == 0 ? blk.x : (j == 1 ? blk.y : (j == 2 ? blk.z : blk.w));
  }
};

// A deal adds a face-down card, so it cannot end the game except by
// truncation (MaxGameLength 45 N): one terminal test, then the bound.
template <int N>
__device__ __forceinline__ void resolve_chance(NLane<N>& L, NRng& rng) {
  if (!is_chance(L) || is_terminal(L)) return;
  do {
    apply_deal(L, sample_card(L.deck, rng.draw(L.episode, L.move)));
    L.move += 1u;
  } while (is_chance(L) && L.move <= 45u * N);
}

// initial_lane + its 2N deals in straight-line form: deal k (slot k) goes to
// seat k mod N, so seat s holds the face-down kinds of deals s and s + N in
// ascending order.
// deal_episode: the same with deal k's draw from draw(k) (the episode's
// draw index k), so a caller can compute the Philox blocks elsewhere
// (k_step_sorted's grouped reset phase).
template <int N, class Draw>
__device__ __forceinline__ NLane<N> deal_episode(uint32_t episode, Draw&& draw) {
  NLane<N> L = initial_lane<N>(episode);
  L.err = L.episode == 0u ? 1u : 0u;  // the counter wrapped: this stream repeats episode 0's
  uint32_t t[2 * N];
#pragma unroll
  for (int k = 0; k < 2 * N; ++k) {
    t[k] = sample_card(L.deck, draw((uint32_t)k));
    L.deck -= 1u << (4u * t[k]);
  }
#pragma unroll
  for (int p = 0; p < N; ++p) {
    const uint32_t lo = t[p] < t[p + N] ? t[p] : t[p + N], hi = t[p] < t[p + N] ? t[p + N] : t[p];
    set_hand(L, (uint32_t)p, (2u * lo) | ((2u * hi) << 4) | 0xFF00u);
  }
  L.init_left = 0u;
  L.move = 2u * N;
  return L;
}

template <int N>
__device__ __forceinline__ NLane<N> new_episode(uint32_t episode, NRng& rng) {
  const uint32_t ep = episode & kNpEpisodeMask;
  return deal_episode<N>(episode, [&](uint32_t k) { return rng.draw(ep, k); });
}

// ObservationTensor (CoupObserver::WriteTensor, coup.cc:248-287, with
// num_players_ = N): one observer row is
//   [observer N | cards 20N | cur_move N | cards_state 8N | coins N | last_action 18N].
// obs_record keeps what the tensor reads (hands, coins, last actions, the
// mover or 7 when terminal); obs_elem is element `pos` of observer o's row.
template <int N>
__device__ __forceinline__ void obs_record(const NLane<N>& L, uint32_t* r) {
  r[0] = L.hA;
  r[1] = L.hB;
  r[2] = L.hC;
  r[3] = L.coins;
  r[4] = L.last;
  r[5] = is_terminal(L) ? 7u : L.M;
}

template <int N>
__device__ __forceinline__ float obs_elem(const uint32_t* r, uint32_t o, uint32_t pos) {
  if (pos < (uint32_t)N) return pos == o ? 1.0f : 0.0f;
  if (pos < 21u * N) {
    const uint32_t x = pos - N, q = x / 20u, s = (x - 20u * q) / 5u, v = x - 20u * q - 5u * s;
    const uint32_t k = nib((r[q >> 1] >> (16u * (q & 1u))) & 0xFFFFu, s);
    return (k != 0xFu && (k >> 1) == v && ((k & 1u) || q == o)) ? 1.0f : 0.0f;
  }
  if (pos < 22u * N) return (pos - 21u * N) == r[5] ? 1.0f : 0.0f;
  if (pos < 30u * N) {
    const uint32_t x = pos - 22u * N, q = x >> 3, s = (x >> 1) & 3u;
    const uint32_t k = nib((r[q >> 1] >> (16u * (q & 1u))) & 0xFFFFu, s);
    return (k != 0xFu && (k & 1u) == (x & 1u)) ? 1.0f : 0.0f;
  }
  if (pos < 31u * N) return (float)((r[3] >> (4u * (pos - 30u * N))) & 0xFu);
  const uint32_t x = pos - 31u * N, q = x / 18u;
  return ((r[4] >> (5u * q)) & 31u) == x - 18u * q ? 1.0f : 0.0f;
}

// First half of step_lane, up to the decision to apply: a lane that was
// terminal starts a new episode (FIRST), pending deals are resolved, the
// uniform policy draws x.  Returns kStepDone when nothing is left to apply
// (the reset, or a rejected action: `error`), else the action x.
constexpr uint32_t kStepDone = 18u;

template <int N, bool UNIFORM>
__device__ __forceinline__ uint32_t step_lane_pre(NLane<N>& L, NRng& rng, uint32_t& x, uint32_t& st, bool& error) {
  error = false;
  if (!UNIFORM && x > 127u) {  // a negative int8 action skips the lane (coup_step)
    st = 3;                    // COUP_STEP_SKIPPED
    return kStepDone;
  }
  if (is_terminal(L)) {
    L = new_episode<N>(L.episode + 1u, rng);
    st = 0;  // FIRST
    return kStepDone;
  }
  resolve_chance(L, rng);
  const uint32_t m = decision_mask(L);
  if (UNIFORM) x = m ? sample_action_select(m, rng.draw(L.episode, L.move)) : 32u;  // lanes in place
  st = 1;  // MID
  if (x > 17u || ((m >> x) & 1u) == 0u || is_terminal(L)) {
    error = true;
    return kStepDone;
  }
  return x;
}

// Second half: apply decision x, resolve the deals, auto-reset.  ret0:
// player 0's return of a game that ends here (read before the reset).
template <int N>
__device__ __forceinline__ void step_lane_post(NLane<N>& L, NRng& rng, uint32_t x, bool auto_reset, int& act,
                                               uint32_t& st, uint32_t& rl, uint32_t& rc, int32_t& ret0,
                                               bool& error) {
  const uint32_t err_before = L.err;
  apply_decision(L, x);
  L.move += 1u;
  resolve_chance(L, rng);
  error = L.err && !err_before;
  act = (int)x;
  rl = L.rloser;
  rc = L.rcount;
  if (is_terminal(L)) {
    st = 2;  // LAST
    ret0 = returns(L, 0u);
    if (auto_reset) L = new_episode<N>(L.episode + 1u, rng);
  }
}

// One rl_environment step of one lane (rl_environment.py:282-322), with
// SyncVectorEnv auto-reset when `auto_reset` (vector_env.py:40-67): the
// 2-player engine's step_lane with the N-player rules.  x is the decision
// to apply (the uniform policy's draw when UNIFORM).  Outputs: the applied
// action (-1 if none), the step type, Rewards() as (loser, count), and
// whether the lane rejected the action or hit a rules error; at LAST, ret0
// is player 0's return of the finished game.
template <int N, bool UNIFORM>
__device__ __forceinline__ void step_lane(NLane<N>& L, NRng& rng, uint32_t x, bool auto_reset, int& act,
                                          uint32_t& st, uint32_t& rl, uint32_t& rc, int32_t& ret0, bool& error) {
  act = -1;
  rl = 0;
  rc = 0;
  ret0 = 0;
  if (step_lane_pre<N, UNIFORM>(L, rng, x, st, error) != kStepDone)
    step_lane_post<N>(L, rng, x, auto_reset, act, st, rl, rc, ret0, error);
}

}  // namespace np
}  // namespace coup
