// coup_lane.h -- Coup rules on a register-resident lane (gfx950 device code).
//
// One lane = one independent 2-player game.  In HBM a lane is a 16-byte
// record (4 x u32); a kernel unpacks it into the Lane
// struct below (scalars only: no per-player arrays, so nothing spills to
// scratch through dynamic indexing), runs the step, and packs it back.
//
// Hands are 16-bit words of four nibbles, one per hand slot, holding the
// card "kind" = 2*type + face (0 = down, 1 = up); empty slots are 0xF.
// Because the reference keeps every hand sorted by (type, face)
// (coup.cc:389-391, coup.h:91-94), a hand is a sorted nibble string with
// the empties on top: inserting, removing and flipping cards are shifts and
// masks, and "slot i" in action ids (LoseCard1/2, ExchangeReturnXY) is
// nibble i.
//
// Every transition cites the reference line it reproduces.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include "coup_regroup.h"

namespace coup {

// ActionType (coup.h:65-85)
enum : uint32_t {
  kIncome = 0, kForeignAid = 1, kCoup = 2, kTax = 3, kAssassinate = 4,
  kExchange = 5, kSteal = 6, kLoseCard1 = 7, kLoseCard2 = 8, kPass = 9,
  kBlock = 10, kChallenge = 11, kExchangeReturn12 = 12, kExchangeReturn34 = 17,
  kNoAction = 31  // ActionType::kNone in the packed record
};
// CardType (coup.h:50-57)
enum : uint32_t { kAssassin = 0, kAmbassador = 1, kCaptain = 2, kContessa = 3, kDuke = 4 };

constexpr uint32_t kEmptyHand = 0xFFFFu;
constexpr uint32_t kInitialDeck = 0x33333u;  // kNumEachCardInDeck = 3 of each type
constexpr uint32_t kMaxGameLength = 90;      // coup.h:219
constexpr uint32_t kChanceFlag = 1u << 31;
// 28-bit episode counter: w3 [31:7] holds bits 24..0, w2 [31:29] bits 27..25.
// It keys the lane's Philox counter, so past 2^28 episodes a lane would
// replay its first games: the wrap sets the record's error flag instead of
// passing silently (new_episode).
constexpr uint32_t kEpisodeMask = 0xFFFFFFFu;

struct Lane {
  uint32_t h0, h1;      // hands of P1 / P2 (16-bit nibble strings)
  uint32_t deck;        // 5 x 4-bit counts (can exceed 3: coup.cc:794 quirk)
  uint32_t c0, c1;      // coins
  int32_t r0;           // cur_rewards_[0]; cur_rewards_[1] == -r0 always
  uint32_t err;         // set where the reference would SpielFatalError
  uint32_t l0, l1;      // last_action (kNoAction = None)
  uint32_t lost0, lost1;
  uint32_t qlen, qids;  // deal_card_to_ FIFO: length, entry j = bit j
  uint32_t T, M, begin; // cur_player_turn_, cur_player_move_, is_turn_begin_
  uint32_t move, turn;  // move_number_, turn_number_
  uint32_t episode;
};

// ---------------------------------------------------------------- packing

__device__ __forceinline__ Lane unpack(uint4 w) {
  Lane L;
  L.h0 = w.x & 0xFFFFu;
  L.h1 = w.x >> 16;
  L.deck = w.y & 0xFFFFFu;
  L.c0 = (w.y >> 20) & 0xFu;
  L.c1 = (w.y >> 24) & 0xFu;
  L.r0 = (int32_t)((w.y >> 28) & 0x7u) - 2;
  L.err = w.y >> 31;
  L.l0 = w.z & 0x1Fu;
  L.l1 = (w.z >> 5) & 0x1Fu;
  L.lost0 = (w.z >> 10) & 1u;
  L.lost1 = (w.z >> 11) & 1u;
  L.qlen = (w.z >> 12) & 0x7u;
  L.qids = (w.z >> 15) & 0xFu;
  L.T = (w.z >> 19) & 1u;
  L.M = (w.z >> 20) & 1u;
  L.begin = (w.z >> 21) & 1u;
  L.move = (w.z >> 22) & 0x7Fu;
  L.turn = w.w & 0x7Fu;
  L.episode = (w.w >> 7) | ((w.z >> 29) << 25);
  return L;
}

__device__ __forceinline__ uint4 pack(const Lane& L) {
  uint4 w;
  w.x = L.h0 | (L.h1 << 16);
  w.y = L.deck | (L.c0 << 20) | (L.c1 << 24) | ((uint32_t)(L.r0 + 2) << 28) | (L.err << 31);
  w.z = L.l0 | (L.l1 << 5) | (L.lost0 << 10) | (L.lost1 << 11) | (L.qlen << 12) | (L.qids << 15) |
        (L.T << 19) | (L.M << 20) | (L.begin << 21) | (L.move << 22) | (((L.episode >> 25) & 7u) << 29);
  w.w = L.turn | (L.episode << 7);
  return w;
}

// CoupState::CoupState (coup.cc:393-428): deck 3 of each, P1 1 coin, P2 2
// coins, no last actions, deal queue [P1, P2, P1, P2], P1 to move.
__device__ __forceinline__ Lane initial_lane(uint32_t episode) {
  Lane L;
  L.h0 = kEmptyHand;
  L.h1 = kEmptyHand;
  L.deck = kInitialDeck;
  L.c0 = 1;
  L.c1 = 2;
  L.r0 = 0;
  L.err = 0;
  L.l0 = kNoAction;
  L.l1 = kNoAction;
  L.lost0 = 0;
  L.lost1 = 0;
  L.qlen = 4;
  L.qids = 0xAu;  // entries 0..3 = 0, 1, 0, 1
  L.T = 0;
  L.M = 0;
  L.begin = 1;
  L.move = 0;
  L.turn = 0;
  L.episode = episode & kEpisodeMask;
  return L;
}

// --------------------------------------------------------- hand nibbles

__device__ __forceinline__ uint32_t nib(uint32_t h, uint32_t i) { return (h >> (4u * i)) & 0xFu; }

// bit 4i set where nibble i == k (k in 0..15)
__device__ __forceinline__ uint32_t nib_eq(uint32_t h, uint32_t k) {
  uint32_t x = (h ^ (k * 0x1111u)) & 0xFFFFu;
  return ~(x | (x >> 1) | (x >> 2) | (x >> 3)) & 0x1111u;
}

// HasFaceDownCard (coup.cc:379-387): some slot holds kind 2*type
__device__ __forceinline__ bool has_face_down(uint32_t h, uint32_t type) { return nib_eq(h, 2u * type) != 0; }

// hand holds a face-down card (kinds are even when face down; 0xF is odd)
__device__ __forceinline__ bool any_face_down(uint32_t h) { return (~h & 0x1111u) != 0; }

// IsTerminal's per-player test (coup.cc:994-1006): fewer than two cards
// (mid-deal) or any face-down card
__device__ __forceinline__ bool alive(uint32_t h) { return nib(h, 1) == 0xFu || any_face_down(h); }

__device__ __forceinline__ uint32_t hand_size(uint32_t h) {
  return (nib(h, 0) != 0xFu) + (nib(h, 1) != 0xFu) + (nib(h, 2) != 0xFu) + (nib(h, 3) != 0xFu);
}

__device__ __forceinline__ uint32_t face_up_count(uint32_t h) {
  uint32_t empty = h & (h >> 1) & (h >> 2) & (h >> 3) & 0x1111u;
  return __popc(h & 0x1111u) - __popc(empty);
}

// Insert kind k keeping the nibble string sorted (push_back + SortCards,
// coup.cc:508-510).  The hand has an empty slot.
__device__ __forceinline__ uint32_t hand_insert(uint32_t h, uint32_t k) {
  uint32_t pos = (nib(h, 0) <= k) + (nib(h, 1) <= k) + (nib(h, 2) <= k) + (nib(h, 3) <= k);
  uint32_t sh = 4u * pos;
  uint32_t keep = (1u << sh) - 1u;
  uint32_t above = ~((1u << (sh + 4u)) - 1u);
  return (h & keep) | (k << sh) | ((h << 4) & 0xFFFFu & above);
}

// Erase slot p (vector::erase, coup.cc:477, 793)
__device__ __forceinline__ uint32_t hand_remove(uint32_t h, uint32_t p) {
  uint32_t keep = (1u << (4u * p)) - 1u;
  return (h & keep) | ((h >> 4) & ~keep & 0x0FFFu) | 0xF000u;
}

// ----------------------------------------------------- per-player access

#define COUP_PGET(L, f, p) ((p) ? (L).f##1 : (L).f##0)
#define COUP_PSET(L, f, p, v)          \
  do {                                 \
    uint32_t _v = (v);                 \
    bool _p = (p) != 0;                \
    (L).f##0 = _p ? (L).f##0 : _v;     \
    (L).f##1 = _p ? _v : (L).f##1;     \
  } while (0)

__device__ __forceinline__ uint32_t deck_count(uint32_t deck, uint32_t t) { return (deck >> (4u * t)) & 0xFu; }

__device__ __forceinline__ bool is_terminal(const Lane& L) {
  // IsTerminal (coup.cc:989-1010): move_number_ > MaxGameLength, or at most
  // one player alive
  return L.move > kMaxGameLength || !(alive(L.h0) && alive(L.h1));
}

__device__ __forceinline__ bool is_chance(const Lane& L) { return L.qlen != 0; }

// Returns()[0] (coup.cc:1016-1032): face-up(P2) - face-up(P1); Returns()[1]
// is its negation.
__device__ __forceinline__ int32_t return0(const Lane& L) {
  return (int32_t)face_up_count(L.h1) - (int32_t)face_up_count(L.h0);
}

// CurrentPlayer (coup.cc:458-466)
__device__ __forceinline__ int current_player(const Lane& L) {
  return is_terminal(L) ? -4 : (is_chance(L) ? -1 : (int)L.M);
}

// ------------------------------------------------------------ legal mask

// LegalLoseCardActions (coup.cc:811-822): only slots 0 and 1 are offered
__device__ __forceinline__ uint32_t lose_card_mask(uint32_t h) {
  return ((nib(h, 0) & 1u) ? 0u : (1u << kLoseCard1)) | ((nib(h, 1) & 1u) ? 0u : (1u << kLoseCard2));
}

// Chance-node legal actions (coup.cc:828-836): card types still in the deck
__device__ __forceinline__ uint32_t chance_mask(uint32_t deck) {
  uint32_t m = 0;
#pragma unroll
  for (uint32_t t = 0; t < 5; ++t) m |= (deck_count(deck, t) != 0) << t;
  return m;
}

// Decision-node LegalActions (coup.cc:838-937) as an 18-bit mask.  Returns 0
// where the reference raises "Invalid action progression".
__device__ __forceinline__ uint32_t decision_mask(const Lane& L) {
  const uint32_t M = L.M, O = M ^ 1u;
  const uint32_t cp_coins = COUP_PGET(L, c, M), op_coins = COUP_PGET(L, c, O);
  const uint32_t cp_last = COUP_PGET(L, l, M), op_last = COUP_PGET(L, l, O);
  const uint32_t cp_hand = COUP_PGET(L, h, M);
  if (L.begin) {
    if (cp_coins >= 10) return 1u << kCoup;
    uint32_t m = (1u << kIncome) | (1u << kForeignAid) | (1u << kTax) | (1u << kExchange);
    m |= (cp_coins >= 7) ? (1u << kCoup) : 0u;
    m |= (cp_coins >= 3) ? (1u << kAssassinate) : 0u;
    m |= (op_coins > 0) ? (1u << kSteal) : 0u;
    return m;
  }
  if (COUP_PGET(L, lost, M)) return lose_card_mask(cp_hand);
  if (M != L.T) {
    // responses to the turn player's claim (coup.cc:860-887)
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
    // coup.cc:889-928: all pairs of returned slots, minus pairs containing
    // the first face-up slot.  Table: for face-up slot s, the 6-bit set of
    // ExchangeReturn ids (relative to 12) that contain s.
    if (nib(cp_hand, 3) == 0xFu) return 0u;  // fewer than 4 cards
    uint32_t up = cp_hand & 0x1111u;
    if (up == 0) return 0x3Fu << kExchangeReturn12;
    uint32_t s = (uint32_t)__builtin_ctz(up) >> 2;
    uint32_t excl = (0x07u | (0x19u << 6) | (0x2Au << 12) | (0x34u << 18)) >> (6u * s);
    return ((~excl) & 0x3Fu) << kExchangeReturn12;
  }
  if (op_last == kBlock) return (1u << kPass) | (1u << kChallenge);
  return 0u;
}

// LegalActionsMask of the current player: decision mask, chance mask with
// kChanceFlag, or 0 when terminal.
__device__ __forceinline__ uint32_t legal_mask(const Lane& L) {
  if (is_terminal(L)) return 0u;
  if (is_chance(L)) return chance_mask(L.deck) | kChanceFlag;
  return decision_mask(L);
}

// ----------------------------------------------------------- transitions

__device__ __forceinline__ void next_turn(Lane& L) {
  // NextPlayerTurn (coup.cc:1079-1086)
  L.T ^= 1u;
  L.M = L.T;
  L.turn += 1u;
  L.begin = 1u;
}

__device__ __forceinline__ void next_move(Lane& L) {
  // NextPlayerMove (coup.cc:1088-1092)
  L.M ^= 1u;
  L.begin = 0u;
}

// +d to cur_rewards_[M], -d to cur_rewards_[O]
__device__ __forceinline__ void reward_mover(Lane& L, int32_t d) { L.r0 += L.M ? -d : d; }

__device__ __forceinline__ void queue_push(Lane& L, uint32_t p) {
  L.qids |= p << L.qlen;
  L.qlen += 1u;
}

// ChallengeFailReplaceCard (coup.cc:468-486): the opponent reveals the
// claimed card, it goes back to the deck and a replacement deal is queued.
__device__ __forceinline__ void replace_card(Lane& L, uint32_t type) {
  const uint32_t O = L.M ^ 1u;
  const uint32_t h = COUP_PGET(L, h, O);
  const uint32_t hit = nib_eq(h, 2u * type);
  if (hit == 0) {
    L.err = 1u;
    return;
  }
  L.deck += 1u << (4u * type);
  COUP_PSET(L, h, O, hand_remove(h, (uint32_t)__builtin_ctz(hit) >> 2));
  queue_push(L, O);
}

// Flip slots 0 and 1 of player p face up (no re-sort), +/-1 reward per
// flipped card to the mover: coup.cc:660-669 (p = O, d = +1) and
// coup.cc:733-742 (p = M, d = -1).
__device__ __forceinline__ void flip_two(Lane& L, uint32_t p, int32_t d) {
  uint32_t h = COUP_PGET(L, h, p);
#pragma unroll
  for (uint32_t i = 0; i < 2; ++i) {
    if ((nib(h, i) & 1u) == 0) {
      h |= 1u << (4u * i);
      reward_mover(L, d);
    }
  }
  COUP_PSET(L, h, p, h);
}

// Second half of FA / Tax / Exchange / Steal, entered through the Pass
// recursion (coup.cc:628) or the lost Exchange challenge (coup.cc:718); the
// mover is the original actor and is_turn_begin_ is false here.
__device__ __forceinline__ void complete_claim(Lane& L, uint32_t a) {
  const uint32_t M = L.M, O = M ^ 1u;
  switch (a) {
    case kForeignAid:  // coup.cc:542-546
      COUP_PSET(L, c, M, COUP_PGET(L, c, M) + 2u);
      next_turn(L);
      break;
    case kTax:  // coup.cc:561-565
      COUP_PSET(L, c, M, COUP_PGET(L, c, M) + 3u);
      next_turn(L);
      break;
    case kExchange:  // coup.cc:581-587: draw two cards
      queue_push(L, M);
      queue_push(L, M);
      break;
    case kSteal: {  // coup.cc:597-603
      const uint32_t oc = COUP_PGET(L, c, O);
      const uint32_t k = oc > 1u ? 2u : 1u;
      COUP_PSET(L, c, M, COUP_PGET(L, c, M) + k);
      COUP_PSET(L, c, O, oc - k);
      next_turn(L);
      break;
    }
    default:
      L.err = 1u;
  }
}

// Challenge (coup.cc:635-771)
__device__ __forceinline__ void apply_challenge(Lane& L) {
  const uint32_t M = L.M, O = M ^ 1u;
  const uint32_t op_last = COUP_PGET(L, l, O);
  const uint32_t cp_last = COUP_PGET(L, l, M);
  const uint32_t op_hand = COUP_PGET(L, h, O);
  COUP_PSET(L, l, M, kChallenge);
  if (op_last == kBlock) {
    // the turn player challenges the block of its own claim (coup.cc:636-693)
    if (cp_last == kForeignAid) {
      if (has_face_down(op_hand, kDuke)) {
        COUP_PSET(L, lost, M, 1u);
        replace_card(L, kDuke);
      } else {
        COUP_PSET(L, lost, O, 1u);
        COUP_PSET(L, c, M, COUP_PGET(L, c, M) + 2u);
        next_move(L);
      }
    } else if (cp_last == kAssassinate) {
      if (has_face_down(op_hand, kContessa)) {
        COUP_PSET(L, lost, M, 1u);
        replace_card(L, kContessa);
      } else {
        flip_two(L, O, +1);
      }
    } else if (cp_last == kSteal) {
      if (has_face_down(op_hand, kCaptain)) {
        COUP_PSET(L, lost, M, 1u);
        replace_card(L, kCaptain);
      } else if (has_face_down(op_hand, kAmbassador)) {
        COUP_PSET(L, lost, M, 1u);
        replace_card(L, kAmbassador);
      } else {
        COUP_PSET(L, lost, O, 1u);
        const uint32_t oc = COUP_PGET(L, c, O);
        const uint32_t k = oc > 1u ? 2u : 1u;
        COUP_PSET(L, c, M, COUP_PGET(L, c, M) + k);
        COUP_PSET(L, c, O, oc - k);
        next_move(L);
      }
    } else {
      COUP_PSET(L, l, M, cp_last);  // the reference aborts before touching state
      L.err = 1u;
    }
    return;
  }
  switch (op_last) {
    case kTax:  // coup.cc:694-706
      if (has_face_down(op_hand, kDuke)) {
        COUP_PSET(L, lost, M, 1u);
        replace_card(L, kDuke);
        COUP_PSET(L, c, O, COUP_PGET(L, c, O) + 3u);
      } else {
        COUP_PSET(L, lost, O, 1u);
        next_move(L);
      }
      break;
    case kExchange:  // coup.cc:708-725
      if (has_face_down(op_hand, kAmbassador)) {
        COUP_PSET(L, lost, M, 1u);
        replace_card(L, kAmbassador);
        next_move(L);
        complete_claim(L, kExchange);  // queue: exchanger x3
      } else {
        COUP_PSET(L, lost, O, 1u);
        next_move(L);
      }
      break;
    case kAssassinate:  // coup.cc:727-749
      if (has_face_down(op_hand, kAssassin)) {
        flip_two(L, M, -1);
      } else {
        COUP_PSET(L, lost, O, 1u);
        COUP_PSET(L, c, O, COUP_PGET(L, c, O) + 3u);  // refund
        next_move(L);
      }
      break;
    case kSteal:  // coup.cc:751-767 (the Ambassador does not count here)
      if (has_face_down(op_hand, kCaptain)) {
        COUP_PSET(L, lost, M, 1u);
        replace_card(L, kCaptain);
        const uint32_t mc = COUP_PGET(L, c, M);
        const uint32_t k = mc > 1u ? 2u : 1u;
        COUP_PSET(L, c, O, COUP_PGET(L, c, O) + k);
        COUP_PSET(L, c, M, mc - k);
      } else {
        COUP_PSET(L, lost, O, 1u);
        next_move(L);
      }
      break;
    default:
      COUP_PSET(L, l, M, cp_last);
      L.err = 1u;
  }
}

// The decision of a regrouping key (coup_regroup.h).
__device__ __forceinline__ uint32_t key_action(uint32_t k) {
  return k < kKeyPassBlock ? k : (k < kKeyChallengeLost ? (uint32_t)kPass : (uint32_t)kChallenge);
}

// The claimed card a Challenge tests: does the challenged player (O) hold
// it?  apply_challenge's first branch (coup.cc:635-771).
__device__ __forceinline__ bool challenge_holds(uint32_t op_last, uint32_t cp_last, uint32_t h) {
  if (op_last == kBlock)
    return cp_last == kForeignAid    ? has_face_down(h, kDuke)
           : cp_last == kAssassinate ? has_face_down(h, kContessa)
                                     : has_face_down(h, kCaptain) || has_face_down(h, kAmbassador);
  return op_last == kTax        ? has_face_down(h, kDuke)
         : op_last == kExchange ? has_face_down(h, kAmbassador)
         : op_last == kAssassinate ? has_face_down(h, kAssassin)
                                    : has_face_down(h, kCaptain);
}

// Regrouping key of decision x at L: Pass split by what it ends, Challenge
// by its outcome (the 2-player sorted kernels).
__device__ __forceinline__ uint32_t refine_key(const Lane& L, uint32_t x) {
  const uint32_t O = L.M ^ 1u;
  if (x == kPass) {
    switch (COUP_PGET(L, l, O)) {
      case kBlock: return kKeyPassBlock;
      case kForeignAid: return kKeyPassComplete + 0u;
      case kTax: return kKeyPassComplete + 1u;
      case kExchange: return kKeyPassComplete + 2u;
      case kSteal: return kKeyPassComplete + 3u;
      default: return kPass;
    }
  }
  if (x == kChallenge)
    return challenge_holds(COUP_PGET(L, l, O), COUP_PGET(L, l, L.M), COUP_PGET(L, h, O)) ? kKeyChallengeLost
                                                                                        : (uint32_t)kChallenge;
  return x;
}

// Decision branch of DoApplyAction (coup.cc:522-808) for a LEGAL action,
// written as the reference's control flow (kept for A/B builds:
// -DCOUP_RULES_V1).  Claims (FA / Tax / Exchange / Steal) are only legal at
// turn begin, so the direct call always takes their "announce" half.
__device__ __forceinline__ void apply_decision_v1(Lane& L, uint32_t a) {
  const uint32_t M = L.M, O = M ^ 1u;
  L.r0 = 0;  // cur_rewards_ = {0, 0} (coup.cc:527)
  if (a == kChallenge) {
    apply_challenge(L);
    return;
  }
  if (a >= kExchangeReturn12) {
    // coup.cc:773-804: erase the higher slot, then the lower; each erased
    // slot INDEX is credited to the deck (coup.cc:794 reference quirk)
    const uint32_t k = a - kExchangeReturn12;
    const uint32_t lo = (0x211000u >> (4u * k)) & 0xFu;  // {0,0,0,1,1,2}
    const uint32_t hi = (0x332321u >> (4u * k)) & 0xFu;  // {1,2,3,2,3,3}
    const uint32_t h = COUP_PGET(L, h, M);
    COUP_PSET(L, h, M, hand_remove(hand_remove(h, hi), lo));
    L.deck += (1u << (4u * hi)) + (1u << (4u * lo));
    COUP_PSET(L, l, M, a);
    if (COUP_PGET(L, lost, O))
      next_move(L);
    else
      next_turn(L);
    return;
  }
  if (a == kLoseCard1 || a == kLoseCard2) {
    // coup.cc:605-616: flip the slot face up, re-sort, -1/+1 reward
    const uint32_t slot = a - kLoseCard1;
    const uint32_t h = COUP_PGET(L, h, M);
    const uint32_t kind = nib(h, slot) | 1u;
    COUP_PSET(L, h, M, hand_insert(hand_remove(h, slot), kind));
    COUP_PSET(L, l, M, a);
    COUP_PSET(L, lost, M, 0u);
    reward_mover(L, -1);
    next_turn(L);
    return;
  }
  if (a == kPass) {
    // coup.cc:618-629
    const uint32_t pending = COUP_PGET(L, l, O);
    COUP_PSET(L, l, M, kPass);
    if (pending == kBlock) {
      next_turn(L);
    } else {
      next_move(L);
      complete_claim(L, pending);
    }
    return;
  }
  COUP_PSET(L, l, M, a);
  switch (a) {
    case kIncome:  // coup.cc:531-534
      COUP_PSET(L, c, M, COUP_PGET(L, c, M) + 1u);
      next_turn(L);
      break;
    case kCoup:  // coup.cc:548-553
      COUP_PSET(L, c, M, COUP_PGET(L, c, M) - 7u);
      next_move(L);
      break;
    case kAssassinate:  // coup.cc:567-573: paid even if blocked/challenged
      COUP_PSET(L, c, M, COUP_PGET(L, c, M) - 3u);
      next_move(L);
      break;
    default:  // FA, Tax, Exchange, Steal announce; Block (coup.cc:631-633)
      next_move(L);
      break;
  }
}

// The same transition as apply_decision_v1, computed as one set of effects
// per lane instead of the reference's nested branches.  A wave holds lanes
// taking many different paths through DoApplyAction, so it executes the
// union of them; here every lane evaluates the same straight-line effect
// formulas (coin deltas, a coin transfer, lost flags, queue pushes, the
// turn transition) and at most one hand operation of each kind, so the
// eight ChallengeFailReplaceCard sites of coup.cc:635-771 become one.
//
// Effects, by action (M mover, O = M ^ 1; citations as in v1):
//   Income (531-534)      +1 coin to M, NextPlayerTurn
//   Coup/Assassinate      -7 / -3 coins to M, NextPlayerMove (548-553, 567-573)
//   FA/Tax/Exch/Steal/Block announce: NextPlayerMove (536-603, 631-633)
//   LoseCard (605-616)    flip slot, re-sort, lost cleared, -1 reward to M, NextPlayerTurn
//   ExchangeReturn (773-804) erase two slots, credit the slot INDICES to the deck,
//                         O lost a challenge ? NextPlayerMove : NextPlayerTurn
//   Pass (618-629)        pending Block: NextPlayerTurn; else the claim completes for O
//                         (FA +2, Tax +3, Steal: k from M to O, then NextPlayerTurn --
//                         NextPlayerMove followed by NextPlayerTurn is NextPlayerTurn;
//                         Exchange: two deals to O, NextPlayerMove)
//   Challenge (635-771)   claim = M's own last action if O blocked it, else O's claim;
//                         the claimed card t1 (and the Ambassador for a blocked Steal);
//                         O holds it face down ("has") or not:
//                           has: M loses the challenge and O's card is replaced
//                                (one deal to O), except a claimed Assassinate: M's two
//                                cards flip (-1 each); Tax +3 to O; Steal: k from M to O;
//                                Exchange: NextPlayerMove and two more deals to O
//                           not: O loses the challenge and NextPlayerMove, except a
//                                blocked Assassinate: O's two cards flip (+1 each to M);
//                                blocked FA +2 to M; blocked Steal: k from O to M;
//                                claimed Assassinate: +3 refund to O
//   k = the giver's coins > 1 ? 2 : 1.
__device__ __forceinline__ void apply_decision_v2(Lane& L, uint32_t a) {
  const uint32_t M = L.M, O = M ^ 1u;
  uint32_t cp_h = COUP_PGET(L, h, M), op_h = COUP_PGET(L, h, O);
  const uint32_t cp_c = COUP_PGET(L, c, M), op_c = COUP_PGET(L, c, O);
  const uint32_t cp_l = COUP_PGET(L, l, M), op_l = COUP_PGET(L, l, O);
  const uint32_t cp_lost = COUP_PGET(L, lost, M), op_lost = COUP_PGET(L, lost, O);

  const bool is_chal = a == kChallenge;
  const bool is_pass = a == kPass;
  const bool is_lose = a == kLoseCard1 || a == kLoseCard2;
  const bool is_xret = a >= kExchangeReturn12;

  // --- the challenged claim
  const bool blk = op_l == kBlock;
  const uint32_t claim = blk ? cp_l : op_l;
  // claimed card by claim id, 3 bits per action id (7 = cannot be challenged):
  // blocked FA -> Duke, blocked Assassinate -> Contessa, blocked Steal ->
  // Captain; Tax -> Duke, Exchange -> Ambassador, Assassinate -> Assassin,
  // Steal -> Captain
  constexpr uint64_t kBlockCard = (0x3FFFFFFFFFFFFFFFull & ~((7ull << 3) | (7ull << 12) | (7ull << 18))) |
                                  ((uint64_t)kDuke << 3) | ((uint64_t)kContessa << 12) | ((uint64_t)kCaptain << 18);
  constexpr uint64_t kClaimCard = (0x3FFFFFFFFFFFFFFFull & ~((7ull << 9) | (7ull << 15) | (7ull << 12) | (7ull << 18))) |
                                  ((uint64_t)kDuke << 9) | ((uint64_t)kAmbassador << 15) |
                                  ((uint64_t)kAssassin << 12) | ((uint64_t)kCaptain << 18);
  const uint32_t cidx = claim < 18u ? claim : 19u;  // None (31) -> a field of 7s
  const uint32_t t1 = (uint32_t)(((blk ? kBlockCard : kClaimCard) >> (3u * cidx)) & 7u);
  const bool valid = t1 != 7u;
  const bool h1 = valid && nib_eq(op_h, 2u * t1) != 0u;
  const bool h2 = blk && claim == kSteal && nib_eq(op_h, 2u * kAmbassador) != 0u;
  const bool has = h1 || h2;
  const bool ass = claim == kAssassinate;
  const bool flip_o = is_chal && blk && ass && !has;
  const bool flip_m = is_chal && !blk && ass && has;
  const bool do_replace = is_chal && has && !(!blk && ass);
  const bool lose_op = is_chal && valid && !has && !(blk && ass);
  const bool exch_more = (is_pass && op_l == kExchange) || (is_chal && !blk && claim == kExchange && has);
  const bool pass_ok = op_l == kBlock || op_l == kForeignAid || op_l == kTax || op_l == kExchange || op_l == kSteal;

  // --- coins: fixed deltas and one transfer of k
  uint32_t dcp = 0u, dop = 0u;
  dcp = a == kIncome ? 1u : dcp;
  dcp = a == kCoup ? (uint32_t)-7 : dcp;
  dcp = a == kAssassinate ? (uint32_t)-3 : dcp;
  dcp = (is_chal && blk && claim == kForeignAid && !has) ? 2u : dcp;
  dop = (is_pass && op_l == kForeignAid) ? 2u : dop;
  dop = (is_pass && op_l == kTax) ? 3u : dop;
  dop = (is_chal && !blk && ((claim == kTax && has) || (ass && !has))) ? 3u : dop;
  const bool give_cp = (is_pass && op_l == kSteal) || (is_chal && !blk && claim == kSteal && has);
  const bool give_op = is_chal && blk && claim == kSteal && !has;
  const uint32_t k_cp = cp_c > 1u ? 2u : 1u, k_op = op_c > 1u ? 2u : 1u;
  const uint32_t k = give_cp ? k_cp : (give_op ? k_op : 0u);
  const uint32_t new_cp_c = cp_c + dcp + (give_op ? k : 0u) - (give_cp ? k : 0u);
  const uint32_t new_op_c = op_c + dop + (give_cp ? k : 0u) - (give_op ? k : 0u);

  // --- hands
  int32_t rew = 0;  // cur_rewards_ of the mover (O gets -rew)
  if (is_lose) {
    const uint32_t slot = a - kLoseCard1;
    cp_h = hand_insert(hand_remove(cp_h, slot), nib(cp_h, slot) | 1u);
    rew = -1;
  } else if (is_xret) {
    const uint32_t kk = a - kExchangeReturn12;
    const uint32_t lo = (0x211000u >> (4u * kk)) & 0xFu, hi = (0x332321u >> (4u * kk)) & 0xFu;
    cp_h = hand_remove(hand_remove(cp_h, hi), lo);
    L.deck += (1u << (4u * hi)) + (1u << (4u * lo));  // the slot INDEX (coup.cc:794 quirk)
  }
  if (do_replace) {
    const uint32_t rtype = h1 ? t1 : kAmbassador;
    op_h = hand_remove(op_h, (uint32_t)__builtin_ctz(nib_eq(op_h, 2u * rtype)) >> 2);
    L.deck += 1u << (4u * rtype);
  }
  if (flip_o || flip_m) {  // no re-sort (coup.cc:660-669, 733-742)
    uint32_t h = flip_o ? op_h : cp_h;
    const uint32_t down = ~h & 0x11u;  // slots 0 and 1 face down
    h |= down;
    const int32_t n = (int32_t)__popc(down);
    rew = flip_o ? n : -n;
    op_h = flip_o ? h : op_h;
    cp_h = flip_o ? cp_h : h;
  }

  // --- write back by seat
  const uint32_t new_cp_l = (is_chal && !valid) ? cp_l : (is_chal ? (uint32_t)kChallenge : a);
  const uint32_t new_cp_lost = is_lose ? 0u : (do_replace ? 1u : cp_lost);
  const uint32_t new_op_lost = lose_op ? 1u : op_lost;
  L.h0 = M ? op_h : cp_h;
  L.h1 = M ? cp_h : op_h;
  L.c0 = M ? new_op_c : new_cp_c;
  L.c1 = M ? new_cp_c : new_op_c;
  L.l0 = M ? op_l : new_cp_l;
  L.l1 = M ? new_cp_l : op_l;
  L.lost0 = M ? new_op_lost : new_cp_lost;
  L.lost1 = M ? new_cp_lost : new_op_lost;
  L.r0 = M ? -rew : rew;  // cur_rewards_ = {0, 0} first (coup.cc:527)
  L.err |= ((is_chal && !valid) || (is_pass && !pass_ok)) ? 1u : 0u;

  // --- deals queued for O: the replacement, then two Exchange draws
  const uint32_t npush = (do_replace ? 1u : 0u) + (exch_more ? 2u : 0u);
  L.qids |= (O ? (1u << npush) - 1u : 0u) << L.qlen;
  L.qlen += npush;

  // --- turn transition
  const bool nt = a == kIncome || is_lose || (is_xret && !op_lost) || (is_pass && pass_ok && op_l != kExchange);
  const bool nm = (a >= kForeignAid && a <= kSteal) || a == kBlock || (is_xret && op_lost) ||
                  (is_pass && !(pass_ok && op_l != kExchange)) || lose_op || (is_chal && exch_more);
  if (nt) {
    L.T ^= 1u;
    L.M = L.T;
    L.turn += 1u;
    L.begin = 1u;
  } else if (nm) {
    L.M ^= 1u;
    L.begin = 0u;
  }
}

#ifdef COUP_RULES_V1
__device__ __forceinline__ void apply_decision(Lane& L, uint32_t a) { apply_decision_v1(L, a); }
#else
__device__ __forceinline__ void apply_decision(Lane& L, uint32_t a) { apply_decision_v2(L, a); }
#endif

// Chance branch of DoApplyAction (coup.cc:491-520): deal card `type` to the
// queue front, keep the hand sorted.
__device__ __forceinline__ void apply_deal(Lane& L, uint32_t type) {
  const uint32_t p = L.qids & 1u;
  L.qids >>= 1;
  L.qlen -= 1u;
  L.deck -= 1u << (4u * type);
  COUP_PSET(L, h, p, hand_insert(COUP_PGET(L, h, p), 2u * type));
}

// ---------------------------------------------------------------- history
//
// Optional per-lane action history (State::history_ + the chance-deal
// owner map history_chance_deal_player_, spiel.h:733, coup.h:182), one byte
// per history index: [4:0] action id or card type, [5] chance deal,
// [6] acting player (decision) or receiving player (deal).  Needed by the
// InformationStateTensor (coup.cc:230-245) and the strings.
constexpr uint32_t kHistoryBytes = 96;  // >= MaxGameLength + 1 = 91 entries

__device__ __forceinline__ uint32_t hist_decision(uint32_t a, uint32_t player) { return a | (player << 6); }
__device__ __forceinline__ uint32_t hist_deal(uint32_t type, uint32_t to) { return type | 0x20u | (to << 6); }

struct NoHistory {
  __device__ __forceinline__ void record(uint32_t, uint32_t) {}
};

// Entries recorded during one transition, held in registers as 16-bit
// (index << 8 | byte) records in a 12-deep shift register (newest in the low
// bits of q0).  One env step records at most 4 pending deals + 1 decision +
// 3 deals + 4 deals of an auto-reset = 12.  The rules themselves never touch
// memory; the kernel flushes the records afterwards, oldest first.
struct RegHistory {
  uint64_t q0 = 0, q1 = 0, q2 = 0;
  uint32_t count = 0;
  __device__ __forceinline__ void record(uint32_t idx, uint32_t entry) {
    q2 = (q2 << 16) | (q1 >> 48);
    q1 = (q1 << 16) | (q0 >> 48);
    q0 = (q0 << 16) | (uint64_t)((idx << 8) | (entry & 0xFFu));
    count += 1u;
  }
  // record k, 0 = newest
  __device__ __forceinline__ uint32_t get(uint32_t k) const {
    const uint64_t w = k < 4u ? q0 : (k < 8u ? q1 : q2);
    return (uint32_t)(w >> (16u * (k & 3u))) & 0xFFFFu;
  }
  // write the records into a lane's history bytes, oldest first.  Fully
  // unrolled so every get() has a constant k: a run-time k selects between
  // the three words, which LLVM lowers to an indexed load from scratch.
  __device__ __forceinline__ void flush(uint8_t* __restrict__ bytes) const {
    const uint32_t n = count < 12u ? count : 12u;
#pragma unroll
    for (int k = 11; k >= 0; --k) {
      if ((uint32_t)k < n) {
        const uint32_t r = get((uint32_t)k);
        const uint32_t idx = r >> 8;
        if (idx < kHistoryBytes) bytes[idx] = (uint8_t)(r & 0xFFu);
      }
    }
  }
};

// State::ApplyAction (spiel.cc:322-331) with a legality check.  Returns false
// (lane untouched) for an illegal action.  The history entry is recorded at
// index move_number_, like history_.push_back.
template <class H>
__device__ __forceinline__ bool apply_action(Lane& L, uint32_t a, H& hist) {
  if (a > 17u) return false;
  const uint32_t m = legal_mask(L);
  if (((m >> a) & 1u) == 0u) return false;
  if (m & kChanceFlag) {
    hist.record(L.move, hist_deal(a, L.qids & 1u));
    apply_deal(L, a);
  } else {
    hist.record(L.move, hist_decision(a, L.M));
    apply_decision(L, a);
  }
  L.move += 1u;
  return true;
}

// ------------------------------------------------ unchecked ApplyAction
//
// pyspiel binds apply_action to State::ApplyAction (pyspiel.cc:266,
// spiel.cc:322-331), which applies an action WITHOUT checking LegalActions:
// DoApplyAction's own checks decide.  The reference's scripts rely on it
// (policy_analysis.py:298 answers a Tax with Block, outside LegalActions,
// coup.cc:867-871).  Per-game ops and caller-action steps apply actions
// this way unless the caller asks for the legality check.  The transition
// below is coup.cc:522-808 for ANY decision at a decision node, in the
// reference's branch order, including the branches legal play never
// reaches: a claim's second half when is_turn_begin_ is false (FA +2, Tax
// +3, Exchange draws two, Steal takes), and the Pass recursion (coup.cc:628)
// completing whatever the opponent did last.  Returns false where the
// reference raises: SPIEL_CHECK_GE on coins (coup.cc:549, 568, 590),
// LoseCard of a missing or face-up slot (:608), a Challenge of nothing
// challengeable (:692, 770), an ExchangeReturn without 4 cards (:787-796,
// or vector::erase past the end), any other id (:806), and the Pass that
// answers a Pass (:628 recurses without end).
__device__ __forceinline__ bool ref_decision_core(Lane& L, uint32_t a) {
  const uint32_t M = L.M, O = M ^ 1u;
  const uint32_t cc = COUP_PGET(L, c, M), oc = COUP_PGET(L, c, O);
  L.r0 = 0;  // coup.cc:527
  if (a == kChallenge) {
    // coup.cc:635-771: a Block of the mover's FA / Assassinate / Steal, or
    // the opponent's Tax / Exchange / Assassinate / Steal; else fatal
    const uint32_t ol = COUP_PGET(L, l, O), cl = COUP_PGET(L, l, M);
    const bool ok = ol == kBlock ? (cl == kForeignAid || cl == kAssassinate || cl == kSteal)
                                 : (ol == kTax || ol == kExchange || ol == kAssassinate || ol == kSteal);
    if (!ok) return false;
    apply_challenge(L);
    return L.err == 0u;
  }
  if (a >= kExchangeReturn12 && a <= kExchangeReturn34) {
    if (hand_size(COUP_PGET(L, h, M)) != 4u) return false;
    apply_decision_v1(L, a);  // coup.cc:773-804
    return true;
  }
  const bool begin = L.begin != 0u;
  switch (a) {
    case kIncome:  // coup.cc:531-534
      COUP_PSET(L, l, M, a);
      COUP_PSET(L, c, M, cc + 1u);
      next_turn(L);
      return true;
    case kForeignAid:  // coup.cc:536-546
    case kTax:         // coup.cc:555-565
      if (begin) {
        COUP_PSET(L, l, M, a);
        next_move(L);
      } else {
        COUP_PSET(L, c, M, cc + (a == kTax ? 3u : 2u));
        next_turn(L);
      }
      return true;
    case kCoup:         // coup.cc:548-553
    case kAssassinate:  // coup.cc:567-573
      if (cc < (a == kCoup ? 7u : 3u)) return false;
      COUP_PSET(L, l, M, a);
      COUP_PSET(L, c, M, cc - (a == kCoup ? 7u : 3u));
      next_move(L);
      return true;
    case kExchange:  // coup.cc:575-587
      if (begin) {
        COUP_PSET(L, l, M, a);
        next_move(L);
      } else {
        queue_push(L, M);
        queue_push(L, M);
      }
      return true;
    case kSteal:  // coup.cc:589-603
      if (oc < 1u) return false;
      if (begin) {
        COUP_PSET(L, l, M, a);
        next_move(L);
      } else {
        const uint32_t k = oc > 1u ? 2u : 1u;
        COUP_PSET(L, c, M, cc + k);
        COUP_PSET(L, c, O, oc - k);
        next_turn(L);
      }
      return true;
    case kLoseCard1:
    case kLoseCard2: {  // coup.cc:605-616
      const uint32_t slot = a - kLoseCard1, h = COUP_PGET(L, h, M);
      if (slot >= hand_size(h) || (nib(h, slot) & 1u)) return false;
      apply_decision_v1(L, a);
      return true;
    }
    case kBlock:  // coup.cc:631-633
      COUP_PSET(L, l, M, a);
      next_move(L);
      return true;
    default:
      return false;  // coup.cc:805-806 (Pass is ref_decision's)
  }
}

__device__ __forceinline__ bool ref_decision(Lane& L, uint32_t a) {
  if (a != kPass) return ref_decision_core(L, a);
  // coup.cc:618-629
  const uint32_t M = L.M, O = M ^ 1u;
  const uint32_t pending = COUP_PGET(L, l, O);
  L.r0 = 0;
  COUP_PSET(L, l, M, kPass);
  if (pending == kBlock) {
    next_turn(L);
    return true;
  }
  if (pending == kPass) return false;  // the recursion never ends
  next_move(L);
  return ref_decision_core(L, pending);  // DoApplyAction(op.last) for the opponent
}

// nibbles ascending (the empties, 0xF, on top): the order SortCards keeps
__device__ __forceinline__ bool hand_sorted(uint32_t h) {
  return nib(h, 0) <= nib(h, 1) && nib(h, 1) <= nib(h, 2) && nib(h, 2) <= nib(h, 3);
}

// The record's field widths: coins 0..15, at most 4
// queued deals, at most 4 cards per hand counting the deals queued for it,
// cur_rewards_[0] in -2..5, hands sorted.  Legal play stays inside them.  A
// hand is left unsorted only by the double flip of a lost assassination
// challenge (coup.cc:660-669, 733-742, no SortCards) on a hand of 3 or 4
// cards, which unchecked play alone produces.
__device__ __forceinline__ bool representable(const Lane& L) {
  if (L.c0 > 15u || L.c1 > 15u || L.qlen > 4u || L.r0 < -2 || L.r0 > 5) return false;
  if (!hand_sorted(L.h0) || !hand_sorted(L.h1)) return false;
  const uint32_t to1 = (uint32_t)__popc(L.qids & ((1u << L.qlen) - 1u)), to0 = L.qlen - to1;
  return hand_size(L.h0) + to0 <= 4u && hand_size(L.h1) + to1 <= 4u;
}

// pyspiel's apply_action on a lane: chance outcomes as apply_action (the
// chance branch checks them, coup.cc:492-495); a decision through
// ref_decision.  Returns false, the lane untouched, where the reference
// raises, on a terminal state (the reference would go on applying decisions
// to a finished game), and where the result leaves the record's fields
// (valid in the reference, e.g. a 16th coin).
template <class H>
__device__ __forceinline__ bool apply_action_unchecked(Lane& L, uint32_t a, H& hist) {
  if (a > 17u || is_terminal(L) || L.err) return false;
  if (is_chance(L)) return apply_action(L, a, hist);
  Lane R = L;
  if (!ref_decision(R, a) || !representable(R)) return false;
  hist.record(L.move, hist_decision(a, L.M));
  R.move += 1u;
  L = R;
  return true;
}

// --------------------------------------------------- sampling contract

// Philox4x32-10 (Salmon et al., SC'11), Random123 constants.
// Each 32x32 -> 64-bit product is one v_mad_u64_u32 (both halves at once)
// instead of a v_mul_lo_u32 + v_mul_hi_u32 pair: half the quarter-rate
// multiplies of the round.
#ifndef COUP_PHILOX_HOOK
#define COUP_PHILOX_HOOK()  // measurement builds count evaluations (COUP_COUNT_PHILOX)
#endif
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint32_t k0, uint32_t k1) {
  COUP_PHILOX_HOOK();
#pragma unroll
#ifndef COUP_ABLATE_PHILOX_ROUNDS
#define COUP_ABLATE_PHILOX_ROUNDS 10  // measurement builds may time fewer rounds (wrong streams)
#endif
  for (int r = 0; r < COUP_ABLATE_PHILOX_ROUNDS; ++r) {
#ifdef COUP_ABLATE_PHILOX_FULLRATE
    // measurement builds only (wrong streams, lanes still decorrelated): the
    // products from full-rate 24-bit multiplies, pricing the 64-bit ones
    const uint64_t p0 = ((uint64_t)__umulhi((c.x & 0xFFFFFFu) << 8, 0xD2511Fu << 8) << 32) | __umul24(c.x, 0x511F53u);
    const uint64_t p1 = ((uint64_t)__umulhi((c.z & 0xFFFFFFu) << 8, 0xCD9E8Du << 8) << 32) | __umul24(c.z, 0x9E8D57u);
#else
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
#endif
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// One 32-bit draw per history slot `idx` of episode `ep` of env `env_id`:
// key = (env_id, seed lo), counter = (idx / 4, ep, seed hi, 'Coup'),
// word idx % 4.  The Rng keeps the last Philox block so consecutive slots
// of one block cost one evaluation.
struct Rng {
  uint32_t seed_lo, seed_hi, env_id;
  uint32_t blk_tag;  // (episode << 5 | block) + 1 of the cached block, 0 = none
  uint4 blk;

  __device__ __forceinline__ uint32_t draw(uint32_t ep, uint32_t idx) {
    const uint32_t tag = ((ep << 5) | (idx >> 2)) + 1u;
    if (tag != blk_tag) {
      blk = philox4x32_10(make_uint4(idx >> 2, ep, seed_hi, 0x436F7570u), env_id, seed_lo);
      blk_tag = tag;
    }
#ifdef COUP_RNG_SELECT_CHAIN
    // measurement builds: rounds 1-5's equality chain
    const uint32_t j = idx & 3u;
    return j == 0 ? blk.x : (j == 1 ? blk.y : (j == 2 ? blk.z : blk.w));
#else
    // two levels of selects on the word index's bits: the equality chain can
    // be folded into a variable extractelement, which the backend lowers
    // through scratch memory (an indexed private load)
    const bool odd = (idx & 1u) != 0u;
    const uint32_t lo = odd ? blk.y : blk.x, hi = odd ? blk.w : blk.z;
    return (idx & 2u) ? hi : lo;
#endif
  }
};

// The same draws with the Philox blocks one env step can need computed
// ahead, outside the rules' branches (step kernels of the rules-bound
// configurations): the lane's current block and the next one (the decision
// at slot move_number_ and up to three deals after it, so slots m..m+3, span
// at most these two) and block 0 of the next episode (an auto-reset's four
// deals).  Any other draw -- a state off that pattern -- computes its block
// as Rng does, so every draw equals Rng::draw.
struct PrefRng {
  uint32_t seed_lo, seed_hi, env_id;
  uint32_t ep, b;  // c0 = block (ep, b), c1 = (ep, b + 1), r0 = ((ep + 1) & kEpisodeMask, 0)
  uint4 c0, c1, r0;

  __device__ __forceinline__ static uint4 block(uint32_t seed_lo, uint32_t seed_hi, uint32_t env_id, uint32_t ep,
                                                uint32_t b) {
    return philox4x32_10(make_uint4(b, ep, seed_hi, 0x436F7570u), env_id, seed_lo);
  }

  __device__ __forceinline__ static uint32_t word(uint4 v, uint32_t j) {
    return j == 0 ? v.x : (j == 1 ? v.y : (j == 2 ? v.z : v.w));
  }

  // Word by word, never a select between the blocks themselves: a select of
  // whole uint4 members became a select of their addresses, which put the
  // struct in memory (promoted to 20 KB of LDS per block) and made the c2
  // step 3x slower.
  __device__ __forceinline__ uint32_t draw(uint32_t e, uint32_t idx) {
    const uint32_t bb = idx >> 2, j = idx & 3u;
    const bool h0 = e == ep && bb == b, h1 = e == ep && bb == b + 1u;
    const bool h2 = e == ((ep + 1u) & kEpisodeMask) && bb == 0u;
    const uint32_t w0 = word(c0, j), w1 = word(c1, j), w2 = word(r0, j);
    uint32_t u = h0 ? w0 : (h1 ? w1 : w2);
    if (!(h0 || h1 || h2)) u = word(block(seed_lo, seed_hi, env_id, e, bb), j);
    return u;
  }
};

// Chance draw: r = floor(u * sum(deck) / 2^32), first type whose cumulative
// count exceeds r.
__device__ __forceinline__ uint32_t sample_card(uint32_t deck, uint32_t u) {
  uint32_t total = 0;
#pragma unroll
  for (uint32_t t = 0; t < 5; ++t) total += deck_count(deck, t);
  const uint32_t r = __umulhi(u, total);
  // r < total, so if no type below the Duke qualifies the Duke does
  uint32_t cum = 0, pick = 4u;
#pragma unroll
  for (uint32_t t = 0; t < 4; ++t) {
    cum += deck_count(deck, t);
    pick = (pick == 4u && cum > r) ? t : pick;
  }
  return pick;
}

// Policy draw: idx = floor(u * popc(mask) / 2^32); the idx-th set bit of the
// ascending mask (== LegalActions()[idx], coup.cc:824-938).  A loop of idx
// iterations: the regrouped kernels' waves hold lanes with similar masks
// and draws, so the loop is short and uniform there.
__device__ __forceinline__ uint32_t sample_action(uint32_t mask, uint32_t u) {
  const uint32_t idx = __umulhi(u, (uint32_t)__popc(mask));
  for (uint32_t i = 0; i < idx; ++i) mask &= mask - 1u;
  return (uint32_t)__builtin_ctz(mask);
}

// The same draw without a loop: five halvings of the bit window.  For the
// in-place rules-bound kernels, whose waves mix every idx (c2r 3.22 -> 3.04
// us per step; the regrouped c4 / c4r lose 0.2 us with it,
// profiles/r02/ab/select_bits.log).
__device__ __forceinline__ uint32_t sample_action_select(uint32_t mask, uint32_t u) {
  uint32_t idx = __umulhi(u, (uint32_t)__popc(mask)), pos = 0u;
#pragma unroll
  for (uint32_t w = 16u; w >= 1u; w >>= 1) {
    const uint32_t c = (uint32_t)__popc(mask & ((1u << w) - 1u));
    const bool up = idx >= c;
    idx -= up ? c : 0u;
    mask = up ? mask >> w : mask;
    pos += up ? w : 0u;
  }
  return pos;
}

// rl_environment._sample_external_events (rl_environment.py:369-382):
// deal until a decision node or a terminal state.
// A deal adds a face-down card, so a player alive before it is alive after
// it: once the state is not terminal, only truncation (move_number_ > 90,
// coup.cc:989-992) can end the deals early.
template <class R, class H>
__device__ __forceinline__ void resolve_chance(Lane& L, R& rng, H& hist) {
  if (L.qlen == 0u || is_terminal(L)) return;
  do {
    const uint32_t u = rng.draw(L.episode, L.move);
    const uint32_t t = sample_card(L.deck, u);
    hist.record(L.move, hist_deal(t, L.qids & 1u));
    apply_deal(L, t);
    L.move += 1u;
  } while (L.qlen != 0u && L.move <= kMaxGameLength);
}

__device__ __forceinline__ void resolve_chance(Lane& L, Rng& rng) {
  NoHistory none;
  resolve_chance(L, rng, none);
}

// CoupState::CoupState (coup.cc:393-428) followed by its four chance deals
// (coup.cc:491-520, rl_environment.py:369-382): initial_lane + resolve_chance
// in straight-line form.  The queue is [P1, P2, P1, P2], deal k draws slot k
// of the episode from the full deck minus the earlier deals, and each hand
// ends as its two face-down kinds in ascending order.  Every wave with a
// finishing lane runs this on an auto-reset step.
template <class R, class H>
__device__ __forceinline__ Lane new_episode(uint32_t episode, R& rng, H& hist) {
  Lane L = initial_lane(episode);
  L.err = L.episode == 0u ? 1u : 0u;  // the counter wrapped: this stream repeats episode 0's
  uint32_t t[4];
#pragma unroll
  for (uint32_t k = 0; k < 4u; ++k) {
    t[k] = sample_card(L.deck, rng.draw(L.episode, k));
    L.deck -= 1u << (4u * t[k]);
    hist.record(k, hist_deal(t[k], k & 1u));
  }
  const uint32_t p0 = t[0] < t[2] ? t[0] : t[2], q0 = t[0] < t[2] ? t[2] : t[0];
  const uint32_t p1 = t[1] < t[3] ? t[1] : t[3], q1 = t[1] < t[3] ? t[3] : t[1];
  L.h0 = (2u * p0) | ((2u * q0) << 4) | 0xFF00u;
  L.h1 = (2u * p1) | ((2u * q1) << 4) | 0xFF00u;
  L.qlen = 0u;
  L.qids = 0u;
  L.move = 4u;
  return L;
}

}  // namespace coup
