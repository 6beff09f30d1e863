// coup_host.cpp -- the per-game State ops on the host, from the same rules
// (coup_lane.h) and tensor decoders (coup_tensor.h) the kernels run, built
// with g++ and linked into libcoup_mi355x.so (open_spiel_coup_amd/build.py).
//
// Why on the host: a single State op is ~0.1 us of integer code, while any
// device round trip is one PCIe crossing each way (7.2 us for the resident
// op-server wave).  The reference runs these ops in
// C++ behind pybind (spiel.cc:322-331, pyspiel.cc:263-345); unchanged
// callers -- MCCFR's per-node apply_action / information_state_string /
// legal_actions (outcome_sampling_mccfr.py:81-87), Deep CFR's state.child
// (deep_cfr.py:440-444) -- need that per-op cost, not a batch.  Batched work
// (the env step, trajectories, SyncVectorEnv, batched children with device
// tensors) stays on the GPU.  These functions exist only inside the HIP
// library: there is no build of the product without it.
//
// A host state is a coup_slot_result (include/coup_mi355x.h): the packed
// record, the 96 history bytes and the answers (legal mask, player, ...)
// that the device ops return, so host and device states convert freely.
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <string>

#include "coup_tensor.h"

using namespace coup;

namespace {

void fill_result(const Lane& L, const uint8_t* hist, uint32_t ok, uint32_t unrep, coup_slot_result* out) {
  const uint4 w = pack(L);
  out->record[0] = w.x;
  out->record[1] = w.y;
  out->record[2] = w.z;
  out->record[3] = w.w;
  if (hist != out->history) std::memcpy(out->history, hist, sizeof(out->history));
  out->legal_mask = legal_mask(L);
  out->cur_player = (int8_t)current_player(L);
  out->terminal = is_terminal(L) ? 1 : 0;
  out->ok = (uint8_t)ok;
  out->unrepresentable = (uint8_t)unrep;
  out->rewards[0] = (int8_t)L.r0;
  out->rewards[1] = (int8_t)(-L.r0);
  const int32_t r0 = return0(L);
  out->returns[0] = (int8_t)r0;
  out->returns[1] = (int8_t)(-r0);
  std::memset(out->pad, 0, sizeof(out->pad));
}

uint4 record_of(const coup_slot_result* st) {
  return make_uint4(st->record[0], st->record[1], st->record[2], st->record[3]);
}

}  // namespace

extern "C" {

// NewInitialState (coup.cc:393-428): episode 0, empty history.
int coup_host_state_init(coup_slot_result* out) {
  if (!out) return COUP_E_INVALID;
  uint8_t hist[kHistoryBytes];
  std::memset(hist, 0xFF, sizeof(hist));
  fill_result(initial_lane(0u), hist, 1u, 0u, out);
  return COUP_OK;
}

// State::ApplyAction on host state `in` into `out` (in == out allowed):
// with COUP_SLOT_UNCHECKED as pyspiel's apply_action (no legality check,
// DoApplyAction's own checks: apply_action_unchecked), else with the
// legality check (apply_action).  Exactly the device slot_transition: a
// rejected action leaves the record and history unchanged with ok = 0 (and
// unrepresentable = 1 where the reference accepts it but the result leaves
// the packed record's fields); an accepted one records its history entry at
// index move_number_.  Ids 18..127 are rejected actions (ok = 0), as
// coup_host_state_step and the device lane op report them (DoApplyAction
// raises: coup.cc:493, :806); negative ids and ids past int8 are invalid
// arguments (the two host entry points disagreed).
int coup_host_state_apply(const coup_slot_result* in, int action, int flags, coup_slot_result* out) {
  if (!in || !out) return COUP_E_INVALID;
  if (action < 0 || action > 127) return COUP_E_INVALID;
  const uint32_t x = (uint32_t)action;
  uint8_t hist[kHistoryBytes];
  std::memcpy(hist, in->history, sizeof(hist));
  const uint4 w = record_of(in);
  Lane L = unpack(w);
  const uint32_t idx = L.move;
  const uint32_t entry = is_chance(L) ? hist_deal(x, L.qids & 1u) : hist_decision(x, L.M);
  NoHistory none;
  Lane R = L;
  bool ok;
  uint32_t unrep = 0u;
  if (flags & COUP_SLOT_UNCHECKED) {
    ok = apply_action_unchecked(R, x, none);
    if (!ok && x < (uint32_t)COUP_NUM_ACTIONS && !is_terminal(L) && !L.err && !is_chance(L)) {
      Lane T = L;
      unrep = (ref_decision(T, x) && !representable(T)) ? 1u : 0u;
    }
  } else {
    const uint32_t err_before = R.err;
    ok = apply_action(R, x, none) && !(R.err && !err_before);
  }
  if (!ok) {
    fill_result(L, hist, 0u, unrep, out);
    return COUP_OK;
  }
  if (idx < kHistoryBytes) hist[idx] = (uint8_t)entry;
  fill_result(R, hist, 1u, 0u, out);
  return COUP_OK;
}

// rl_environment's ops on a host state (the device's COUP_SLOT_RESET /
// COUP_SLOT_DEAL lane ops, slot_step in coup_kernels.hip, on the host):
//   mode COUP_SLOT_INIT  -- start from the lane coup_create leaves (episode 0,
//                           NewInitialState, empty history; `in` may be null)
//   mode COUP_SLOT_RESET -- the lane's next episode (episode + 1, NewInitialState)
//   action >= 0          -- State::ApplyAction (COUP_SLOT_UNCHECKED: as pyspiel's)
//   mode COUP_SLOT_DEAL  -- then the pending chance deals under the sampling
//                           contract of stream (seed, env_id),
//                           as rl_environment samples chance (rl_environment.py:369-382)
// every entry to the history bytes.  A rejected action leaves `in` as it was
// (the reset included) with ok = 0.  Same draws as the device, so the same
// games as the env's device lane would play.
int coup_host_state_step(const coup_slot_result* in, int action, int mode, uint64_t seed, uint32_t env_id,
                         coup_slot_result* out) {
  if (!out || (!in && !(mode & COUP_SLOT_INIT))) return COUP_E_INVALID;
  // 18..127: a rejected action (ok = 0, state unchanged), as the device lane
  // op reports it (DoApplyAction raises: coup.cc:493, :806); past an int8 id
  // the argument itself is invalid
  if (action > 127) return COUP_E_INVALID;
  uint8_t hist[kHistoryBytes];
  Lane L;
  if (mode & COUP_SLOT_INIT) {
    std::memset(hist, 0xFF, sizeof(hist));
    L = initial_lane(0u);
  } else {
    std::memcpy(hist, in->history, sizeof(hist));
    L = unpack(record_of(in));
  }
  struct Bytes {
    uint8_t* b;
    void record(uint32_t idx, uint32_t entry) {
      if (idx < kHistoryBytes) b[idx] = (uint8_t)entry;
    }
  } rec{hist};
  if (mode & COUP_SLOT_RESET) {
    L = initial_lane(L.episode + 1u);
    L.err = L.episode == 0u ? 1u : 0u;  // the episode counter wrapped (coup_lane.h kEpisodeMask)
  }
  if (action >= 0) {
    const uint32_t x = (uint32_t)action;
    const uint32_t idx = L.move;
    const uint32_t entry = is_chance(L) ? hist_deal(x, L.qids & 1u) : hist_decision(x, L.M);
    NoHistory none;
    Lane R = L;
    bool ok;
    uint32_t unrep = 0u;
    if (mode & COUP_SLOT_UNCHECKED) {
      ok = apply_action_unchecked(R, x, none);
      if (!ok && x < (uint32_t)COUP_NUM_ACTIONS && !is_terminal(L) && !L.err && !is_chance(L)) {
        Lane T = L;
        unrep = (ref_decision(T, x) && !representable(T)) ? 1u : 0u;
      }
    } else {
      const uint32_t err_before = R.err;
      ok = apply_action(R, x, none) && !(R.err && !err_before);
    }
    if (!ok) {
      if (in) {
        fill_result(unpack(record_of(in)), in->history, 0u, unrep, out);
      } else {
        std::memset(hist, 0xFF, sizeof(hist));
        fill_result(initial_lane(0u), hist, 0u, unrep, out);
      }
      return COUP_OK;
    }
    L = R;
    rec.record(idx, entry);
  }
  if (mode & COUP_SLOT_DEAL) {
    Rng rng{(uint32_t)seed, (uint32_t)(seed >> 32), env_id, 0u, make_uint4(0, 0, 0, 0)};
    resolve_chance(L, rng, rec);
  }
  fill_result(L, hist, 1u, 0u, out);
  return COUP_OK;
}

// ObservationTensor(p) of both players ([2][98], obs) and / or
// InformationStateTensor(p) of both players ([2][2492], info) of host state
// st; either pointer may be null.
int coup_host_state_tensors(const coup_slot_result* st, float* obs, float* info) {
  if (!st) return COUP_E_INVALID;
  const Lane L = unpack(record_of(st));
  if (obs) {
    const bool term = is_terminal(L);
    for (int g = 0; g < 2 * kObsSize; ++g) obs[g] = obs_pair_at(L, term, g);
  }
  if (info) {
    // info_f4's values written sparsely: the same prefix words, then zeros
    // except the prefix's set bits, the two coin counts and one entry per
    // history row the player saw (a decision, or a deal to that player)
    uint32_t pre[kPreWords];
    info_prefix_to_lds(L, pre);
    std::memset(info, 0, sizeof(float) * 2 * kInfoSize);
    const uint32_t meta = pre[4], len = std::min<uint32_t>(meta >> 16, (uint32_t)kHist);
    for (uint32_t p = 0; p < 2; ++p) {
      float* t = info + p * kInfoSize;
      const uint64_t prefix = (uint64_t)pre[2 * p] | ((uint64_t)pre[2 * p + 1] << 32);
      for (int f = 0; f < 60; ++f)
        if ((prefix >> f) & 1u) t[f] = 1.0f;
      t[60] = (float)(meta & 0xFFu);
      t[61] = (float)((meta >> 8) & 0xFFu);
      for (uint32_t r = 0; r < len; ++r) {
        const uint32_t e = st->history[r], a = e & 0x1Fu;
        const bool seen = (e & 0x20u) == 0u || ((e >> 6) & 1u) == p;  // deals: observer's only
        if (seen && a < 18u) t[62 + 18 * r + a] = 1.0f;
      }
    }
  }
  return COUP_OK;
}

// The human-readable forms (kind 0 ObservationString, 1
// InformationStateString -- CoupObserver::StringFrom, coup.cc:290-373 -- and 2
// ToString, coup.cc:945-987) of host state st for `player`, into buf (cap
// bytes, NUL-terminated when it fits).  Returns the string's length (>= cap:
// truncated, call again with more room), or -1 for a bad argument.  The
// formats are verbatim with integration_tests/playthroughs/coup.txt
// (open_spiel_coup_amd/strings.py is the same in Python; the tests hold the
// two equal).
int64_t coup_host_state_string(const coup_slot_result* st, int kind, int player, char* buf, int64_t cap) {
  static const char* const kCard[5] = {"Assassin", "Ambassador", "Captain", "Contessa", "Duke"};
  static const char* const kAction[18] = {
      "Income", "ForeignAid", "Coup", "Tax", "Assassinate", "Exchange", "Steal", "LoseCard1", "LoseCard2",
      "Pass", "Block", "Challenge", "ExchangeReturn12", "ExchangeReturn13", "ExchangeReturn14",
      "ExchangeReturn23", "ExchangeReturn24", "ExchangeReturn34"};
  static const char* const kFace[2] = {"FaceDown", "FaceUp"};
  if (!st || kind < 0 || kind > 2 || (kind < 2 && (player < 0 || player > 1)) || cap < 0 || (cap > 0 && !buf))
    return -1;
  const Lane L = unpack(record_of(st));
  const bool recall = kind == 1, all = kind == 2;
  // appended piece by piece (no printf formatting: ~10-30 calls per string)
  std::string s;
  s.reserve(1024);
  auto put = [&s](const char* t) { s.append(t); };
  auto putu = [&s](uint32_t v) {
    char d[10];
    int n = 0;
    do {
      d[n++] = (char)('0' + v % 10u);
      v /= 10u;
    } while (v);
    while (n) s.push_back(d[--n]);
  };
  if (!all) {
    put("Observer: P");
    putu((uint32_t)player + 1u);
    put("\n");
  }
  put("Turn: ");
  putu(L.turn);
  put("\nMove: P");
  putu(L.M + 1u);
  put("\n");
  for (uint32_t p = 0; p < 2; ++p) {
    const uint32_t h = p ? L.h1 : L.h0;
    put("P");
    putu(p + 1u);
    put("\n        Card         State\n");
    for (uint32_t i = 0; i < 4; ++i) {
      const uint32_t k = nib(h, i);
      if (k == 0xFu) break;
      const bool shown = all || (k & 1u) || p == (uint32_t)player;
      const char* name = shown ? kCard[k >> 1] : "-";
      put("Card ");
      putu(i + 1u);
      put(": ");
      put(name);
      const size_t w = std::strlen(name);
      if (w < 11) s.append(11 - w, ' ');  // %-11s
      put("| ");
      put(kFace[k & 1u]);
      put("\n");
    }
    put("Coins: ");
    putu(p ? L.c1 : L.c0);
    put("\n");
    if (recall) {
      put("\n");
    } else {
      const uint32_t la = p ? L.l1 : L.l0;
      put("Last Action: ");
      put(la == kNoAction ? "None" : kAction[la]);
      put("\n\n");
    }
  }
  if (recall || all) {
    // coup.cc:351-371 (recall): a deal is shown to its receiver only, but the
    // ", " after it depends on its position in the full history
    put("Action Sequence: ");
    const uint32_t n = L.move < kHistoryBytes ? L.move : kHistoryBytes;
    bool first = true;
    for (uint32_t i = 0; i < n; ++i) {
      const uint32_t e = st->history[i];
      const bool deal = (e & 0x20u) != 0u;
      const uint32_t who = (e >> 6) & 1u, a = e & 0x1Fu;
      if (all) {
        if (!first) put(", ");
        first = false;
      }
      if (deal) {
        if (all || who == (uint32_t)player) {
          put("PC-");
          put(kCard[a < 5u ? a : 0u]);
          if (!all && i + 1 < n) put(", ");
        }
      } else {
        put("P");
        putu(who + 1u);
        put("-");
        put(kAction[a < 18u ? a : 0u]);
        if (!all && i + 1 < n) put(", ");
      }
    }
    put("\n");
  }
  const int64_t len = (int64_t)s.size();
  if (cap > 0) {
    const int64_t m = len < cap ? len : cap - 1;
    std::memcpy(buf, s.data(), (size_t)m);
    buf[m] = '\0';
  }
  return len;
}

}  // extern "C"
