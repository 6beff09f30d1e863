/*
 * coup_mi355x.hpp -- C++ host layer over the C ABI (coup_mi355x.h).
 *
 * Header-only, C++17.  Two surfaces:
 *
 *   coup_amd::BatchedEnv     RAII owner of a coup_env: the batched
 *                            reset / step / rollout / State-API calls on
 *                            caller-owned device buffers.
 *   coup_amd::CoupGame,      the open_spiel::Game / open_spiel::State
 *   coup_amd::CoupState      methods the reference's C++ and Python callers
 *                            use (spiel.h:210-1035, coup.h:111-231), one
 *                            game per object.
 *
 * Every live CoupState owns one lane of a device-resident lane pool
 * (detail::Pool: 2-player history envs of 4096 lanes, grown on demand, slots
 * reused).  Each rules operation (ApplyAction, the tensors, ...) is one
 * coup_slot_op launch on that lane, and the 128-byte coup_slot_result it
 * returns (record, history, legal mask, player, rewards, returns) answers
 * the accessors until the next op; a Clone is a device-side lane copy.
 * There is no CPU rules engine.  The pool is guarded by a mutex, so States
 * may be used from several threads.  Strings are formatted on the host from the record and the
 * history (coup.cc:60-135, 290-373, 945-987), as open_spiel_coup_amd/strings.py
 * does.  Errors throw coup_amd::SpielError (SpielFatalError,
 * spiel_utils.cc:132-136; pyspiel.SpielError).
 *
 * Link with libcoup_mi355x.so and libamdhip64.so.  Needs <hip/hip_runtime_api.h>
 * (define __HIP_PLATFORM_AMD__ when compiling with g++).
 */
#ifndef COUP_MI355X_HPP_
#define COUP_MI355X_HPP_

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <array>
#include <cstdint>
#include <cstring>
#include <memory>
#include <cstdlib>
#include <mutex>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "coup_mi355x.h"

namespace coup_amd {

using Action = int64_t;
using Player = int;
constexpr Player kChancePlayerId = COUP_CHANCE_PLAYER;      // spiel_globals.h:34
constexpr Player kTerminalPlayerId = COUP_TERMINAL_PLAYER;  // spiel_globals.h:28

class SpielError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

// An action the reference's DoApplyAction ACCEPTS whose result leaves the
// packed record's fields (coup_slot_result.unrepresentable; a 16th coin, an
// unsorted 3-4 card hand): a known parity gap, not a
// reference raise.  The state is left unchanged.
class UnrepresentableActionError : public SpielError {
 public:
  using SpielError::SpielError;
};

namespace detail {
[[noreturn]] inline void ThrowRejected(const std::string& op, int64_t a, const coup_slot_result& r) {
  if (r.unrepresentable)
    throw UnrepresentableActionError(op + "(" + std::to_string(a) +
                                     "): the reference accepts it, but the result leaves the packed record's fields");
  throw SpielError(op + "(" + std::to_string(a) + "): DoApplyAction raises here");
}
}  // namespace detail

inline void Check(int rc, const char* what) {
  if (rc != COUP_OK) throw SpielError(std::string(what) + ": " + coup_last_error());
}

inline void CheckHip(hipError_t e, const char* what) {
  if (e != hipSuccess) throw SpielError(std::string(what) + ": " + hipGetErrorString(e));
}

// ------------------------------------------------------------ BatchedEnv

class BatchedEnv {
 public:
  BatchedEnv(int64_t batch, uint64_t seed, uint32_t env_id_base = 0, int flags = COUP_FLAG_AUTO_RESET,
             int num_players = COUP_NUM_PLAYERS) {
    Check(coup_create_ex(batch, seed, env_id_base, flags, num_players, &env_), "coup_create_ex");
  }
  ~BatchedEnv() {
    if (env_) coup_destroy(env_);
  }
  BatchedEnv(const BatchedEnv&) = delete;
  BatchedEnv& operator=(const BatchedEnv&) = delete;
  BatchedEnv(BatchedEnv&& o) noexcept : env_(o.env_) { o.env_ = nullptr; }

  coup_env* get() const { return env_; }
  int64_t batch() const { return coup_batch(env_); }
  int num_players() const { return coup_num_players(env_); }
  int state_bytes() const { return coup_state_bytes(env_); }
  void SetStream(hipStream_t s) { Check(coup_set_stream(env_, (void*)s), "coup_set_stream"); }

  // all pointers are device pointers (lane-major); see coup_mi355x.h
  void Reset(const uint8_t* lane_mask = nullptr) { Check(coup_reset(env_, lane_mask), "coup_reset"); }
  void Step(const int8_t* actions, const coup_step_outputs& out) {
    Check(coup_step(env_, actions, &out), "coup_step");
  }
  // one step whose outputs land in host memory (coup_step_host): host
  // actions (or null), COUP_HOST_* flags, host_out laid out as
  // coup_step_host_layout describes
  void StepHost(const int8_t* host_actions, int want, void* host_out) {
    Check(coup_step_host(env_, host_actions, want, host_out), "coup_step_host");
  }
  // `steps` uniform steps in one launch, step t's outputs in slice t of
  // out's [steps][B] buffers (coup_step_trajectory; no obs / info_state)
  void StepTrajectory(int64_t steps, const coup_step_outputs& out) {
    Check(coup_step_trajectory(env_, steps, &out), "coup_step_trajectory");
  }
  void Rollout(int64_t steps, const coup_rollout_stats* stats = nullptr) {
    Check(coup_rollout(env_, steps, stats), "coup_rollout");
  }
  void NewInitialState(const uint8_t* lane_mask = nullptr) {
    Check(coup_new_initial_state(env_, lane_mask), "coup_new_initial_state");
  }
  void ApplyAction(const int8_t* actions) { Check(coup_apply_action(env_, actions), "coup_apply_action"); }
  void Query(const coup_query_outputs& out) { Check(coup_query(env_, &out), "coup_query"); }
  void ExportState(uint32_t* dst) { Check(coup_export_state(env_, dst), "coup_export_state"); }
  void ImportState(const uint32_t* src) { Check(coup_import_state(env_, src), "coup_import_state"); }
  void ExportHistory(uint8_t* dst) { Check(coup_export_history(env_, dst), "coup_export_history"); }
  void ImportHistory(const uint8_t* src) { Check(coup_import_history(env_, src), "coup_import_history"); }
  int64_t ErrorCount() {
    int64_t n = 0;
    Check(coup_error_count(env_, &n), "coup_error_count");
    return n;
  }

 private:
  coup_env* env_ = nullptr;
};

// --------------------------------------------------------------- strings

namespace detail {

inline const char* CardName(int t) {
  static const char* k[] = {"Assassin", "Ambassador", "Captain", "Contessa", "Duke"};
  return k[t];
}

inline const char* ActionName(int a) {
  static const char* k[] = {"Income",           "ForeignAid",       "Coup",      "Tax",
                            "Assassinate",      "Exchange",         "Steal",     "LoseCard1",
                            "LoseCard2",        "Pass",             "Block",     "Challenge",
                            "ExchangeReturn12", "ExchangeReturn13", "ExchangeReturn14",
                            "ExchangeReturn23", "ExchangeReturn24", "ExchangeReturn34"};
  return k[a];
}

// fields of the 16-byte record
struct Fields {
  std::array<std::vector<std::pair<int, int>>, 2> cards;  // (type, face) per slot
  std::array<int, 5> deck;
  std::array<int, 2> coins, last;  // last: -1 = None
  int move_player, move_number, turn_number;
};

inline Fields Decode(const std::array<uint32_t, 4>& w) {
  Fields f;
  for (int p = 0; p < 2; ++p) {
    const uint32_t h = (w[0] >> (16 * p)) & 0xFFFFu;
    for (int i = 0; i < 4; ++i) {
      const uint32_t k = (h >> (4 * i)) & 0xFu;
      if (k == 0xFu) break;
      f.cards[p].emplace_back((int)(k >> 1), (int)(k & 1u));
    }
    f.coins[p] = (int)((w[1] >> (20 + 4 * p)) & 0xFu);
    const int l = (int)((w[2] >> (5 * p)) & 0x1Fu);
    f.last[p] = l == 31 ? -1 : l;
  }
  for (int t = 0; t < 5; ++t) f.deck[t] = (int)((w[1] >> (4 * t)) & 0xFu);
  f.move_player = (int)((w[2] >> 20) & 1u);
  f.move_number = (int)((w[2] >> 22) & 0x7Fu);
  f.turn_number = (int)(w[3] & 0x7Fu);
  return f;
}

inline std::string CardRow(int slot, const std::string& value, int face) {
  std::string v = value;
  if (v.size() < 11) v.append(11 - v.size(), ' ');
  return "Card " + std::to_string(slot + 1) + ": " + v + "| " + (face ? "FaceUp" : "FaceDown") + "\n";
}

inline std::string LastAction(int a) { return a < 0 ? "None" : ActionName(a); }

// CoupObserver::StringFrom (coup.cc:290-373); observer < 0 = ToString
// (coup.cc:945-987, every card shown)
inline std::string StateString(const Fields& f, const uint8_t* hist, int observer, bool perfect_recall) {
  std::string s;
  if (observer >= 0) s += "Observer: P" + std::to_string(observer + 1) + "\n";
  s += "Turn: " + std::to_string(f.turn_number) + "\n";
  s += "Move: P" + std::to_string(f.move_player + 1) + "\n";
  for (int p = 0; p < 2; ++p) {
    s += "P" + std::to_string(p + 1) + "\n        Card         State\n";
    for (size_t i = 0; i < f.cards[p].size(); ++i) {
      const auto& c = f.cards[p][i];
      const bool shown = observer < 0 || c.second == 1 || p == observer;
      s += CardRow((int)i, shown ? CardName(c.first) : "-", c.second);
    }
    s += "Coins: " + std::to_string(f.coins[p]) + "\n";
    if (perfect_recall)
      s += "\n";
    else
      s += "Last Action: " + LastAction(f.last[p]) + "\n\n";
  }
  if (observer < 0 || perfect_recall) {
    s += "Action Sequence: ";
    const int n = f.move_number;
    for (int i = 0; i < n; ++i) {
      const uint8_t e = hist[i];
      const bool deal = (e & 0x20) != 0;
      const int a = e & 0x1F, who = (e >> 6) & 1;
      if (observer < 0) {
        s += deal ? std::string("PC-") + CardName(a) : "P" + std::to_string(who + 1) + "-" + ActionName(a);
        if (i < n - 1) s += ", ";
      } else if (!deal || who == observer) {
        // deals are shown to their receiver only; the separator depends on
        // the position in the full history (coup.cc:351-371)
        s += deal ? std::string("PC-") + CardName(a) : "P" + std::to_string(who + 1) + "-" + ActionName(a);
        if (i < n - 1) s += ", ";
      }
    }
    s += "\n";
  }
  return s;
}

// Device-resident lane pool: every live CoupState owns one lane of a
// 2-player history env (segments of kSeg lanes, grown on demand); each State
// op is one coup_slot_op on that lane -- run by the pool's device-resident
// op server (coup_server_create: one resident wave, no launch per op;
// COUP_SERVER=0 in the environment keeps one launch per op) -- and only ops
// that need an answer copy the 128-byte coup_slot_result back.
class Pool {
 public:
  static constexpr int64_t kSeg = 4096;
  struct Slot {
    int seg = -1;
    int64_t lane = 0;
  };

  Pool() {
    const char* e = std::getenv("COUP_SERVER");
    if (!(e && std::atoi(e) == 0)) {
      const char* idle = std::getenv("COUP_SERVER_IDLE_US");
      if (coup_server_create(idle ? std::atoll(idle) : 2000, &srv_) != COUP_OK) srv_ = nullptr;
    }
  }
  ~Pool() {
    // the wave leaves before the segments it serves are freed
    for (auto& env : segs_) (void)coup_attach_server(env->get(), nullptr);
    if (srv_) (void)coup_server_destroy(srv_);
  }
  Pool(const Pool&) = delete;
  Pool& operator=(const Pool&) = delete;

  Slot Alloc() {
    std::lock_guard<std::mutex> g(mu_);
    if (free_.empty()) {
      segs_.emplace_back(new BatchedEnv(kSeg, 0, 0, COUP_FLAG_HISTORY));
      if (srv_) Check(coup_attach_server(segs_.back()->get(), srv_), "coup_attach_server");
      const int k = (int)segs_.size() - 1;
      for (int64_t i = kSeg - 1; i >= 0; --i) free_.push_back({k, i});
    }
    Slot s = free_.back();
    free_.pop_back();
    return s;
  }
  void Release(const Slot& s) {
    std::lock_guard<std::mutex> g(mu_);
    if (s.seg >= 0) free_.push_back(s);
  }
  // n requests on segment `seg` in one launch (coup_slot_ops); copies read
  // segment src_seg (-1: none); host_out: n results (+ tensors per flags)
  void Ops(int seg, const std::vector<coup_slot_req>& reqs, int src_seg, int flags, void* host_out) {
    std::lock_guard<std::mutex> g(mu_);
    coup_env* src_env = src_seg >= 0 ? segs_[src_seg]->get() : nullptr;
    Check(coup_slot_ops(segs_[seg]->get(), (int64_t)reqs.size(), reqs.data(), src_env, flags, host_out),
          "coup_slot_ops");
  }
  // host_out: coup_slot_result followed by the tensors the flags ask for
  void Op(const Slot& s, const Slot* src, int action, int flags, void* host_out) {
    // one op at a time: each segment answers through one pinned scratch buffer
    std::lock_guard<std::mutex> g(mu_);
    coup_env* src_env = src ? segs_[src->seg]->get() : nullptr;
    Check(coup_slot_op(segs_[s.seg]->get(), s.lane, src_env, src ? src->lane : 0, action, flags, host_out),
          "coup_slot_op");
  }

 private:
  std::vector<std::unique_ptr<BatchedEnv>> segs_;
  std::vector<Slot> free_;
  std::mutex mu_;
  coup_server* srv_ = nullptr;
};

inline Pool& ThePool() {
  static Pool p;  // one per process (current HIP device at first use)
  return p;
}

// States are host-resident unless COUP_STATE_DEVICE=1 (read once): the
// library's host build of the lane rules (coup_host_state_*) applies each
// op on the calling thread instead of a device round trip (DESIGN.md
// section 12).  A host state has no pool slot (seg < 0).
inline bool DeviceStates() {
  static const bool v = [] {
    const char* e = std::getenv("COUP_STATE_DEVICE");
    return e && std::atoi(e) == 1;
  }();
  return v;
}

}  // namespace detail

// ---------------------------------------------------------- Game / State

class CoupGame;

struct PlayerAction {
  Player player;
  Action action;
};

// open_spiel::coup::CoupState (coup.h:111-197) on the MI355X engine: host-
// resident by default (its coup_slot_result is the state; the library's
// host rules apply each op), or on a lane of the device pool
// (COUP_STATE_DEVICE=1; every op a coup_slot_op).  Same results either way.
class CoupState {
 public:
  explicit CoupState(const CoupGame* game) : game_(game) {
    detail::Pool& pool = detail::ThePool();  // the HIP device is required either way
    if (!detail::DeviceStates()) {
      Check(coup_host_state_init(&q_), "coup_host_state_init");
      return;
    }
    slot_ = pool.Alloc();
    pool.Op(slot_, nullptr, -1, COUP_SLOT_INIT, &q_);
  }
  // State::Clone (spiel.h:822): the result copied (host), or a device-side
  // lane copy with no round trip
  CoupState(const CoupState& o) : game_(o.game_), history_(o.history_), q_(o.q_) {
    if (!o.Host()) {
      slot_ = detail::ThePool().Alloc();
      detail::ThePool().Op(slot_, &o.slot_, -1, COUP_SLOT_NO_RESULT, nullptr);
    }
  }
  CoupState& operator=(const CoupState&) = delete;
  ~CoupState() { detail::ThePool().Release(slot_); }

  Player CurrentPlayer() const { return Q().cur_player; }
  bool IsTerminal() const { return Q().terminal != 0; }
  bool IsChanceNode() const { return CurrentPlayer() == kChancePlayerId; }
  bool IsPlayerNode() const { return CurrentPlayer() >= 0; }
  int NumPlayers() const { return COUP_NUM_PLAYERS; }
  int NumDistinctActions() const { return COUP_NUM_ACTIONS; }

  // LegalActions (coup.cc:824-938): ascending; throws at a decision node no
  // legal play reaches (coup.cc:886, 892, 936), as the reference does
  std::vector<Action> LegalActions() const {
    std::vector<Action> out;
    if (IsTerminal()) return out;
    const uint32_t m = Q().legal_mask & 0x3FFFFu;
    if (m == 0u && IsPlayerNode()) throw SpielError("Error in LegalActions(): Invalid action progression");
    for (int a = 0; a < COUP_NUM_ACTIONS; ++a)
      if ((m >> a) & 1u) out.push_back(a);
    return out;
  }
  std::vector<Action> LegalActions(Player p) const {
    return p == CurrentPlayer() ? LegalActions() : std::vector<Action>();
  }
  // LegalActionsMask (spiel.cc:371-377): 5 entries at chance nodes
  std::vector<int> LegalActionsMask() const {
    std::vector<int> mask(IsChanceNode() ? COUP_NUM_CARD_TYPES : COUP_NUM_ACTIONS, 0);
    for (Action a : LegalActions()) mask[a] = 1;
    return mask;
  }
  // ChanceOutcomes (coup.cc:1062-1077)
  std::vector<std::pair<Action, double>> ChanceOutcomes() const {
    if (!IsChanceNode()) throw SpielError("ChanceOutcomes() at a non-chance node");
    const detail::Fields f = detail::Decode(Rec());
    double total = 0;
    for (int t = 0; t < 5; ++t) total += f.deck[t];
    std::vector<std::pair<Action, double>> out;
    for (int t = 0; t < 5; ++t)
      if (f.deck[t] > 0) out.emplace_back(t, f.deck[t] / total);
    return out;
  }

  // State::ApplyAction (spiel.cc:322-331): no LegalActions() check, as the
  // reference's; DoApplyAction's own checks decide (COUP_SLOT_UNCHECKED).
  // Throws, the state unchanged, where the reference throws (coup.cc:
  // 490-809), on a terminal state, or where the result leaves the packed
  // record's fields.
  void ApplyAction(Action a) {
    const Player p = CurrentPlayer();
    CheckId(a, "ApplyAction");
    coup_slot_result r;
    if (Host())
      Check(coup_host_state_apply(&q_, (int)a, COUP_SLOT_UNCHECKED, &r), "coup_host_state_apply");
    else
      detail::ThePool().Op(slot_, nullptr, (int)a, COUP_SLOT_UNCHECKED, &r);
    if (!r.ok) detail::ThrowRejected("ApplyAction", a, r);
    q_ = r;
    history_.push_back({p, a});
  }
  // State::ApplyActionWithLegalityCheck (spiel.cc:334-344)
  void ApplyActionWithLegalityCheck(Action a) {
    if (!Legal(a))
      throw SpielError("Current player " + std::to_string(CurrentPlayer()) + " calling ApplyAction with illegal action (" +
                       std::to_string(a) + ")");
    ApplyAction(a);
  }
  // Clone + ApplyAction as ONE op: the child's lane is a copy of this one
  // with `a` applied
  std::unique_ptr<CoupState> Child(Action a) const {
    const Player p = CurrentPlayer();
    CheckId(a, "Child");
    if (Host()) {
      coup_slot_result r;
      Check(coup_host_state_apply(&q_, (int)a, COUP_SLOT_UNCHECKED, &r), "coup_host_state_apply");
      if (!r.ok) detail::ThrowRejected("Child", a, r);
      std::vector<PlayerAction> h = history_;
      h.push_back({p, a});
      return std::unique_ptr<CoupState>(new CoupState(game_, detail::Pool::Slot{}, std::move(h), r));
    }
    detail::Pool& pool = detail::ThePool();
    const detail::Pool::Slot slot = pool.Alloc();
    coup_slot_result r;
    try {
      pool.Op(slot, &slot_, (int)a, COUP_SLOT_UNCHECKED, &r);
      if (!r.ok) detail::ThrowRejected("Child", a, r);
    } catch (...) {
      pool.Release(slot);
      throw;
    }
    std::vector<PlayerAction> h = history_;
    h.push_back({p, a});
    return std::unique_ptr<CoupState>(new CoupState(game_, slot, std::move(h), r));
  }
  std::unique_ptr<CoupState> Clone() const { return std::unique_ptr<CoupState>(new CoupState(*this)); }
  // Child(a) for every a in `actions`, one coup_slot_ops launch per pool
  // segment: the expansion of a Deep CFR traverser node (deep_cfr.py:440-471)
  std::vector<std::unique_ptr<CoupState>> Children(const std::vector<Action>& actions) const {
    const Player p = CurrentPlayer();
    const int32_t rf = COUP_SLOT_UNCHECKED;
    for (Action a : actions) CheckId(a, "Children");
    if (Host()) {
      std::vector<std::unique_ptr<CoupState>> out;
      for (Action a : actions) {
        coup_slot_result r;
        Check(coup_host_state_apply(&q_, (int)a, COUP_SLOT_UNCHECKED, &r), "coup_host_state_apply");
        if (!r.ok) detail::ThrowRejected("Children", a, r);
        std::vector<PlayerAction> h = history_;
        h.push_back({p, a});
        out.emplace_back(new CoupState(game_, detail::Pool::Slot{}, std::move(h), r));
      }
      return out;
    }
    detail::Pool& pool = detail::ThePool();
    std::vector<detail::Pool::Slot> slots;
    for (size_t k = 0; k < actions.size(); ++k) slots.push_back(pool.Alloc());
    std::vector<coup_slot_result> res(actions.size());
    try {
      std::vector<size_t> done;
      for (size_t k = 0; k < slots.size(); ++k) {  // group the requests by destination segment
        if (std::find(done.begin(), done.end(), k) != done.end()) continue;
        std::vector<coup_slot_req> reqs;
        std::vector<size_t> ks;
        for (size_t j = k; j < slots.size(); ++j)
          if (slots[j].seg == slots[k].seg) {
            reqs.push_back({slots[j].lane, slot_.lane, (int32_t)actions[j], rf});
            ks.push_back(j);
            done.push_back(j);
          }
        std::vector<coup_slot_result> part(reqs.size());
        pool.Ops(slots[k].seg, reqs, slot_.seg, 0, part.data());
        for (size_t j = 0; j < ks.size(); ++j) {
          if (!part[j].ok) detail::ThrowRejected("Children", actions[ks[j]], part[j]);
          res[ks[j]] = part[j];
        }
      }
    } catch (...) {
      for (const auto& s : slots) pool.Release(s);
      throw;
    }
    std::vector<std::unique_ptr<CoupState>> out;
    for (size_t k = 0; k < actions.size(); ++k) {
      std::vector<PlayerAction> h = history_;
      h.push_back({p, actions[k]});
      out.emplace_back(new CoupState(game_, slots[k], std::move(h), res[k]));
    }
    return out;
  }

  std::vector<double> Rewards() const { return {(double)Q().rewards[0], (double)Q().rewards[1]}; }
  std::vector<double> Returns() const { return {(double)Q().returns[0], (double)Q().returns[1]}; }
  double PlayerReturn(Player p) const { return Returns()[p]; }

  std::vector<float> ObservationTensor(Player p) const {
    if (Host()) {
      std::vector<float> both(2 * COUP_OBS_SIZE);
      Check(coup_host_state_tensors(&q_, both.data(), nullptr), "coup_host_state_tensors");
      return std::vector<float>(both.begin() + p * COUP_OBS_SIZE, both.begin() + (p + 1) * COUP_OBS_SIZE);
    }
    std::vector<uint8_t> buf(sizeof(coup_slot_result) + 2 * COUP_OBS_SIZE * 4);
    detail::ThePool().Op(slot_, nullptr, -1, COUP_SLOT_OBS, buf.data());
    const float* both = reinterpret_cast<const float*>(buf.data() + sizeof(coup_slot_result));
    return std::vector<float>(both + p * COUP_OBS_SIZE, both + (p + 1) * COUP_OBS_SIZE);
  }
  std::vector<float> InformationStateTensor(Player p) const {
    if (Host()) {
      std::vector<float> both(2 * COUP_INFO_STATE_SIZE);
      Check(coup_host_state_tensors(&q_, nullptr, both.data()), "coup_host_state_tensors");
      return std::vector<float>(both.begin() + p * COUP_INFO_STATE_SIZE,
                                both.begin() + (p + 1) * COUP_INFO_STATE_SIZE);
    }
    std::vector<uint8_t> buf(sizeof(coup_slot_result) + 2 * COUP_INFO_STATE_SIZE * 4);
    detail::ThePool().Op(slot_, nullptr, -1, COUP_SLOT_INFO, buf.data());
    const float* both = reinterpret_cast<const float*>(buf.data() + sizeof(coup_slot_result));
    return std::vector<float>(both + p * COUP_INFO_STATE_SIZE, both + (p + 1) * COUP_INFO_STATE_SIZE);
  }

  std::string ObservationString(Player p) const {
    return detail::StateString(detail::Decode(Rec()), q_.history, p, false);
  }
  std::string InformationStateString(Player p) const {
    return detail::StateString(detail::Decode(Rec()), q_.history, p, true);
  }
  std::string ToString() const { return detail::StateString(detail::Decode(Rec()), q_.history, -1, false); }
  std::string ActionToString(Player p, Action a) const;

  std::vector<Action> History() const {
    std::vector<Action> h;
    for (const auto& pa : history_) h.push_back(pa.action);
    return h;
  }
  const std::vector<PlayerAction>& FullHistory() const { return history_; }
  int MoveNumber() const { return detail::Decode(Rec()).move_number; }
  // State::Serialize (spiel.cc:297-311)
  std::string Serialize() const {
    std::string s;
    for (const auto& pa : history_) s += std::to_string(pa.action) + "\n";
    return s;
  }
  std::array<uint32_t, 4> PackedRecord() const { return Rec(); }

 private:
  CoupState(const CoupGame* game, detail::Pool::Slot slot, std::vector<PlayerAction> history,
            const coup_slot_result& q)
      : game_(game), slot_(slot), history_(std::move(history)), q_(q) {}
  // the result of the last op on this lane (every op refreshes it)
  const coup_slot_result& Q() const { return q_; }
  bool Host() const { return slot_.seg < 0; }
  // in LegalActions() (ApplyActionWithLegalityCheck)
  bool Legal(Action a) const {
    return a >= 0 && a < COUP_NUM_ACTIONS && ((Q().legal_mask >> a) & 1u) && CurrentPlayer() != kTerminalPlayerId;
  }
  // ids outside 0..17: DoApplyAction raises at any node (coup.cc:493, 806; spiel.cc:327)
  static void CheckId(Action a, const char* what) {
    if (a < 0 || a >= COUP_NUM_ACTIONS) throw SpielError(std::string(what) + ": invalid action " + std::to_string(a));
  }
  std::array<uint32_t, 4> Rec() const { return {q_.record[0], q_.record[1], q_.record[2], q_.record[3]}; }

  const CoupGame* game_;
  detail::Pool::Slot slot_;
  std::vector<PlayerAction> history_;
  coup_slot_result q_{};
};

// open_spiel::coup::CoupGame (coup.h:199-231)
class CoupGame {
 public:
  std::unique_ptr<CoupState> NewInitialState() const { return std::unique_ptr<CoupState>(new CoupState(this)); }
  int NumDistinctActions() const { return COUP_NUM_ACTIONS; }
  int MaxChanceOutcomes() const { return COUP_NUM_CARD_TYPES; }
  int NumPlayers() const { return COUP_NUM_PLAYERS; }
  double MinUtility() const { return -2; }
  double MaxUtility() const { return 2; }
  double UtilitySum() const { return 0; }
  int MaxGameLength() const { return COUP_MAX_GAME_LENGTH; }
  int MaxChanceNodesInHistory() const { return 45; }
  std::vector<int> ObservationTensorShape() const { return {COUP_OBS_SIZE}; }
  std::vector<int> InformationStateTensorShape() const { return {COUP_INFO_STATE_SIZE}; }
  // ActionToString (coup.cc:1143-1149)
  std::string ActionToString(Player p, Action a) const {
    return p == kChancePlayerId ? std::string("Chance drawn card:") + detail::CardName((int)a)
                                : std::string(detail::ActionName((int)a));
  }
  std::string ToString() const { return "coup()"; }
  // Game::DeserializeState (spiel.cc:393-425): replay the history
  std::unique_ptr<CoupState> DeserializeState(const std::string& text) const {
    auto st = NewInitialState();
    size_t i = 0;
    while (i < text.size()) {
      size_t j = text.find('\n', i);
      if (j == std::string::npos) j = text.size();
      if (j > i) st->ApplyAction(std::stoll(text.substr(i, j - i)));
      i = j + 1;
    }
    return st;
  }
};

inline std::string CoupState::ActionToString(Player p, Action a) const { return game_->ActionToString(p, a); }

// LoadGame (spiel.h:1081-1090) for the one game this build provides
inline std::shared_ptr<const CoupGame> LoadGame(const std::string& name) {
  if (name.substr(0, name.find('(')) != "coup") throw SpielError("unknown game '" + name + "'");
  return std::make_shared<const CoupGame>();
}

}  // namespace coup_amd

#endif  // COUP_MI355X_HPP_
