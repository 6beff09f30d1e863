// rust_spiel.cpp -- librust_spiel.so: the reference's per-state C ABI
// (open_spiel/rust/src/rust_open_spiel.h:24-84, declared here as
// include/coup_rust_abi.h) on the MI355X engine.
//
// The reference builds this API as the shared library `rust_spiel` over the
// whole OpenSpiel core (rust_open_spiel.cc, open_spiel/rust/CMakeLists.txt);
// its Rust crate links `dylib=rust_spiel` (open_spiel/rust/build.rs).  This
// file implements the same entry points over include/coup_mi355x.hpp: a
// state handle is a coup_amd::CoupState, i.e. one lane of the device-
// resident lane pool, and every rules operation is a coup_slot_op launch on
// that lane.  Host-only C++ (the kernels live in libcoup_mi355x.so).
//
// Conventions kept from the reference:
//   - malloc'd result buffers owned by the caller (rust_open_spiel.cc:38-53);
//     strings are copied without a terminating NUL, length through `length`;
//   - fatal errors print "Spiel Fatal Error: <msg>" and exit(1)
//     (SpielDefaultErrorHandler, spiel_utils.cc:119-136).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "coup_mi355x.hpp"
#include "coup_rust_abi.h"

namespace {

using coup_amd::CoupGame;
using coup_amd::CoupState;

[[noreturn]] void Fatal(const std::string& msg) {
  std::fprintf(stderr, "Spiel Fatal Error: %s\n\n", msg.c_str());
  std::fflush(stderr);
  std::exit(1);
}

// Runs f; a coup_amd::SpielError (illegal action, HIP failure, ...) becomes a
// SpielFatalError, as an exception cannot cross the C ABI.
template <class F>
auto Guard(F&& f) -> decltype(f()) {
  try {
    return f();
  } catch (const std::exception& e) {
    Fatal(e.what());
  }
}

// GameParameter (game_parameters.h:39-150) reduced to what the C API sets:
// int, double and string values.
struct Param {
  enum Kind { kInt, kDouble, kString } kind;
  int i = 0;
  double d = 0;
  std::string s;
};
using Params = std::map<std::string, Param>;

// FormatDouble (spiel_utils.cc:100-117): "%.15f" with trailing zeros
// trimmed to one decimal.
std::string FormatDouble(double v) {
  char buf[64];
  std::snprintf(buf, sizeof(buf), "%.15f", v);
  std::string s(buf);
  const size_t dot = s.find('.');
  if (dot == std::string::npos) return s + ".0";
  while (s.size() > dot + 2 && s.back() == '0') s.pop_back();
  return s;
}

// GameParameter::Serialize + SerializeGameParameters (game_parameters.cc:
// 78-135): name=kType/value/false joined by '|', in key order.
std::string Serialize(const Params& p) {
  std::string out;
  for (const auto& kv : p) {
    if (!out.empty()) out += "|";
    const Param& v = kv.second;
    out += kv.first + "=";
    if (v.kind == Param::kInt) {
      out += "kInt/" + std::to_string(v.i);
    } else if (v.kind == Param::kDouble) {
      out += "kDouble/" + FormatDouble(v.d);
    } else {
      std::string s = v.s;
      for (size_t k = 0; (k = s.find('\n', k)) != std::string::npos; k += 3) s.replace(k, 1, "\\\\n");
      out += "kString/" + s;
    }
    out += "/false";
  }
  return out;
}

struct GameHolder {  // GamePointerHolder (rust_open_spiel.cc:40-45)
  std::shared_ptr<const CoupGame> game;
};

const CoupGame& GameOf(const void* game_ptr) {
  if (!game_ptr) Fatal("null game handle");
  return *static_cast<const GameHolder*>(game_ptr)->game;
}

CoupState& StateOf(const void* state_ptr) {
  if (!state_ptr) Fatal("null state handle");
  return *static_cast<CoupState*>(const_cast<void*>(state_ptr));
}

char* CopyString(const std::string& s, unsigned long* length) {  // NOLINT
  *length = s.size();
  char* buf = static_cast<char*>(std::malloc(s.size() > 0 ? s.size() : 1));
  if (!s.empty()) std::memcpy(buf, s.data(), s.size());
  return buf;
}

template <class T, class U>
T* CopyVector(const std::vector<U>& v, int* size) {
  *size = (int)v.size();
  T* buf = static_cast<T*>(std::malloc(v.empty() ? sizeof(T) : v.size() * sizeof(T)));
  for (size_t k = 0; k < v.size(); ++k) buf[k] = (T)v[k];
  return buf;
}

// The player-indexed observers check 0 <= player < NumPlayers (coup.cc:251-252,
// 291-292).
void CheckPlayer(int player) {
  if (player < 0 || player >= COUP_NUM_PLAYERS)
    Fatal("coup.cc:251 CHECK_GE(player, 0) / CHECK_LT(player, num_players_) failed for player " +
          std::to_string(player));
}

// UniformRandomBot (open_spiel/bots): a uniform draw over LegalActions() at
// decision nodes and over ChanceOutcomes() by probability at chance nodes.
struct UniformBot {
  int player;
  int seed;
  std::mt19937 rng;
};

}  // namespace

extern "C" {

// ------------------------------------------------------------ parameters
void* NewGameParameters() { return new Params(); }

void DeleteGameParameters(void* params_ptr) { delete static_cast<Params*>(params_ptr); }

void GameParametersSetInt(void* params_ptr, const char* key, int value) {
  Param p{Param::kInt};
  p.i = value;
  (*static_cast<Params*>(params_ptr))[key] = p;
}

void GameParametersSetDouble(void* params_ptr, const char* key, double value) {
  Param p{Param::kDouble};
  p.d = value;
  (*static_cast<Params*>(params_ptr))[key] = p;
}

void GameParametersSetString(void* params_ptr, const char* key, const char* value) {
  Param p{Param::kString};
  p.s = value;
  (*static_cast<Params*>(params_ptr))[key] = p;
}

char* GameParametersSerialize(const void* params_ptr, unsigned long* length) {  // NOLINT
  return CopyString(Serialize(*static_cast<const Params*>(params_ptr)), length);
}

// ------------------------------------------------------------------ game
void* LoadGame(const char* name) {
  return Guard([&] { return static_cast<void*>(new GameHolder{coup_amd::LoadGame(name ? name : "")}); });
}

// LoadGame(GameParameters) (spiel.cc:225-240): the "name" entry picks the
// game, every other entry is a game parameter -- Coup has none (coup.cc:51-52).
void* LoadGameFromParameters(const void* params_ptr) {
  const Params& p = *static_cast<const Params*>(params_ptr);
  auto it = p.find("name");
  if (it == p.end()) Fatal("No 'name' parameter in params: " + Serialize(p));
  if (it->second.kind != Param::kString) Fatal("parameter 'name' must be a string");
  for (const auto& kv : p)
    if (kv.first != "name") Fatal("Unknown parameter '" + kv.first + "' for game coup (coup takes none)");
  return LoadGame(it->second.s.c_str());
}

void DeleteGame(void* game_ptr) { delete static_cast<GameHolder*>(game_ptr); }

char* GameShortName(const void* game_ptr, unsigned long* length) {  // NOLINT
  (void)GameOf(game_ptr);
  return CopyString("coup", length);  // coup.cc:38-52
}

char* GameLongName(const void* game_ptr, unsigned long* length) {  // NOLINT
  (void)GameOf(game_ptr);
  return CopyString("Coup", length);
}

void* GameNewInitialState(const void* game_ptr) {
  const CoupGame& g = GameOf(game_ptr);
  return Guard([&] { return static_cast<void*>(g.NewInitialState().release()); });
}

int GameNumPlayers(const void* game_ptr) { return GameOf(game_ptr).NumPlayers(); }

int GameMaxGameLength(const void* game_ptr) { return GameOf(game_ptr).MaxGameLength(); }

int GameNumDistinctActions(const void* game_ptr) { return GameOf(game_ptr).NumDistinctActions(); }

int* GameObservationTensorShape(const void* game_ptr, int* size) {
  return CopyVector<int>(GameOf(game_ptr).ObservationTensorShape(), size);
}

int* GameInformationStateTensorShape(const void* game_ptr, int* size) {
  return CopyVector<int>(GameOf(game_ptr).InformationStateTensorShape(), size);
}

// ----------------------------------------------------------------- state
void DeleteState(void* state_ptr) { delete static_cast<CoupState*>(state_ptr); }

void* StateClone(const void* state_ptr) {
  CoupState& s = StateOf(state_ptr);
  return Guard([&] { return static_cast<void*>(s.Clone().release()); });
}

char* StateToString(const void* state_ptr, unsigned long* length) {  // NOLINT
  return CopyString(StateOf(state_ptr).ToString(), length);
}

long* StateLegalActions(const void* state_ptr, int* num_legal_actions) {  // NOLINT
  static_assert(sizeof(long) == sizeof(coup_amd::Action), "Action is int64_t");  // NOLINT
  return CopyVector<long>(StateOf(state_ptr).LegalActions(), num_legal_actions);  // NOLINT
}

int StateCurrentPlayer(const void* state_ptr) { return StateOf(state_ptr).CurrentPlayer(); }

char* StateActionToString(const void* state_ptr, int player, long action, unsigned long* length) {  // NOLINT
  return CopyString(StateOf(state_ptr).ActionToString(player, action), length);
}

int StateIsTerminal(const void* state_ptr) { return StateOf(state_ptr).IsTerminal() ? 1 : 0; }

int StateIsChanceNode(const void* state_ptr) { return StateOf(state_ptr).IsChanceNode() ? 1 : 0; }

int StateNumPlayers(const void* state_ptr) { return StateOf(state_ptr).NumPlayers(); }

void StateApplyAction(void* state_ptr, long action) {  // NOLINT
  CoupState& s = StateOf(state_ptr);
  Guard([&] {
    s.ApplyAction(action);
    return 0;
  });
}

void StateReturns(const void* state_ptr, double* returns_buf) {
  const std::vector<double> r = StateOf(state_ptr).Returns();
  std::memcpy(returns_buf, r.data(), r.size() * sizeof(double));
}

double StatePlayerReturn(const void* state_ptr, int player) {
  CheckPlayer(player);
  return StateOf(state_ptr).PlayerReturn(player);
}

double* StateChanceOutcomeProbs(const void* state_ptr, int* size) {
  CoupState& s = StateOf(state_ptr);
  const auto outcomes = Guard([&] { return s.ChanceOutcomes(); });  // coup.cc:1063 CHECK(IsChanceNode())
  std::vector<double> p;
  for (const auto& o : outcomes) p.push_back(o.second);
  return CopyVector<double>(p, size);
}

char* StateObservationString(const void* state_ptr, unsigned long* length) {  // NOLINT
  CoupState& s = StateOf(state_ptr);
  const int p = s.CurrentPlayer();  // State::ObservationString() (spiel.h:543-545)
  CheckPlayer(p);
  return CopyString(s.ObservationString(p), length);
}

char* StateInformationStateString(const void* state_ptr, unsigned long* length) {  // NOLINT
  CoupState& s = StateOf(state_ptr);
  const int p = s.CurrentPlayer();  // State::InformationStateString() (spiel.h:484-486)
  CheckPlayer(p);
  return CopyString(s.InformationStateString(p), length);
}

int StateInformationStateTensorSize(const void* state_ptr) {
  (void)StateOf(state_ptr);
  return COUP_INFO_STATE_SIZE;
}

int StateObservationTensorSize(const void* state_ptr) {
  (void)StateOf(state_ptr);
  return COUP_OBS_SIZE;
}

// ContiguousAllocator over a span of `length` floats (observer.h:159-176): the
// span must hold the whole tensor.
void StateObservationTensor(const void* state_ptr, int player, float* obs_buf, int length) {
  CheckPlayer(player);
  if (length != COUP_OBS_SIZE) Fatal("ObservationTensor: span of " + std::to_string(length) + " floats, need 98");
  CoupState& s = StateOf(state_ptr);
  const std::vector<float> t = Guard([&] { return s.ObservationTensor(player); });
  std::memcpy(obs_buf, t.data(), t.size() * sizeof(float));
}

void StateInformationStateTensor(const void* state_ptr, int player, float* infostate_buf, int length) {
  CheckPlayer(player);
  if (length != COUP_INFO_STATE_SIZE)
    Fatal("InformationStateTensor: span of " + std::to_string(length) + " floats, need 2492");
  CoupState& s = StateOf(state_ptr);
  const std::vector<float> t = Guard([&] { return s.InformationStateTensor(player); });
  std::memcpy(infostate_buf, t.data(), t.size() * sizeof(float));
}

// ------------------------------------------------------------------ bots
void DeleteBot(void* bot_ptr) { delete static_cast<UniformBot*>(bot_ptr); }

long BotStep(void* bot_ptr, const void* state_ptr) {  // NOLINT
  UniformBot& b = *static_cast<UniformBot*>(bot_ptr);
  CoupState& s = StateOf(state_ptr);
  if (s.IsChanceNode()) {
    const auto outcomes = s.ChanceOutcomes();
    const double z = std::uniform_real_distribution<double>(0.0, 1.0)(b.rng);
    double sum = 0;
    for (const auto& o : outcomes) {  // SampleAction's rule (spiel.cc:279-286)
      if (sum <= z && z < sum + o.second) return (long)o.first;  // NOLINT
      sum += o.second;
    }
    return (long)outcomes.back().first;  // NOLINT
  }
  const std::vector<coup_amd::Action> legal = s.LegalActions();
  if (legal.empty()) Fatal("BotStep: no legal actions (terminal state)");
  const size_t k = std::uniform_int_distribution<size_t>(0, legal.size() - 1)(b.rng);
  return (long)legal[k];  // NOLINT
}

void BotInformAction(void* bot_ptr, const void* state_ptr, int player_id, long action) {  // NOLINT
  (void)bot_ptr;
  (void)state_ptr;
  (void)player_id;
  (void)action;  // a uniform bot keeps no state
}

void BotRestart(void* bot_ptr) {
  UniformBot& b = *static_cast<UniformBot*>(bot_ptr);
  b.rng.seed((unsigned)b.seed);
}

// BotRegisterer::CreateByName (spiel_bots.cc): this build registers one bot.
void* BotRegistererCreateByName(const char* bot_name_ptr, const void* game_ptr, int player_id,
                                const void* params_ptr) {
  (void)GameOf(game_ptr);
  const std::string name = bot_name_ptr ? bot_name_ptr : "";
  if (name != "uniform_random") Fatal("Unknown bot: " + name + " (this build provides uniform_random)");
  int seed = 0;
  if (params_ptr) {
    const Params& p = *static_cast<const Params*>(params_ptr);
    auto it = p.find("seed");
    if (it != p.end()) {
      if (it->second.kind != Param::kInt) Fatal("uniform_random: 'seed' must be an int");
      seed = it->second.i;
    }
  }
  return new UniformBot{player_id, seed, std::mt19937((unsigned)seed)};
}

}  // extern "C"
