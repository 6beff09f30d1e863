// Drives the C++ host layer (include/coup_mi355x.hpp) through one game and
// prints one JSON object per state, so tests/test_gpu_cpp_api.py can compare
// it with the reference's golden transcript.  Test tooling.
//   state_driver <action> <action> ...      (the history to replay)
//   state_driver --illegal                  (error behaviour check)
//   state_driver --unchecked                (ApplyAction without a legality check)
//   state_driver --children                 (batched Children == Child one by one)
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>

#include "coup_mi355x.hpp"

using namespace coup_amd;

static std::string Quote(const std::string& s) {
  std::string o = "\"";
  for (char c : s) {
    if (c == '"' || c == '\\') {
      o += '\\';
      o += c;
    } else if (c == '\n') {
      o += "\\n";
    } else {
      o += c;
    }
  }
  return o + "\"";
}

template <class V>
static std::string List(const V& v) {
  std::string o = "[";
  for (size_t i = 0; i < v.size(); ++i) o += (i ? "," : "") + std::to_string(v[i]);
  return o + "]";
}

// sparse [[index, value], ...] like tests/golden/playthrough_coup.json
static std::string Sparse(const std::vector<float>& v) {
  std::string o = "[";
  bool first = true;
  for (size_t i = 0; i < v.size(); ++i) {
    if (v[i] == 0.0f) continue;
    o += (first ? "[" : ",[") + std::to_string(i) + "," + std::to_string((int)v[i]) + "]";
    first = false;
  }
  return o + "]";
}

static void Dump(const CoupState& s) {
  std::string o = "{\"history\":" + List(s.History());
  o += ",\"current_player\":" + std::to_string(s.CurrentPlayer());
  o += ",\"is_terminal\":" + std::string(s.IsTerminal() ? "true" : "false");
  o += ",\"is_chance\":" + std::string(s.IsChanceNode() ? "true" : "false");
  o += ",\"legal_actions\":" + List(s.LegalActions());
  if (s.IsChanceNode()) {
    o += ",\"chance_outcomes\":[";
    const auto co = s.ChanceOutcomes();
    for (size_t i = 0; i < co.size(); ++i) {
      char buf[64];
      std::snprintf(buf, sizeof buf, "%s[%lld,%.17g]", i ? "," : "", (long long)co[i].first, co[i].second);
      o += buf;
    }
    o += "]";
  }
  o += ",\"rewards\":" + List(s.Rewards()) + ",\"returns\":" + List(s.Returns());
  o += ",\"to_string\":" + Quote(s.ToString());
  for (int p = 0; p < 2; ++p) {
    const std::string k = std::to_string(p);
    o += ",\"obs" + k + "\":" + Sparse(s.ObservationTensor(p));
    o += ",\"info" + k + "\":" + Sparse(s.InformationStateTensor(p));
    o += ",\"obs_str" + k + "\":" + Quote(s.ObservationString(p));
    o += ",\"info_str" + k + "\":" + Quote(s.InformationStateString(p));
  }
  o += ",\"serialize\":" + Quote(s.Serialize()) + "}";
  std::printf("%s\n", o.c_str());
}

int main(int argc, char** argv) {
  try {
    auto game = LoadGame("coup");
    auto state = game->NewInitialState();
    if (argc == 2 && std::string(argv[1]) == "--children") {
      std::mt19937 rng(5);
      int checked = 0;
      for (int game_no = 0; game_no < 6; ++game_no) {
        auto st = game->NewInitialState();
        for (int d = 0; d < 100 && !st->IsTerminal(); ++d) {
          const auto legal = st->LegalActions();
          auto kids = st->Children(legal);
          for (size_t k = 0; k < legal.size(); ++k) {
            auto c = st->Child(legal[k]);
            if (c->PackedRecord() != kids[k]->PackedRecord() || c->History() != kids[k]->History() ||
                c->LegalActions() != kids[k]->LegalActions() || c->ToString() != kids[k]->ToString()) {
              std::printf("{\"mismatch\":%s}\n", List(c->History()).c_str());
              return 1;
            }
            ++checked;
          }
          st = std::move(kids[rng() % kids.size()]);
        }
      }
      std::printf("{\"children_checked\":%d}\n", checked);
      return 0;
    }
    if (argc == 2 && std::string(argv[1]) == "--unchecked") {
      // policy_analysis.py:283-299: a Tax answered by Block, outside
      // LegalActions (coup.cc:867-871): the legality-checked form throws,
      // ApplyAction applies it as the reference does
      for (int a : {1, 1, 3, 3, 3}) state->ApplyAction(a);
      bool checked_threw = false;
      try {
        state->ApplyActionWithLegalityCheck(10);
      } catch (const SpielError&) {
        checked_threw = true;
      }
      state->ApplyAction(10);
      auto child = state->Child(9);  // the Pass that ends the blocked turn
      std::printf("{\"checked_threw\":%s,\"history\":%s,\"child\":%s,\"child_player\":%d,\"child_legal\":%s}\n",
                  checked_threw ? "true" : "false", List(state->History()).c_str(), List(child->History()).c_str(),
                  child->CurrentPlayer(), List(child->LegalActions()).c_str());
      return 0;
    }
    if (argc == 2 && std::string(argv[1]) == "--illegal") {
      for (int a : {4, 3, 2, 0}) state->ApplyAction(a);
      const auto before = state->History();
      try {
        state->ApplyAction(9);  // Pass at the first decision
        std::printf("{\"illegal\":\"accepted\"}\n");
        return 1;
      } catch (const SpielError& e) {
        auto clone = state->Clone();
        auto child = state->Child(0);
        std::printf("{\"illegal\":\"rejected\",\"history\":%s,\"clone\":%s,\"child\":%s,\"roundtrip\":%s}\n",
                    List(before).c_str(), List(clone->History()).c_str(), List(child->History()).c_str(),
                    List(game->DeserializeState(child->Serialize())->History()).c_str());
        return 0;
      }
    }
    Dump(*state);
    for (int i = 1; i < argc; ++i) {
      state->ApplyAction(std::atoll(argv[i]));
      Dump(*state);
    }
  } catch (const SpielError& e) {
    std::fprintf(stderr, "SpielError: %s\n", e.what());
    return 2;
  }
  return 0;
}
