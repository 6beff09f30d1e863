/* Drives librust_spiel.so -- the reference's per-state C ABI
 * (rust_open_spiel.h:24-84, include/coup_rust_abi.h) on the MI355X engine --
 * with the call pattern of the reference's Rust crate
 * (open_spiel/rust/src/rust_open_spiel.rs: State::legal_actions frees the
 * malloc'd buffer, chance_outcomes pairs StateLegalActions with
 * StateChanceOutcomeProbs, returns sizes its buffer by StateNumPlayers,
 * tensors are sized by State*TensorSize, strings come back with a length and
 * no NUL).  Pure C: it includes only coup_rust_abi.h.  Test tooling for
 * tests/test_rust_abi.py.
 *   rust_abi_driver <action> ...     replay a history, one JSON line per state
 *   rust_abi_driver --clone          Clone / DeleteState independence
 *   rust_abi_driver --params         GameParameters + LoadGameFromParameters
 *   rust_abi_driver --bot SEED       two uniform_random bots play one game
 *   rust_abi_driver --illegal        an illegal action: SpielFatalError, exit 1
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "coup_rust_abi.h"

static void put_quoted(const char* s, unsigned long n) {
  putchar('"');
  for (unsigned long i = 0; i < n; ++i) {
    const char c = s[i];
    if (c == '"' || c == '\\') {
      putchar('\\');
      putchar(c);
    } else if (c == '\n') {
      fputs("\\n", stdout);
    } else {
      putchar(c);
    }
  }
  putchar('"');
}

/* a returned string: print it, free it */
static void put_string(char* s, unsigned long n) {
  put_quoted(s, n);
  free(s);
}

static void put_sparse(const float* v, int n) {
  int first = 1;
  putchar('[');
  for (int i = 0; i < n; ++i) {
    if (v[i] == 0.0f) continue;
    printf("%s[%d,%d]", first ? "" : ",", i, (int)v[i]);
    first = 0;
  }
  putchar(']');
}

static void dump(const void* st, const long* hist, int nhist) {
  unsigned long n;
  printf("{\"history\":[");
  for (int i = 0; i < nhist; ++i) printf("%s%ld", i ? "," : "", hist[i]);
  const int cur = StateCurrentPlayer(st);
  printf("],\"current_player\":%d,\"is_terminal\":%s,\"is_chance\":%s", cur,
         StateIsTerminal(st) ? "true" : "false", StateIsChanceNode(st) ? "true" : "false");
  int nl = 0;
  long* legal = StateLegalActions(st, &nl);
  printf(",\"legal_actions\":[");
  for (int i = 0; i < nl; ++i) printf("%s%ld", i ? "," : "", legal[i]);
  printf("]");
  if (StateIsChanceNode(st)) {
    int np = 0;
    double* probs = StateChanceOutcomeProbs(st, &np);
    printf(",\"chance_outcomes\":[");
    for (int i = 0; i < np; ++i) printf("%s[%ld,%.17g]", i ? "," : "", legal[i], probs[i]);
    printf("]");
    free(probs);
  }
  if (nl > 0) {
    char* a = StateActionToString(st, cur, legal[0], &n);
    printf(",\"action0_str\":");
    put_string(a, n);
  }
  free(legal);
  const int players = StateNumPlayers(st);
  double* ret = (double*)malloc(sizeof(double) * players);
  StateReturns(st, ret);
  printf(",\"returns\":[%g,%g],\"player_return1\":%g", ret[0], ret[1], StatePlayerReturn(st, 1));
  free(ret);
  char* str = StateToString(st, &n); /* n is set by the call: never read it in the same expression */
  printf(",\"to_string\":");
  put_string(str, n);
  const int osz = StateObservationTensorSize(st), isz = StateInformationStateTensorSize(st);
  float* obs = (float*)malloc(sizeof(float) * osz);
  float* info = (float*)malloc(sizeof(float) * isz);
  for (int p = 0; p < players; ++p) {
    StateObservationTensor(st, p, obs, osz);
    StateInformationStateTensor(st, p, info, isz);
    printf(",\"obs%d\":", p);
    put_sparse(obs, osz);
    printf(",\"info%d\":", p);
    put_sparse(info, isz);
  }
  free(obs);
  free(info);
  if (cur >= 0) { /* the no-argument strings are for the current player (spiel.h:484-486, 543-545) */
    str = StateObservationString(st, &n);
    printf(",\"obs_str\":");
    put_string(str, n);
    str = StateInformationStateString(st, &n);
    printf(",\"info_str\":");
    put_string(str, n);
  }
  printf("}\n");
}

static void* load_coup(void) {
  void* game = LoadGame("coup");
  unsigned long n;
  char* s = GameShortName(game, &n);
  if (n != 4 || memcmp(s, "coup", 4) != 0) exit(3);
  free(s);
  return game;
}

int main(int argc, char** argv) {
  if (argc >= 2 && strcmp(argv[1], "--params") == 0) {
    void* params = NewGameParameters();
    GameParametersSetString(params, "name", "coup");
    unsigned long n;
    char* ser = GameParametersSerialize(params, &n);
    printf("{\"serialized\":");
    put_string(ser, n);
    void* game = LoadGameFromParameters(params);
    int sz = 0;
    int* shape = GameObservationTensorShape(game, &sz);
    int isz = 0;
    int* ishape = GameInformationStateTensorShape(game, &isz);
    char* ln = GameLongName(game, &n);
    printf(",\"long_name\":");
    put_string(ln, n);
    printf(",\"players\":%d,\"max_len\":%d,\"actions\":%d,\"obs_shape\":[%d],\"info_shape\":[%d],\"dims\":[%d,%d]",
           GameNumPlayers(game), GameMaxGameLength(game), GameNumDistinctActions(game), shape[0], ishape[0], sz,
           isz);
    free(shape);
    free(ishape);
    GameParametersSetInt(params, "seed", 7);
    GameParametersSetDouble(params, "x", 0.25);
    ser = GameParametersSerialize(params, &n);
    printf(",\"serialized3\":");
    put_string(ser, n);
    printf("}\n");
    DeleteGameParameters(params);
    DeleteGame(game);
    return 0;
  }
  void* game = load_coup();
  if (argc >= 2 && strcmp(argv[1], "--clone") == 0) {
    void* st = GameNewInitialState(game);
    const long deal[] = {4, 3, 2, 0};
    for (int i = 0; i < 4; ++i) StateApplyAction(st, deal[i]);
    void* c = StateClone(st);
    StateApplyAction(c, 0); /* Income on the clone only */
    unsigned long n1, n2;
    char* a = StateToString(st, &n1);
    char* b = StateToString(c, &n2);
    printf("{\"differ\":%s,\"orig_player\":%d,\"clone_player\":%d}\n",
           (n1 != n2 || memcmp(a, b, n1) != 0) ? "true" : "false", StateCurrentPlayer(st), StateCurrentPlayer(c));
    free(a);
    free(b);
    DeleteState(st); /* the clone outlives its source */
    printf("{\"clone_after_delete\":%d}\n", StateCurrentPlayer(c));
    DeleteState(c);
    DeleteGame(game);
    return 0;
  }
  if (argc >= 3 && strcmp(argv[1], "--bot") == 0) {
    void* params = NewGameParameters();
    GameParametersSetInt(params, "seed", atoi(argv[2]));
    void* bots[2] = {BotRegistererCreateByName("uniform_random", game, 0, params),
                     BotRegistererCreateByName("uniform_random", game, 1, params)};
    void* chance = BotRegistererCreateByName("uniform_random", game, -1, params);
    void* st = GameNewInitialState(game);
    int moves = 0;
    while (!StateIsTerminal(st)) {
      const int p = StateCurrentPlayer(st);
      const long a = BotStep(p < 0 ? chance : bots[p], st);
      for (int k = 0; k < 2; ++k) BotInformAction(bots[k], st, p, a);
      StateApplyAction(st, a);
      ++moves;
    }
    double r[2];
    StateReturns(st, r);
    printf("{\"moves\":%d,\"returns\":[%g,%g]}\n", moves, r[0], r[1]);
    BotRestart(bots[0]);
    DeleteBot(bots[0]);
    DeleteBot(bots[1]);
    DeleteBot(chance);
    DeleteGameParameters(params);
    DeleteState(st);
    DeleteGame(game);
    return 0;
  }
  if (argc >= 2 && strcmp(argv[1], "--unchecked") == 0) {
    /* the actions, legal or not, then the current player, its legal
     * actions and player 0's observation tensor */
    void* st = GameNewInitialState(game);
    for (int i = 2; i < argc; ++i) StateApplyAction(st, atol(argv[i]));
    int n = 0;
    long* legal = StateLegalActions(st, &n);
    float obs[98];
    StateObservationTensor(st, 0, obs, 98);
    printf("{\"player\":%d,\"legal\":[", StateCurrentPlayer(st));
    for (int i = 0; i < n; ++i) printf(i ? ",%ld" : "%ld", legal[i]);
    printf("],\"obs0\":[");
    for (int i = 0; i < 98; ++i) printf(i ? ",%g" : "%g", obs[i]);
    printf("]}\n");
    free(legal);
    DeleteState(st);
    DeleteGame(game);
    return 0;
  }
  if (argc >= 2 && strcmp(argv[1], "--illegal") == 0) {
    void* st = GameNewInitialState(game);
    const long deal[] = {4, 3, 2, 0};
    for (int i = 0; i < 4; ++i) StateApplyAction(st, deal[i]);
    printf("{\"before\":\"ok\"}\n");
    fflush(stdout);
    StateApplyAction(st, 9); /* Pass at the first decision: not legal */
    printf("{\"illegal\":\"accepted\"}\n");
    return 0;
  }
  void* st = GameNewInitialState(game);
  long* hist = (long*)malloc(sizeof(long) * (size_t)(argc > 1 ? argc : 1));
  dump(st, hist, 0);
  for (int i = 1; i < argc; ++i) {
    hist[i - 1] = atol(argv[i]);
    StateApplyAction(st, hist[i - 1]);
    dump(st, hist, i);
  }
  free(hist);
  DeleteState(st);
  DeleteGame(game);
  return 0;
}
