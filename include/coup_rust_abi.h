/*
 * coup_rust_abi.h -- the reference's per-state C ABI, served by the MI355X
 * engine.
 *
 * BStarcheus/open_spiel_coup exposes Game / State to Rust (and other FFI
 * users) through a pure C API, open_spiel/rust/src/rust_open_spiel.h:24-84,
 * built as the shared library `rust_spiel` (open_spiel/rust/CMakeLists.txt,
 * linked by open_spiel/rust/build.rs as `dylib=rust_spiel`).  This header
 * declares the same functions with the same C signatures; the build ships
 * them as open_spiel_coup_amd/librust_spiel.so, so the reference's Rust
 * crate (rust_open_spiel.rs) links it unchanged and plays "coup" on the GPU.
 *
 * Behind the entry points (open_spiel_coup_amd/csrc/rust_spiel.cpp):
 *   - a game handle is the one game this build provides, "coup";
 *   - a state handle is a coup_amd::CoupState (include/coup_mi355x.hpp):
 *     one lane of a device-resident lane pool, every rules operation one
 *     coup_slot_op launch (include/coup_mi355x.h);
 *   - returned buffers (char*, long*, int*, double*) are malloc'd and owned by
 *     the caller, who frees them, as in rust_open_spiel.cc:38-53; strings are
 *     NOT NUL-terminated, their length is returned through `length`;
 *   - errors follow SpielFatalError (spiel_utils.cc:119-136): the message
 *     "Spiel Fatal Error: ..." goes to stderr and the process exits with
 *     status 1 -- illegal actions, chance outcomes at a decision node, a
 *     string or tensor for a negative player, an unknown game or bot.
 */
#ifndef COUP_RUST_ABI_H_
#define COUP_RUST_ABI_H_

#ifdef __cplusplus
extern "C" {
#endif

/* GameParameters (rust_open_spiel.h:24-31).  Coup has no parameters
 * (coup.cc:51-52): LoadGameFromParameters accepts only {"name": "coup"}. */
void* NewGameParameters();
void DeleteGameParameters(void* params_ptr);
void GameParametersSetInt(void* params_ptr, const char* key, int value);
void GameParametersSetDouble(void* params_ptr, const char* key, double value);
void GameParametersSetString(void* params_ptr, const char* key, const char* value);
/* name=kType/value/is_mandatory joined by '|' (game_parameters.h:187-193) */
char* GameParametersSerialize(const void* params_ptr, unsigned long* length); /* NOLINT */

/* Game (rust_open_spiel.h:33-45, spiel.h:746-1035, coup.h:199-231) */
void* LoadGame(const char* name);
void* LoadGameFromParameters(const void* params_ptr);
void DeleteGame(void* game_ptr);
char* GameShortName(const void* game_ptr, unsigned long* length); /* NOLINT */
char* GameLongName(const void* game_ptr, unsigned long* length);  /* NOLINT */
void* GameNewInitialState(const void* game_ptr);
int GameNumPlayers(const void* game_ptr);
int GameMaxGameLength(const void* game_ptr);
int GameNumDistinctActions(const void* game_ptr);
int* GameObservationTensorShape(const void* game_ptr, int* size);
int* GameInformationStateTensorShape(const void* game_ptri, int* size);

/* State (rust_open_spiel.h:47-72, spiel.h:210-740, coup.h:111-197) */
void DeleteState(void* state_ptr);
void* StateClone(const void* state_ptr);
char* StateToString(const void* state_ptr, unsigned long* length); /* NOLINT */
long* StateLegalActions(const void* state_ptr, int* num_legal_actions); /* NOLINT */
int StateCurrentPlayer(const void* state_ptr);
char* StateActionToString(const void* state_ptr, int player, long action, /* NOLINT */
                          unsigned long* length);                         /* NOLINT */
int StateIsTerminal(const void* state_ptr);
int StateIsChanceNode(const void* state_ptr);
int StateNumPlayers(const void* state_ptr);
void StateApplyAction(void* state_ptr, long action); /* NOLINT */
void StateReturns(const void* state_ptr, double* returns_buf);
double StatePlayerReturn(const void* state_ptr, int player);
double* StateChanceOutcomeProbs(const void* state_ptr, int* size);
char* StateObservationString(const void* state_ptr, unsigned long* length);       /* NOLINT */
char* StateInformationStateString(const void* state_ptr, unsigned long* length);  /* NOLINT */
int StateInformationStateTensorSize(const void* state_ptr);
int StateObservationTensorSize(const void* state_ptr);
void StateObservationTensor(const void* state_ptr, int player, float* obs_buf, int length);
void StateInformationStateTensor(const void* state_ptr, int player, float* infostate_buf, int length);

/* Bots (rust_open_spiel.h:74-84).  The registry holds "uniform_random"
 * (open_spiel/bots: uniform over LegalActions / ChanceOutcomes, parameter
 * "seed", std::mt19937 here -- its stream is not the reference's absl one). */
void DeleteBot(void* bot_ptr);
long BotStep(void* bot_ptr, const void* state_ptr); /* NOLINT */
void BotInformAction(void* bot_ptr, const void* state_ptr, int player_id, long action); /* NOLINT */
void BotRestart(void* bot_ptr);
void* BotRegistererCreateByName(const char* bot_name_ptr, const void* game_ptr, int player_id,
                                const void* params_ptr);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* COUP_RUST_ABI_H_ */
