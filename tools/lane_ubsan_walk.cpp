// Host build of the lane rules under UBSan (apply_decision = the effect
// form apply_decision_v2 by default, -DCOUP_RULES_V1 for the branch form): random legal-action walks
// (decisions and chance outcomes) against the oracle, every step.
//   g++ -O2 -g -fsanitize=undefined -fno-sanitize-recover=all -I tools/hoststub \
//       -I open_spiel_coup_amd/csrc -I oracle tools/lane_ubsan_walk.cpp oracle/coup_oracle.c -o /tmp/lane_ubsan_walk
#include <cstdio>
#include <cstdlib>
#include "coup_lane.h"
extern "C" {
#include "coup_oracle.h"
}
using namespace coup;
int main(int argc, char** argv) {
  const int games = argc > 1 ? atoi(argv[1]) : 20000;
  uint64_t x = 88172645463325252ull;
  auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return (uint32_t)x; };
  long steps = 0;
  for (int g = 0; g < games; ++g) {
    Lane L = initial_lane(0);
    oc_state s;
    oc_init(&s);
    while (!is_terminal(L)) {
      const uint32_t m = legal_mask(L) & 0x3FFFFu;
      if (!m) { printf("empty mask game %d\n", g); return 1; }
      uint32_t k = rnd() % __builtin_popcount(m), a = 0;
      for (uint32_t mm = m;; mm &= mm - 1) if (k-- == 0) { a = __builtin_ctz(mm); break; }
      NoHistory none;
      if (!apply_action(L, a, none)) { printf("rejected\n"); return 1; }
      oc_apply_action(&s, (int)a);
      uint4 w = pack(L);
      uint32_t o[4];
      oc_pack(&s, 0, 0, o);
      ++steps;
      if (w.x != o[0] || w.y != o[1] || w.z != o[2] || w.w != o[3] || current_player(L) != oc_current_player(&s)) {
        printf("DIFF game %d step %ld a=%u\n", g, steps, a);
        return 1;
      }
    }
  }
  printf("ok %d games %ld actions\n", games, steps);
  return 0;
}
