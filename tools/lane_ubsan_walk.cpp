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
// Unchecked walks (argv[2] == "unchecked"): at decision nodes half the
// actions are any id 0..17; the lane applies every one with
// apply_action_unchecked (the per-game ops' path), the oracle with
// oc_apply_action_unchecked; accepted / rejected and the records must agree.
// A legal action through apply_action_unchecked must also equal
// apply_action on a copy wherever the reference accepts it.
static int unchecked_walks(int games, uint32_t (*rnd)()) {
  long steps = 0, rejected = 0;
  for (int g = 0; g < games; ++g) {
    Lane L = initial_lane(0);
    oc_state s;
    oc_init(&s);
    for (int k = 0; k < 200 && !is_terminal(L); ++k) {
      const uint32_t m = legal_mask(L);
      uint32_t a;
      if ((m & 0x3FFFFu) && ((m & kChanceFlag) || (rnd() & 1u))) {
        const uint32_t mm0 = m & 0x3FFFFu;
        uint32_t j = rnd() % __builtin_popcount(mm0);
        a = 0;
        for (uint32_t mm = mm0;; mm &= mm - 1) if (j-- == 0) { a = __builtin_ctz(mm); break; }
      } else {
        a = rnd() % 18u;
      }
      NoHistory none;
      const bool legal = (m >> a) & 1u;
      Lane C = L;
      const uint4 pre = pack(L);
      const bool lane_ok = apply_action_unchecked(L, a, none);
      const bool lane_ok2 = lane_ok && !L.err;
      if (legal && lane_ok) {
        apply_action(C, a, none);
        const uint4 c = pack(C), u = pack(L);
        if (c.x != u.x || c.y != u.y || c.z != u.z || c.w != u.w) {
          printf("CHECKED/UNCHECKED DIFF game %d step %d a=%u\n", g, k, a);
          return 1;
        }
      }
      const bool ref_ok = oc_apply_action_unchecked(&s, (int)a) == 0;
      ++steps;
      rejected += !ref_ok;
      uint4 w = pack(L);
      uint32_t o[4];
      oc_pack(&s, 0, 0, o);
      if (lane_ok2 != ref_ok || w.x != o[0] || w.y != o[1] || w.z != o[2] || w.w != o[3]) {
        printf("DIFF game %d step %d a=%u legal=%d lane_ok=%d err=%u ref_ok=%d\n", g, k, a, (int)legal, (int)lane_ok,
               L.err, (int)ref_ok);
        printf("  pre  %08x %08x %08x %08x\n", pre.x, pre.y, pre.z, pre.w);
        printf("  lane %08x %08x %08x %08x\n  ref  %08x %08x %08x %08x\n", w.x, w.y, w.z, w.w, o[0], o[1], o[2], o[3]);
        return 1;
      }
      if (!ref_ok && !(legal_mask(L) & 0x3FFFFu) && !is_terminal(L)) break;  // nothing left to play
    }
  }
  printf("ok %d games %ld actions %ld rejected\n", games, steps, rejected);
  return 0;
}

static uint64_t g_x = 88172645463325252ull;
static uint32_t xorshift() { g_x ^= g_x << 13; g_x ^= g_x >> 7; g_x ^= g_x << 17; return (uint32_t)g_x; }

int main(int argc, char** argv) {
  const int games = argc > 1 ? atoi(argv[1]) : 20000;
  if (argc > 2 && argv[2][0] == 'u') return unchecked_walks(games, xorshift);
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
