// Host build of the N-player lane rules (open_spiel_coup_amd/csrc/coup_nlane.h)
// checked step for step against the N-player specification
// (oracle/coup_nplayer.c).  Test tooling: tests/test_nlane_host.py builds and
// runs it on the CPU, so the device rules are checked before any GPU run.
//   g++ -O2 -std=c++17 -I tools/hoststub -I open_spiel_coup_amd/csrc -I oracle
//       tools/nlane_host_check.cpp oracle/coup_oracle.c oracle/coup_nplayer.c -o nlane_host_check
//   ./nlane_host_check N seed lanes steps auto_reset
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "coup_nlane.h"
extern "C" {
#include "coup_nplayer.h"
}

using namespace coup;
using namespace coup::np;

template <int N>
int run(uint64_t seed, int64_t n, int64_t steps, int auto_reset) {
  std::vector<int8_t> act(steps * n), rew(steps * n * N);
  std::vector<uint8_t> st(steps * n);
  std::vector<uint32_t> legal(steps * n), fin(n * 8);
  std::vector<float> obs(steps * n * N * 49 * N);
  int64_t done = 0, ret0 = 0;
  np_rollout_args a{};
  a.n_players = N;
  a.seed = seed;
  a.env_id_base = 0;
  a.n = n;
  a.steps = steps;
  a.auto_reset = auto_reset;
  a.actions = act.data();
  a.rewards = rew.data();
  a.step_type = st.data();
  a.legal = legal.data();
  a.final_state = fin.data();
  a.obs = obs.data();
  a.episodes_done = &done;
  a.return_sum_p0 = &ret0;
  std::vector<int32_t> lane_eps(n, 0), lane_ret(n, 0);
  a.lane_episodes = lane_eps.data();
  a.lane_return_sum = lane_ret.data();
  np_rollout(&a);
  int bad = 0;
  for (int64_t i = 0; i < n && bad < 5; ++i) {
    NRng rng{(uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)i, 0u, make_uint4(0, 0, 0, 0)};
    NLane<N> L = initial_lane<N>(0);
    resolve_chance(L, rng);
    int32_t eps = 0, rsum = 0;
    for (int64_t t = 0; t < steps && bad < 5; ++t) {
      int x;
      uint32_t s, rl, rc;
      int32_t r0;
      bool err;
      step_lane<N, true>(L, rng, 0u, auto_reset != 0, x, s, rl, rc, r0, err);
      if (s == 2u) {
        eps += 1;
        rsum += r0;
      }
      const int64_t o = t * n + i;
      bool ok = !err && x == act[o] && s == st[o] && legal_mask(L) == legal[o];
      for (int p = 0; p < N; ++p) {
        const int r = (uint32_t)p == rl ? -(int)((N - 1) * rc) : (int)rc;
        ok = ok && r == rew[o * N + p];
      }
      uint32_t rec[8];
      obs_record(L, rec);
      const float* ob = obs.data() + o * N * 49 * N;
      for (int q = 0; q < N && ok; ++q)
        for (int e = 0; e < 49 * N; ++e)
          if (obs_elem<N>(rec, (uint32_t)q, (uint32_t)e) != ob[q * 49 * N + e]) {
            std::printf("obs observer %d element %d\n", q, e);
            ok = false;
            break;
          }
      if (!ok) {
        std::printf("lane %lld step %lld: act %d/%d type %u/%u legal %x/%x err %d\n", (long long)i, (long long)t, x,
                    act[o], s, st[o], legal_mask(L), legal[o], (int)err);
        ++bad;
      }
    }
    if (eps != lane_eps[i] || rsum != lane_ret[i]) {
      std::printf("lane %lld episodes %d/%d return sum %d/%d\n", (long long)i, eps, lane_eps[i], rsum, lane_ret[i]);
      ++bad;
    }
    uint4 wa, wb;
    pack(L, wa, wb);
    const uint32_t g[8] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
    for (int k = 0; k < 8; ++k) {
      if (g[k] != fin[i * 8 + k]) {
        std::printf("lane %lld final word %d: %08x vs %08x\n", (long long)i, k, g[k], fin[i * 8 + k]);
        ++bad;
        break;
      }
    }
  }
  if (bad == 0) std::printf("OK N=%d lanes=%lld steps=%lld episodes=%lld\n", N, (long long)n, (long long)steps,
                            (long long)done);
  return bad ? 1 : 0;
}

int main(int argc, char** argv) {
  if (argc != 6) {
    std::fprintf(stderr, "usage: %s N seed lanes steps auto_reset\n", argv[0]);
    return 2;
  }
  const int N = std::atoi(argv[1]);
  const uint64_t seed = std::strtoull(argv[2], nullptr, 10);
  const int64_t n = std::atoll(argv[3]), steps = std::atoll(argv[4]);
  const int ar = std::atoi(argv[5]);
  switch (N) {
    case 2: return run<2>(seed, n, steps, ar);
    case 3: return run<3>(seed, n, steps, ar);
    case 4: return run<4>(seed, n, steps, ar);
    case 5: return run<5>(seed, n, steps, ar);
    case 6: return run<6>(seed, n, steps, ar);
    default: return 2;
  }
}
