// Host build of the lane rules for debugging against the oracle:
//   g++ -O1 -g -I tools/hoststub -I open_spiel_coup_amd/csrc -I oracle \
//       tools/lane_host_check.cpp oracle/coup_oracle.c -o /tmp/lane_host_check
#include <cstdio>
#include "coup_lane.h"
extern "C" {
#include "coup_oracle.h"
}
using namespace coup;
int main(int argc, char** argv) {
  int hist[] = {4, 3, 2, 0, 1, 10, 11, 7, 5, 9, 3, 4, 16, 5, 11, 7, 0, 6, 10, 9, 3, 11, 8};
  Lane L = initial_lane(1);
  oc_state s;
  oc_init(&s);
  uint8_t hb[96];
  for (int k = 0; k < 23; ++k) {
    RegHistory rec;
    bool ok = apply_action(L, (uint32_t)hist[k], rec);
    rec.flush(hb);
    oc_apply_action(&s, hist[k]);
    uint4 g = pack(L);
    uint32_t o[4];
    oc_pack(&s, 1, 0, o);
    printf("%2d a=%2d ok=%d gpu %08x %08x %08x %08x  oracle %08x %08x %08x %08x %s\n", k, hist[k], ok, g.x, g.y, g.z,
           g.w, o[0], o[1], o[2], o[3], (g.x == o[0] && g.y == o[1] && g.z == o[2] && g.w == o[3]) ? "" : "DIFF");
  }
  return 0;
}
