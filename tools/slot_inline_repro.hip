// slot_inline_repro.hip -- standalone reproducer for the k_slot code-generation
// hazard: the Coup rules of coup_lane.h applied by
// thread 0 of a wave to a WAVE-UNIFORM record (loaded through a uniform
// pointer, as k_slot does) give different records than the same rules on
// per-lane values.  Measurement / investigation tool, not product code.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I open_spiel_coup_amd/csrc \
//       tools/slot_inline_repro.hip open_spiel_coup_amd/csrc/coup_nplayer.hip -o build/slot_inline_repro
//   build/slot_inline_repro [cases]
//
// 1. k_gen: lane i plays a random legal prefix (decisions and deals) from
//    NewInitialState with its own xorshift stream and emits one case =
//    (packed record, a legal action).
// 2. k_lane: one thread per case applies it (the per-lane form every batched
//    kernel uses; bit-exact with the oracle in the GPU suite) -> expected.
// 3. k_uniform_inline: one wave per case, thread 0 loads the record through
//    the block's uniform pointer and runs the rules inlined (the original
//    k_slot) -> the compiler keeps the whole transition in SGPRs.
// 4. k_uniform_call: the same with the rules behind __noinline__ functions
//    (the shipped k_slot).
// 5. the product's own k_slot<false> built with COUP_SLOT_INLINE, one launch
//    per case, and stripped copies of it (variants below), to find the
//    construct that breaks it.
// 6. k_apply_bytehist: round 1's k_apply with the history byte stored from
//    inside the rules, batched and one lane per launch.
// Prints mismatches per action id, and the first few cases.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#ifndef COUP_SLOT_INLINE
#define COUP_SLOT_INLINE 1  // k_slot's rules inlined (the hazard under study)
#endif
#define COUP_INVESTIGATION_BUILD 1  // allows COUP_SLOT_INLINE (coup_kernels.hip refuses it otherwise)
#include "coup_kernels.hip"  // the product's k_slot, slot_transition, slot_result

using namespace coup;

struct Result {
  uint4 rec;
  uint32_t code;  // bit 0 accepted, bits 8..15 history index, 16..23 entry
  uint32_t legal;
  int32_t cur, term, r0, ret0;
};

__device__ __forceinline__ uint32_t xs(uint32_t& s) {
  s ^= s << 13;
  s ^= s >> 17;
  s ^= s << 5;
  return s;
}

__global__ void k_gen(int n, uint4* recs, uint32_t* acts) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t s = 0x9E3779B9u * (uint32_t)(i + 1) | 1u;
  Lane L = initial_lane(0u);
  const uint32_t steps = xs(s) % 64u;
  NoHistory none;
  for (uint32_t k = 0; k < steps; ++k) {
    const uint32_t m = legal_mask(L) & 0x3FFFFu;
    if (m == 0u) break;
    uint32_t mm = m, idx = xs(s) % (uint32_t)__popc(m);
    for (uint32_t j = 0; j < idx; ++j) mm &= mm - 1u;
    Lane T = L;
    if (!apply_action(T, (uint32_t)__builtin_ctz(mm), none)) break;
    if ((legal_mask(T) & 0x3FFFFu) == 0u) break;  // keep a non-terminal state to act on
    L = T;
  }
  const uint32_t m = legal_mask(L) & 0x3FFFFu;
  uint32_t mm = m, idx = m ? xs(s) % (uint32_t)__popc(m) : 0u;
  for (uint32_t j = 0; j < idx; ++j) mm &= mm - 1u;
  recs[i] = pack(L);
  acts[i] = m ? (uint32_t)__builtin_ctz(mm) : 0u;
}

__device__ __forceinline__ void run(uint4 w, uint32_t x, Result* out) {
  Lane L = unpack(w);
  const uint32_t idx = L.move;
  const uint32_t entry = is_chance(L) ? hist_deal(x, L.qids & 1u) : hist_decision(x, L.M);
  NoHistory none;
  const bool ok = apply_action(L, x, none);
  out->rec = ok ? pack(L) : w;
  out->code = (ok ? 1u : 0u) | (idx << 8) | (entry << 16);
  const Lane R = unpack(out->rec);
  out->legal = legal_mask(R);
  out->cur = current_player(R);
  out->term = is_terminal(R) ? 1 : 0;
  out->r0 = R.r0;
  out->ret0 = (int32_t)face_up_count(R.h1) - (int32_t)face_up_count(R.h0);
}

__device__ __noinline__ void run_call(uint4 w, uint32_t x, Result* out) { run(w, x, out); }

__global__ void k_lane(int n, const uint4* recs, const uint32_t* acts, Result* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  run(recs[i], acts[i], out + i);
}

// one wave per case; the record and the action are wave-uniform
__global__ __launch_bounds__(64) void k_uniform_inline(const uint4* recs, const uint32_t* acts, Result* out) {
  if (threadIdx.x == 0u) run(recs[blockIdx.x], acts[blockIdx.x], out + blockIdx.x);
}

__global__ __launch_bounds__(64) void k_uniform_call(const uint4* recs, const uint32_t* acts, Result* out) {
  if (threadIdx.x == 0u) run_call(recs[blockIdx.x], acts[blockIdx.x], out + blockIdx.x);
}

// Stripped copies of k_slot (inline build).  V = 0: exact copy;
// 1: no LDS history at all; 2: history in LDS but no entry write after the
// transition; 3: no slot_result; 4: no L = unpack(rec) after it;
// 5: as 1, record always loaded (no select with NewInitialState's constant);
// 6: as 5, the transition written as one expression (no early return);
// 7: as 1, the action is not checked against 0 (always applied).
__device__ __forceinline__ uint32_t transition_expr(uint4 w, uint32_t x, uint4* out) {
  Lane L = unpack(w);
  const uint32_t idx = L.move;
  const uint32_t entry = is_chance(L) ? hist_deal(x, L.qids & 1u) : hist_decision(x, L.M);
  NoHistory none;
  const bool ok = apply_action(L, x, none);
  *out = ok ? pack(L) : w;
  return (ok ? 1u : 0u) | 2u | (idx << 8) | (entry << 16);
}

template <int V>
__global__ __launch_bounds__(64) void k_slot_var(SlotArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t hist[kHist];
  const uint32_t t = threadIdx.x;
  const uint4* rs = a.src_state ? a.src_state : a.dst_state;
  const uint8_t* hs = a.src_state ? a.src_hist : a.dst_hist;
  if (V != 1 && t < 6u)
    reinterpret_cast<uint4*>(hist)[t] =
        a.init ? make_uint4(~0u, ~0u, ~0u, ~0u) : reinterpret_cast<const uint4*>(hs)[t];
  wave_sync();
  Lane L = initial_lane(0u);
  if (t == 0u) {
    uint4 rec = (V == 5 || V == 6) ? *rs : (a.init ? pack(initial_lane(0u)) : *rs);
    uint32_t ok = 1u;
    if (V == 7 || a.action >= 0) {
      const uint32_t r = V == 6 ? transition_expr(rec, (uint32_t)a.action, &rec)
                                : slot_transition(rec, (uint32_t)a.action, 0u, &rec);
      ok = r & 1u;
      if (V != 1 && V != 2 && (r & 2u)) hist[(r >> 8) & 0xFFu] = (uint8_t)(r >> 16);
    }
    if (a.store) *a.dst_state = rec;
    if (V != 3 && a.out) slot_result(rec, ok, a.out);
    if (V != 4) L = unpack(rec);
  }
  wave_sync();
  if (V != 1 && t < 6u) {
    const uint4 h = reinterpret_cast<const uint4*>(hist)[t];
    if (a.store) reinterpret_cast<uint4*>(a.dst_hist)[t] = h;
    if (a.out) reinterpret_cast<uint4*>(a.out->history)[t] = h;
  }
  if (t == 0u && a.out) a.out->pad[0] = (uint8_t)L.turn;  // keep L live
}

// Minimal forms between k_uniform_inline (correct) and k_slot (wrong), with
// SlotArgs input.  W = 0: thread 0 loads *dst_state, applies, stores it back
// (k_uniform_inline's shape); 1: + `if (a.action >= 0)` around the
// transition; 2: + `if (a.store)` around the store; 3: + slot_result;
// 4: + wave barriers before and after the thread-0 block.
template <int W>
__global__ __launch_bounds__(64) void k_min(SlotArgs a) {
  if (W >= 4) wave_sync();
  if (threadIdx.x == 0u) {
    uint4 rec = *a.dst_state;
    uint32_t ok = 1u;
    if (W < 1 || a.action >= 0) ok = transition_expr(rec, (uint32_t)a.action, &rec) & 1u;
    if (W < 2 || a.store) *a.dst_state = rec;
    if (W >= 3 && a.out) slot_result(rec, ok, a.out);
  }
  if (W >= 4) wave_sync();
}

// The round-1 k_apply form: the history byte stored
// from INSIDE the inlined rules through a per-lane pointer, one thread per
// lane.  Launched over all cases (a batch) and one case per launch (the
// 1-lane env of a per-game State then, only thread 0 active).
struct ByteHistory {
  uint8_t* bytes;
  __device__ __forceinline__ void record(uint32_t idx, uint32_t entry) {
    if (idx < (uint32_t)kHist) bytes[idx] = (uint8_t)entry;
  }
};

__global__ __launch_bounds__(256) void k_apply_bytehist(int n, uint4* state, const uint32_t* acts, uint8_t* hist) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Lane L = unpack(state[i]);
  ByteHistory h{hist + (size_t)i * kHist};
  if (!apply_action(L, acts[i], h)) return;
  state[i] = pack(L);
}

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      std::exit(2);                                                            \
    }                                                                          \
  } while (0)

static bool same(const Result& a, const Result& b) {
  return a.rec.x == b.rec.x && a.rec.y == b.rec.y && a.rec.z == b.rec.z && a.rec.w == b.rec.w && a.code == b.code &&
         a.legal == b.legal && a.cur == b.cur && a.term == b.term && a.r0 == b.r0 && a.ret0 == b.ret0;
}

#ifndef REPRO_NO_MAIN  // tools/w3_module_check.hip reuses the kernels above
int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 200000;
  uint4* recs;
  uint32_t* acts;
  Result *ra, *rb, *rc;
  CHECK(hipMalloc(&recs, n * sizeof(uint4)));
  CHECK(hipMalloc(&acts, n * sizeof(uint32_t)));
  CHECK(hipMalloc(&ra, n * sizeof(Result)));
  CHECK(hipMalloc(&rb, n * sizeof(Result)));
  CHECK(hipMalloc(&rc, n * sizeof(Result)));
  k_gen<<<(n + 255) / 256, 256>>>(n, recs, acts);
  k_lane<<<(n + 255) / 256, 256>>>(n, recs, acts, ra);
  k_uniform_inline<<<n, 64>>>(recs, acts, rb);
  k_uniform_call<<<n, 64>>>(recs, acts, rc);
  CHECK(hipDeviceSynchronize());
  std::vector<uint4> hr(n);
  std::vector<uint32_t> ha(n);
  std::vector<Result> a(n), b(n), c(n);
  CHECK(hipMemcpy(hr.data(), recs, n * sizeof(uint4), hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(ha.data(), acts, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(a.data(), ra, n * sizeof(Result), hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(b.data(), rb, n * sizeof(Result), hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(c.data(), rc, n * sizeof(Result), hipMemcpyDeviceToHost));
  // the product's k_slot (and stripped copies), one launch per case, on a
  // copy of the records; expected: k_lane's record
  const int m = n < 20000 ? n : 20000;
  uint4* slot_recs;
  uint8_t* slot_hist;
  coup_slot_result* slot_out;
  CHECK(hipMalloc(&slot_recs, m * sizeof(uint4)));
  CHECK(hipMalloc(&slot_hist, (size_t)m * kHist));
  CHECK(hipMalloc(&slot_out, m * sizeof(coup_slot_result)));
  std::printf("{\"slot_variants\":{");
  for (int v = 0; v < 16; ++v) {
    CHECK(hipMemcpy(slot_recs, recs, m * sizeof(uint4), hipMemcpyDeviceToDevice));
    CHECK(hipMemset(slot_hist, 0xFF, (size_t)m * kHist));
    if (v == 14) k_apply_bytehist<<<(m + 255) / 256, 256>>>(m, slot_recs, acts, slot_hist);
    for (int i = 0; v < 14 && i < m; ++i) {
      SlotArgs sa;
      sa.dst_state = slot_recs + i;
      sa.dst_hist = slot_hist + (size_t)i * kHist;
      sa.src_state = nullptr;
      sa.src_hist = nullptr;
      sa.action = (int)ha[i];
      sa.init = 0;
      sa.store = 1;
      sa.out = slot_out + i;
      sa.obs = nullptr;
      sa.done = nullptr;  // no completion flag: the launches are synchronised below
      sa.seq = 0;
      switch (v) {
        case 0: k_slot<false><<<1, 64>>>(sa); break;
        case 1: k_slot_var<0><<<1, 64>>>(sa); break;
        case 2: k_slot_var<1><<<1, 64>>>(sa); break;
        case 3: k_slot_var<2><<<1, 64>>>(sa); break;
        case 4: k_slot_var<3><<<1, 64>>>(sa); break;
        case 5: k_slot_var<4><<<1, 64>>>(sa); break;
        case 6: k_slot_var<5><<<1, 64>>>(sa); break;
        case 7: k_slot_var<6><<<1, 64>>>(sa); break;
        case 8: k_slot_var<7><<<1, 64>>>(sa); break;
        case 9: k_min<0><<<1, 64>>>(sa); break;
        case 10: k_min<1><<<1, 64>>>(sa); break;
        case 11: k_min<2><<<1, 64>>>(sa); break;
        case 12: k_min<3><<<1, 64>>>(sa); break;
        default: k_min<4><<<1, 64>>>(sa); break;
      }
    }
    if (v == 15)
      for (int i = 0; i < m; ++i) k_apply_bytehist<<<1, 256>>>(1, slot_recs + i, acts + i, slot_hist + (size_t)i * kHist);
    CHECK(hipDeviceSynchronize());
    std::vector<uint4> got(m);
    CHECK(hipMemcpy(got.data(), slot_recs, m * sizeof(uint4), hipMemcpyDeviceToHost));
    std::vector<uint8_t> gh;
    if (v >= 14) {  // the history byte too: entry at index move_number_
      gh.resize((size_t)m * kHist);
      CHECK(hipMemcpy(gh.data(), slot_hist, gh.size(), hipMemcpyDeviceToHost));
    }
    int bad = 0, first = -1;
    int by[18] = {0};
    for (int i = 0; i < m; ++i) {
      const uint4 e = a[i].rec, g = got[i];
      bool hist_bad = false;
      if (v >= 14 && (a[i].code & 1u)) {
        const uint32_t idx = (a[i].code >> 8) & 0xFFu;
        hist_bad = idx < (uint32_t)kHist && gh[(size_t)i * kHist + idx] != (uint8_t)(a[i].code >> 16);
      }
      if (hist_bad || e.x != g.x || e.y != g.y || e.z != g.z || e.w != g.w) {
        ++bad;
        by[ha[i] < 18u ? ha[i] : 0]++;
        if (first < 0) first = i;
      }
    }
    std::printf("%s\"%s\":{\"mismatch\":%d,\"by_action\":[", v ? "," : "",
                v == 0 ? "k_slot" : v == 1 ? "copy" : v == 2 ? "no_lds_hist" : v == 3 ? "no_entry_write" :
                v == 4 ? "no_slot_result" : v == 5 ? "no_unpack_after" : v == 6 ? "always_load" :
                v == 7 ? "always_load_expr" : v == 8 ? "always_apply" : v == 9 ? "min0_load_apply_store" :
                v == 10 ? "min1_if_action" : v == 11 ? "min2_if_store" : v == 12 ? "min3_slot_result" :
                v == 13 ? "min4_barriers" : v == 14 ? "apply_bytehist_batch" : "apply_bytehist_1lane", bad);
    for (int x = 0; x < 18; ++x) std::printf("%s%d", x ? "," : "", by[x]);
    std::printf("]");
    if (first >= 0)
      std::printf(",\"first\":{\"case\":%d,\"act\":%u,\"rec\":[%u,%u,%u,%u],\"want\":[%u,%u,%u,%u],\"got\":[%u,%u,%u,%u]}",
                  first, ha[first], hr[first].x, hr[first].y, hr[first].z, hr[first].w, a[first].rec.x,
                  a[first].rec.y, a[first].rec.z, a[first].rec.w, got[first].x, got[first].y, got[first].z,
                  got[first].w);
    std::printf("}");
  }
  std::printf("}}\n");
  int bad_b[18] = {0}, bad_c[18] = {0}, per[18] = {0}, shown = 0, tb = 0, tc = 0;
  for (int i = 0; i < n; ++i) {
    const uint32_t x = ha[i] < 18u ? ha[i] : 0u;
    per[x]++;
    if (!same(a[i], b[i])) {
      bad_b[x]++;
      tb++;
      if (shown < 8) {
        ++shown;
        std::printf("case %d act %u rec %08x %08x %08x %08x\n  lane:   %08x %08x %08x %08x code %08x legal %08x cur %d\n"
                    "  inline: %08x %08x %08x %08x code %08x legal %08x cur %d\n",
                    i, ha[i], hr[i].x, hr[i].y, hr[i].z, hr[i].w, a[i].rec.x, a[i].rec.y, a[i].rec.z, a[i].rec.w,
                    a[i].code, a[i].legal, a[i].cur, b[i].rec.x, b[i].rec.y, b[i].rec.z, b[i].rec.w, b[i].code,
                    b[i].legal, b[i].cur);
      }
    }
    if (!same(a[i], c[i])) {
      bad_c[x]++;
      tc++;
    }
  }
  std::printf("{\"cases\":%d,\"uniform_inline_mismatch\":%d,\"uniform_call_mismatch\":%d,\"by_action\":{", n, tb, tc);
  for (int x = 0; x < 18; ++x)
    std::printf("%s\"%d\":[%d,%d,%d]", x ? "," : "", x, per[x], bad_b[x], bad_c[x]);
  std::printf("}}\n");
  return 0;
}
#endif  // REPRO_NO_MAIN
