// split_probe.hip -- would a split c3 step (rules kernel writing a 32-byte
// observation bitmap per lane + a separate store-stream expansion kernel)
// beat the fused step kernel if consecutive steps overlap on two streams?
// Measures (1) expansion kernels alone, (2) the bare step (coup_step, no
// outputs but the record) alone, (3) both launched concurrently on two
// streams (no dependency: the overlap a pipelined step would get), and
// (4) the fused c3 step for reference.  Measurement tool only.
//   hipcc --offload-arch=gfx950 -O3 -I include -o tools/split_probe tools/split_probe.hip \
//         -L open_spiel_coup_amd -lcoup_mi355x -Wl,-rpath,'$ORIGIN/../open_spiel_coup_amd'
#include <hip/hip_runtime.h>

#include <cstdio>

#include "coup_mi355x.h"

typedef float v4f __attribute__((ext_vector_type(4)));
constexpr uint32_t kRowF4 = 49;

__device__ __forceinline__ v4f expand_f4(uint32_t word, uint32_t coins, uint32_t c) {
  const uint32_t nb = word >> (4u * (c & 7u));
  v4f v;
  v.x = (float)(nb & 1u);
  v.y = (float)((nb >> 1) & 1u);
  v.z = (float)((nb >> 2) & 1u);
  v.w = (float)((nb >> 3) & 1u);
  const float c0 = (float)(coins & 0xFFu), c1 = (float)(coins >> 8);
  v.x = c == 15u ? c0 : v.x;
  v.y = c == 15u ? c1 : v.y;
  v.z = c == 39u ? c0 : v.z;
  v.w = c == 39u ? c1 : v.w;
  return v;
}

// Persistent expansion: wave w of W handles super-chunks q = w, w + W, ...
// of S x 64 float4 (S KiB contiguous); the <= 8 lanes' bitmap words a
// super-chunk needs are loaded one super-chunk ahead (one coalesced load)
// and handed to the storing lanes with ds_bpermute.
template <int S, int POL = 1>
__global__ __launch_bounds__(256) void k_expand_pipe(const uint32_t* __restrict__ rec, v4f* __restrict__ dst,
                                                     uint32_t lanes) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t W = gridDim.x * 4u;
  const uint32_t wid = blockIdx.x * 4u + (threadIdx.x >> 6);
  const uint32_t nf4 = lanes * kRowF4;
  const uint32_t nsc = (nf4 + 64u * S - 1u) / (64u * S);
  auto load = [&](uint32_t q) -> uint32_t {
    const uint32_t o0 = (q * 64u * S) / kRowF4;
    const uint32_t o = o0 + (lane >> 3);
    return (q < nsc && o < lanes) ? rec[8u * o0 + lane] : 0u;
  };
  uint32_t q = wid;
  uint32_t nxt = load(q);
  for (; q < nsc; q += W) {
    const uint32_t cur = nxt;
    nxt = load(q + W);
    const uint32_t o0 = (q * 64u * S) / kRowF4;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const uint32_t x = (q * S + (uint32_t)s) * 64u + lane;
      const uint32_t o = x / kRowF4, c = x - o * kRowF4;
      const uint32_t base = (o - o0) * 8u;
      const uint32_t word = (uint32_t)__shfl((int)cur, (int)(base + (c >> 3)), 64);
      const uint32_t coins = (uint32_t)__shfl((int)cur, (int)(base + 7u), 64);
      if (x < nf4) {
        if (POL == 1)
          __builtin_nontemporal_store(expand_f4(word, coins, c), dst + x);
        else
          dst[x] = expand_f4(word, coins, c);
      }
    }
  }
}

// Round 4: one block per chunk of S x 256 float4 (S x 4 KiB contiguous), no
// persistence -- the grid-stride sweep's order, with the <= 22 lanes'
// bitmaps a chunk needs loaded by its first threads into LDS.  POL: 0 plain,
// 1 non-temporal, 2 sc1 buffer stores (the fused step's policy).
template <int S, int POL>
__global__ __launch_bounds__(256) void k_expand_blk(const uint32_t* __restrict__ rec, v4f* __restrict__ dst,
                                                    uint32_t lanes) {
  constexpr uint32_t kMaxLanes = (256u * S + kRowF4 - 1u) / kRowF4 + 1u;
  __shared__ uint4 bits[2 * kMaxLanes];
  const uint32_t t = threadIdx.x;
  const uint32_t nf4 = lanes * kRowF4;
  const uint32_t x0 = blockIdx.x * 256u * S;
  const uint32_t o0 = x0 / kRowF4;
  if (t < 2u * kMaxLanes && o0 + t / 2u < lanes)
    bits[t] = reinterpret_cast<const uint4*>(rec)[2u * o0 + t];
  __syncthreads();
  const uint32_t* w = reinterpret_cast<const uint32_t*>(bits);
  __amdgpu_buffer_rsrc_t rsrc;
  if (POL == 2) rsrc = __builtin_amdgcn_make_buffer_rsrc(dst, (short)0, (int)(nf4 * 16u), 0x00020000);
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const uint32_t x = x0 + (uint32_t)s * 256u + t;
    const uint32_t o = x / kRowF4, c = x - o * kRowF4;
    const uint32_t base = (o - o0) * 8u;
    const v4f v = expand_f4(w[base + (c >> 3)], w[base + 7u], c);
    if (POL == 2) {
      typedef uint32_t v4u __attribute__((ext_vector_type(4)));
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), rsrc, (int)(16u * x), 0, 16);
    } else if (x < nf4) {
      if (POL == 1)
        __builtin_nontemporal_store(v, dst + x);
      else
        dst[x] = v;
    }
  }
}

#define CK(x)                                                    \
  do {                                                           \
    hipError_t e = (x);                                          \
    if (e != hipSuccess) {                                       \
      std::printf("%s: %s\n", #x, hipGetErrorString(e));         \
      return 1;                                                  \
    }                                                            \
  } while (0)
#define CC(x)                                                    \
  do {                                                           \
    int r = (x);                                                 \
    if (r != 0) {                                                \
      std::printf("%s: %d %s\n", #x, r, coup_last_error());      \
      return 1;                                                  \
    }                                                            \
  } while (0)

int main() {
  const uint32_t lanes = 1u << 20;
  const size_t bytes = (size_t)lanes * 784;
  v4f* obs;
  uint32_t* rec;
  CK(hipMalloc(&obs, bytes));
  CK(hipMalloc(&rec, (size_t)lanes * 32));
  CK(hipMemset(rec, 0x5A, (size_t)lanes * 32));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t e0, e1, j;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&j));
  const int reps = 50;
  // time `reps` launches on s1 (f receives the rep index); s2 work joins s1
  auto timed = [&](const char* name, auto f) -> int {
    for (int w = 0; w < 5; ++w) f(w);
    CK(hipStreamSynchronize(s1));
    CK(hipStreamSynchronize(s2));
    CK(hipEventRecord(e0, s1));
    CK(hipStreamWaitEvent(s2, e0, 0));
    for (int r = 0; r < reps; ++r) f(r);
    CK(hipEventRecord(j, s2));
    CK(hipStreamWaitEvent(s1, j, 0));
    CK(hipEventRecord(e1, s1));
    CK(hipEventSynchronize(e1));
    CK(hipGetLastError());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("{\"what\": \"%s\", \"us_per_rep\": %.2f}\n", name, ms * 1e3 / reps);
    std::fflush(stdout);
    return 0;
  };
  char name[96];
  for (int grid : {1024}) {
    std::snprintf(name, sizeof name, "expand_pipe_S1_nt_g%d", grid);
    timed(name, [&](int) { k_expand_pipe<1, 1><<<grid, 256, 0, s1>>>(rec, obs, lanes); });
    std::snprintf(name, sizeof name, "expand_pipe_S1_plain_g%d", grid);
    timed(name, [&](int) { k_expand_pipe<1, 0><<<grid, 256, 0, s1>>>(rec, obs, lanes); });
    std::snprintf(name, sizeof name, "expand_pipe_S4_plain_g%d", grid);
    timed(name, [&](int) { k_expand_pipe<4, 0><<<grid, 256, 0, s1>>>(rec, obs, lanes); });
  }
  const uint32_t nf4 = lanes * kRowF4;
  auto blocks = [&](int S) { return (unsigned)((nf4 + 256u * S - 1u) / (256u * S)); };
  timed("expand_blk_S1_nt", [&](int) { k_expand_blk<1, 1><<<blocks(1), 256, 0, s1>>>(rec, obs, lanes); });
  timed("expand_blk_S1_sc1", [&](int) { k_expand_blk<1, 2><<<blocks(1), 256, 0, s1>>>(rec, obs, lanes); });
  timed("expand_blk_S4_nt", [&](int) { k_expand_blk<4, 1><<<blocks(4), 256, 0, s1>>>(rec, obs, lanes); });
  timed("expand_blk_S4_sc1", [&](int) { k_expand_blk<4, 2><<<blocks(4), 256, 0, s1>>>(rec, obs, lanes); });
  timed("expand_blk_S4_plain", [&](int) { k_expand_blk<4, 0><<<blocks(4), 256, 0, s1>>>(rec, obs, lanes); });
  coup_env* bare;
  coup_env* fused;
  CC(coup_create(lanes, 1, 0, COUP_FLAG_AUTO_RESET, &bare));
  CC(coup_create(lanes, 1, 0, COUP_FLAG_AUTO_RESET, &fused));
  CC(coup_set_stream(bare, s1));
  CC(coup_set_stream(fused, s1));
  CC(coup_rollout(bare, 256, nullptr));
  CC(coup_rollout(fused, 256, nullptr));
  coup_step_outputs none{};
  coup_step_outputs with_obs{};
  with_obs.obs = reinterpret_cast<float*>(obs);
  timed("bare_step", [&](int) { coup_step(bare, nullptr, &none); });
  timed("fused_c3_step", [&](int) { coup_step(fused, nullptr, &with_obs); });
  for (int grid : {512, 1024}) {
    std::snprintf(name, sizeof name, "overlap_bare_step+expand_S1_plain_g%d", grid);
    timed(name, [&](int) {
      coup_step(bare, nullptr, &none);
      k_expand_pipe<1, 0><<<grid, 256, 0, s2>>>(rec, obs, lanes);
    });
  }
  timed("overlap_bare_step+expand_blk_S4_sc1", [&](int) {
    coup_step(bare, nullptr, &none);
    k_expand_blk<4, 2><<<blocks(4), 256, 0, s2>>>(rec, obs, lanes);
  });
  timed("overlap_bare_step+expand_blk_S1_nt", [&](int) {
    coup_step(bare, nullptr, &none);
    k_expand_blk<1, 1><<<blocks(1), 256, 0, s2>>>(rec, obs, lanes);
  });
  // the chunked split step: the batch as C envs of 2^20 / C lanes (the rules
  // kernel of chunk c), each followed on s2 by the expansion of its obs
  // chunk, and s1 waiting for the last expansion before the next step (a
  // step's outputs complete on s1: no overlap across steps)
  for (int C : {1, 2, 4, 8}) {
    coup_env* ch[8];
    hipEvent_t ev[8], done;
    CK(hipEventCreateWithFlags(&done, hipEventDisableTiming));
    for (int c = 0; c < C; ++c) {
      CC(coup_create(lanes / C, 1, (int64_t)c * (lanes / C), COUP_FLAG_AUTO_RESET, &ch[c]));
      CC(coup_set_stream(ch[c], s1));
      CC(coup_rollout(ch[c], 256, nullptr));
      CK(hipEventCreateWithFlags(&ev[c], hipEventDisableTiming));
    }
    const uint32_t cl = lanes / C, cf4 = cl * kRowF4;
    const unsigned cb = (unsigned)((cf4 + 255u) / 256u);
    std::snprintf(name, sizeof name, "chunked_split_C%d_bare_then_expand_blk_S1_nt", C);
    timed(name, [&](int) {
      for (int c = 0; c < C; ++c) {
        coup_step(ch[c], nullptr, &none);
        hipEventRecord(ev[c], s1);
        hipStreamWaitEvent(s2, ev[c], 0);
        k_expand_blk<1, 1><<<cb, 256, 0, s2>>>(rec + (size_t)c * cl * 8u, obs + (size_t)c * cf4, cl);
      }
      hipEventRecord(done, s2);
      hipStreamWaitEvent(s1, done, 0);
    });
    for (int c = 0; c < C; ++c) {
      CC(coup_destroy(ch[c]));
      CK(hipEventDestroy(ev[c]));
    }
    CK(hipEventDestroy(done));
  }
  // the split step on ONE stream (no events): the bare step, then the sweep
  // expansion of the whole batch
  timed("seq_bare_then_expand_blk_S1_nt", [&](int) {
    coup_step(bare, nullptr, &none);
    k_expand_blk<1, 1><<<blocks(1), 256, 0, s1>>>(rec, obs, lanes);
  });
  timed("fused_c3_step_again", [&](int) { coup_step(fused, nullptr, &with_obs); });
  CC(coup_destroy(bare));
  CC(coup_destroy(fused));
  return 0;
}
