// info_prefix_repro.hip -- standalone reproducer of round 4's second
// section-12 sighting: the split InformationStateTensor
// writer k_info_sweep, as first written, got the observer one-hot bits of a
// few lanes in 1000 wrong while its per-lane prefix words were stored by
// info_prefix_to_lds in its uint2 form (two <2 x i32> LDS stores).  The
// shipped writer stores the words as 32-bit values (one observer row per
// thread), and info_prefix_to_lds itself now does too.  Investigation tool,
// not product code; tests/test_gpu_codegen_hazard.py runs it.
//
//   hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -std=c++17 -I include \
//       -I open_spiel_coup_amd/csrc tools/info_prefix_repro.hip -o build/info_prefix_repro
//   build/info_prefix_repro [lanes]
//
// 1. k_gen: lane i plays a random legal game prefix (decisions and deals,
//    some to the end) from NewInitialState with its own xorshift stream,
//    keeping the history bytes.
// 2. k_ref: the InformationStateTensor of every lane, one thread per float4
//    (k_info_elems' form: the decode of the GPU suite's oracle-checked
//    writers), prefix words as 32-bit values.
// 3. k_sweep_uint2<T, S>: round 4's first k_info_sweep, verbatim in shape:
//    the block's first kLanes threads store a lane's 6 prefix words with
//    two uint2 stores, then every thread decodes its float4s.
// 4. k_sweep_rows<T, S>: the shipped form (one observer row per thread,
//    32-bit stores).
// Prints one JSON line per kernel: lanes whose tensor differs from k_ref.
//
//   build/info_prefix_repro [lanes] [module.co ...]
//
// With code objects (tools/info_modules.sh: this file's device IR through
// llc at chosen settings), each module's k_sweep_uint2<512, 2> and
// k_sweep_rows<512, 2> are loaded (hipModuleLoad) and checked against k_ref
// the same way, one JSON line per module and kernel (INFO_REPRO_DYN_LDS:
// launched with that much extra dynamic LDS per block).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "coup_lane.h"
#include "coup_tensor.h"

using namespace coup;

__device__ __forceinline__ uint32_t xs(uint32_t& s) {
  s ^= s << 13;
  s ^= s >> 17;
  s ^= s << 5;
  return s;
}

// history entries straight to the lane's 96 bytes (the generator only)
struct GlobalHistory {
  uint8_t* h;
  __device__ void record(uint32_t idx, uint32_t entry) {
    if (idx < (uint32_t)kHist) h[idx] = (uint8_t)entry;
  }
};

__global__ void k_gen(int n, uint4* recs, uint8_t* hist, uint32_t* terminal) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t s = 0x9E3779B9u * (uint32_t)(i + 1) | 1u;
  for (int k = 0; k < kHist; ++k) hist[(size_t)i * kHist + k] = 0xFFu;
  GlobalHistory H{hist + (size_t)i * kHist};
  Lane L = initial_lane(0u);
  const uint32_t steps = xs(s) % 80u;
  for (uint32_t k = 0; k < steps; ++k) {
    const uint32_t m = legal_mask(L) & 0x3FFFFu;  // chance outcomes or decisions; 0 when terminal
    if (m == 0u) break;
    uint32_t mm = m, idx = xs(s) % (uint32_t)__popc(m);
    for (uint32_t j = 0; j < idx; ++j) mm &= mm - 1u;
    if (!apply_action(L, (uint32_t)__builtin_ctz(mm), H)) break;
  }
  recs[i] = pack(L);
  if (is_terminal(L)) atomicAdd(terminal, 1u);
}

// the reference: one thread per float4, 32-bit prefix words
__global__ __launch_bounds__(256) void k_ref(const uint4* __restrict__ state, const uint8_t* __restrict__ hist,
                                             int64_t n, float* __restrict__ info) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= n * kInfoF4) return;
  const int64_t row = g / kInfoF4;
  const uint32_t c = (uint32_t)(g - row * kInfoF4);
  uint32_t pre[kPreWords];
  info_prefix_to_lds(unpack(state[row]), pre);
  reinterpret_cast<float4*>(info)[g] = info_f4(pre, hist + row * kHist, c);
}

// round 4's first form of the prefix words: two uint2 (<2 x i32>) stores
__device__ __forceinline__ void prefix_uint2(const Lane& L, uint32_t* __restrict__ pre) {
  const bool term = is_terminal(L);
  uint64_t a_lo, a_hi, b_lo, b_hi;
  obs_row_bits<0>(L, term, a_lo, a_hi);
  obs_row_bits<1>(L, term, b_lo, b_hi);
  const uint64_t m62 = (1ull << 62) - 1ull;
  reinterpret_cast<uint2*>(pre)[0] = make_uint2((uint32_t)a_lo, (uint32_t)((a_lo & m62) >> 32));
  reinterpret_cast<uint2*>(pre)[1] = make_uint2((uint32_t)b_lo, (uint32_t)((b_lo & m62) >> 32));
  pre[4] = L.c0 | (L.c1 << 8) | (L.move << 16);
  pre[5] = 0;
}

template <int T, int S>
__device__ __forceinline__ void sweep_store(float* info, const uint32_t* pre, const uint4* h4, int64_t x0,
                                            int64_t o0, int64_t n) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  const uint32_t t = threadIdx.x;
  const int64_t nf4 = n * kInfoF4;
  const uint32_t rel0 = (uint32_t)(x0 - o0 * kInfoF4);
  const uint8_t* hb = reinterpret_cast<const uint8_t*>(h4);
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const int64_t x = x0 + j * T + t;
    if (x >= nf4) break;
    const uint32_t rel = rel0 + (uint32_t)(j * T) + t;
    const uint32_t o = rel / (uint32_t)kInfoF4, c = rel - o * (uint32_t)kInfoF4;
    const float4 f = info_f4(pre + kPreWords * o, hb + kHist * o, c);
    v4f v;
    v.x = f.x;
    v.y = f.y;
    v.z = f.z;
    v.w = f.w;
    __builtin_nontemporal_store(v, reinterpret_cast<v4f*>(info) + x);
  }
}

// round 4's first k_info_sweep (the declarations as they were: pre[] with
// no alignment attribute, then the history uint4s)
template <int T, int S>
__global__ __launch_bounds__(T) void k_sweep_uint2(const uint4* __restrict__ state, const uint8_t* __restrict__ hist,
                                                   float* __restrict__ info, int64_t n) {
  constexpr uint32_t kLanes = ((uint32_t)(T * S) + (uint32_t)kInfoF4 - 1u) / (uint32_t)kInfoF4 + 1u;
  constexpr uint32_t kHistU4 = (uint32_t)kHist / 16u;
  __shared__ uint32_t pre[kLanes * kPreWords];
  __shared__ uint4 h4[kLanes * kHistU4];
  const uint32_t t = threadIdx.x;
  const int64_t x0 = (int64_t)blockIdx.x * (T * S);
  const int64_t o0 = x0 / kInfoF4;
  if (t < kLanes && o0 + t < n) prefix_uint2(unpack(state[o0 + t]), pre + kPreWords * t);
  if (t < kLanes * kHistU4 && o0 + t / kHistU4 < n) h4[t] = reinterpret_cast<const uint4*>(hist)[o0 * kHistU4 + t];
  __syncthreads();
  sweep_store<T, S>(info, pre, h4, x0, o0, n);
}

// the shipped form: one observer row per thread, 32-bit stores
template <int T, int S>
__global__ __launch_bounds__(T) void k_sweep_rows(const uint4* __restrict__ state, const uint8_t* __restrict__ hist,
                                                  float* __restrict__ info, int64_t n) {
  constexpr uint32_t kLanes = ((uint32_t)(T * S) + (uint32_t)kInfoF4 - 1u) / (uint32_t)kInfoF4 + 1u;
  constexpr uint32_t kHistU4 = (uint32_t)kHist / 16u;
  __shared__ __attribute__((aligned(16))) uint32_t pre[kLanes * kPreWords];
  __shared__ uint4 h4[kLanes * kHistU4];
  const uint32_t t = threadIdx.x;
  const int64_t x0 = (int64_t)blockIdx.x * (T * S);
  const int64_t o0 = x0 / kInfoF4;
  if (t < 2u * kLanes && o0 + (t >> 1) < n) {
    const Lane L = unpack(state[o0 + (t >> 1)]);
    const uint32_t p = t & 1u;
    uint64_t lo, hi;
    obs_row_bits_rt(L, is_terminal(L), p, lo, hi);
    const uint64_t m62 = (1ull << 62) - 1ull;
    uint32_t* w = pre + kPreWords * (t >> 1);
    w[2u * p] = (uint32_t)lo;
    w[2u * p + 1u] = (uint32_t)((lo & m62) >> 32);
    if (p == 0u) {
      w[4] = L.c0 | (L.c1 << 8) | (L.move << 16);
      w[5] = 0u;
    }
  }
  if (t < kLanes * kHistU4 && o0 + t / kHistU4 < n) h4[t] = reinterpret_cast<const uint4*>(hist)[o0 * kHistU4 + t];
  __syncthreads();
  sweep_store<T, S>(info, pre, h4, x0, o0, n);
}

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      std::exit(2);                                                                  \
    }                                                                                \
  } while (0)

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 100000;
  if (n <= 0 || n > (1 << 22)) return 2;
  uint4* recs;
  uint8_t* hist;
  float *ref, *out;
  uint32_t* d_term;
  const size_t fl = (size_t)n * kInfoF4 * 4;
  CHECK(hipMalloc(&recs, (size_t)n * sizeof(uint4)));
  CHECK(hipMalloc(&hist, (size_t)n * kHist));
  CHECK(hipMalloc(&ref, fl * sizeof(float)));
  CHECK(hipMalloc(&out, fl * sizeof(float)));
  CHECK(hipMalloc(&d_term, sizeof(uint32_t)));
  CHECK(hipMemset(d_term, 0, sizeof(uint32_t)));
  k_gen<<<(n + 255) / 256, 256>>>(n, recs, hist, d_term);
  CHECK(hipGetLastError());
  const int64_t nf4 = (int64_t)n * kInfoF4;
  k_ref<<<(unsigned)((nf4 + 255) / 256), 256>>>(recs, hist, n, ref);
  CHECK(hipGetLastError());
  std::vector<float> h_ref(fl), h_out(fl);
  CHECK(hipMemcpy(h_ref.data(), ref, fl * sizeof(float), hipMemcpyDeviceToHost));
  uint32_t terminal = 0;
  CHECK(hipMemcpy(&terminal, d_term, sizeof(uint32_t), hipMemcpyDeviceToHost));
  auto compare = [&](const char* name) {
    CHECK(hipMemcpy(h_out.data(), out, fl * sizeof(float), hipMemcpyDeviceToHost));
    int bad = 0, first = -1, first_f = -1;
    for (int i = 0; i < n; ++i) {
      const float* a = h_ref.data() + (size_t)i * kInfoF4 * 4;
      const float* b = h_out.data() + (size_t)i * kInfoF4 * 4;
      if (std::memcmp(a, b, (size_t)kInfoF4 * 16) != 0) {
        if (first < 0) {
          first = i;
          for (int f = 0; f < kInfoF4 * 4; ++f)
            if (a[f] != b[f]) {
              first_f = f;
              break;
            }
        }
        ++bad;
      }
    }
    std::printf("{\"kernel\": \"%s\", \"lanes\": %d, \"terminal_lanes\": %d, \"mismatching_lanes\": %d, "
                "\"first_lane\": %d, \"first_float\": %d}\n",
                name, n, (int)terminal, bad, first, first_f);
  };
  auto run = [&](auto kern, int T, int S, const char* name) {
    CHECK(hipMemset(out, 0xFF, fl * sizeof(float)));
    kern<<<(unsigned)((nf4 + T * S - 1) / (T * S)), T>>>(recs, hist, out, n);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    compare(name);
  };
  if (argc > 2) {  // code objects: the modules' kernels instead of this binary's
    for (int m = 2; m < argc; ++m) {
      hipModule_t mod;
      CHECK(hipModuleLoad(&mod, argv[m]));
      const char* names[2] = {"_Z13k_sweep_uint2ILi512ELi2EEvPK15HIP_vector_typeIjLj4EEPKhPfl",
                              "_Z12k_sweep_rowsILi512ELi2EEvPK15HIP_vector_typeIjLj4EEPKhPfl"};
      for (const char* kn : names) {
        hipFunction_t fn;
        if (hipModuleGetFunction(&fn, mod, kn) != hipSuccess) continue;
        CHECK(hipMemset(out, 0xFF, fl * sizeof(float)));
        int64_t n64 = n;
        void* args[] = {&recs, &hist, &out, &n64};
        // INFO_REPRO_DYN_LDS: extra dynamic LDS per block (fewer blocks per CU)
        const char* dl = std::getenv("INFO_REPRO_DYN_LDS");
        const unsigned dyn = dl ? (unsigned)std::atoi(dl) : 0u;
        CHECK(hipModuleLaunchKernel(fn, (unsigned)((nf4 + 1023) / 1024), 1, 1, 512, 1, 1, dyn, nullptr, args, nullptr));
        CHECK(hipDeviceSynchronize());
        std::string label = std::string(argv[m]) + " " + (std::strstr(kn, "uint2") ? "uint2" : "rows");
        compare(label.c_str());
      }
      CHECK(hipModuleUnload(mod));
    }
    return 0;
  }
  run(k_sweep_rows<1024, 2>, 1024, 2, "k_sweep_rows<1024, 2> (shipped form)");
  run(k_sweep_rows<512, 2>, 512, 2, "k_sweep_rows<512, 2>");
  run(k_sweep_uint2<512, 2>, 512, 2, "k_sweep_uint2<512, 2> (round 4's first form)");
  run(k_sweep_uint2<1024, 2>, 1024, 2, "k_sweep_uint2<1024, 2>");
  run(k_sweep_uint2<256, 2>, 256, 2, "k_sweep_uint2<256, 2>");
  CHECK(hipFree(recs));
  CHECK(hipFree(hist));
  CHECK(hipFree(ref));
  CHECK(hipFree(out));
  CHECK(hipFree(d_term));
  return 0;
}
