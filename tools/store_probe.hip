// store_probe.hip -- store-order probe for the ObservationTensor write-out
// (DESIGN.md section 5).  Every variant writes the same 784 MiB buffer
// ([2^20][2][98] fp32) with no compute, under the step kernel's constraint
// that a wave (or block) owns the rows of its own lanes; only the order,
// the cache policy, the block size and the block -> chunk mapping change.
// Measurement tool only.
//   hipcc --offload-arch=gfx950 -O3 -o tools/store_probe tools/store_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float v4f __attribute__((ext_vector_type(4)));

constexpr int kRowF4 = 49;              // float4 per lane (2 x 98 floats)
constexpr int kWaveF4 = 64 * kRowF4;    // 3136 float4 = 50,176 B per wave

// cache policy of one 16-byte store: 0 plain, 1 nt, 2 sc1, 3 sc0 sc1, 4 sc0 sc1 nt
template <int POL>
__device__ __forceinline__ void st(v4f* p, v4f v) {
  if (POL == 0) {
    *p = v;
  } else if (POL == 1) {
    __builtin_nontemporal_store(v, p);
  } else if (POL == 2) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  } else if (POL == 3) {
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
  } else {
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
  }
}

// XCD-aware chunk id: blocks are dealt round-robin over the 8 XCDs, so
// block b runs on XCD b % 8; give XCD x the contiguous run of chunks
// [x * G/8, (x+1) * G/8) in dispatch order.
// With S < G/8, XCD x owns every 8th run of S consecutive chunks instead.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t G, uint32_t S) {
  if (S == 0u) S = G / 8u;
  const uint32_t r = b / 8u;  // rank of the block among its XCD's blocks
  return (r / S) * 8u * S + (b % 8u) * S + r % S;
}

// Wave chunks: each wave writes its own 50 KiB as 49 x 1 KiB instructions.
// ROT: wave w starts at iteration w % 49 (spreads concurrent writes over rows).
template <int T, int POL, bool XCD, bool ROT>
__global__ __launch_bounds__(T) void k_wave_chunks(v4f* __restrict__ dst, uint32_t waves, uint32_t S) {
  const v4f z = {0.f, 1.f, 0.f, 0.f};
  const uint32_t b = XCD ? xcd_remap(blockIdx.x, gridDim.x, S) : blockIdx.x;
  const uint32_t wave = b * (T / 64) + threadIdx.x / 64;
  const uint32_t lane = threadIdx.x & 63u;
  if (wave >= waves) return;
  v4f* base = dst + (size_t)wave * kWaveF4;
  const uint32_t r = ROT ? wave % kRowF4 : 0u;
#pragma unroll 7
  for (uint32_t j = 0; j < (uint32_t)kRowF4; ++j) {
    uint32_t jj = j + r;
    jj = jj >= (uint32_t)kRowF4 ? jj - kRowF4 : jj;
    st<POL>(base + 64u * jj + lane, z);
  }
}

// Block chunks: the block's T lanes own T x 784 B; iteration j writes T float4.
template <int T, int POL, bool XCD>
__global__ __launch_bounds__(T) void k_block_chunks(v4f* __restrict__ dst, uint32_t S) {
  const v4f z = {0.f, 1.f, 0.f, 0.f};
  const uint32_t b = XCD ? xcd_remap(blockIdx.x, gridDim.x, S) : blockIdx.x;
  v4f* base = dst + (size_t)b * T * kRowF4;
#pragma unroll 7
  for (uint32_t j = 0; j < (uint32_t)kRowF4; ++j) st<POL>(base + T * j + threadIdx.x, z);
}


// Unit-strided lane ownership (a narrow chip-wide write window under lane
// ownership): a block owns J units of U lanes; unit j of block b' lies at
// global unit (s*J + j)*R + r, with s = b' / R, r = b' % R, so at sub-step j
// the R co-resident blocks write R adjacent units (R*U*784 B) and the window
// sweeps the buffer.  COOP: the block stores its J units in j order
// (256 threads per iteration); otherwise wave w stores units [w*J/4, (w+1)*J/4).
// XR: r is remapped so that each XCD (b' % 8) owns a contiguous run of units.
template <int U, int J, bool COOP, bool XR>
__global__ __launch_bounds__(256) void k_unit_strided(v4f* __restrict__ dst, uint32_t R) {
  const v4f z = {0.f, 1.f, 0.f, 0.f};
  constexpr uint32_t kUnitF4 = U * kRowF4;
  const uint32_t s = blockIdx.x / R, r0 = blockIdx.x % R;
  const uint32_t r = XR ? (r0 % 8u) * (R / 8u) + r0 / 8u : r0;
  if (COOP) {
    constexpr uint32_t tot = J * kUnitF4;
    for (uint32_t q = threadIdx.x; q < tot; q += 256u) {
      const uint32_t j = q / kUnitF4, f = q - j * kUnitF4;
      st<0>(dst + ((size_t)(s * J + j) * R + r) * kUnitF4 + f, z);
    }
  } else {
    constexpr uint32_t per = J / 4, tot = per * kUnitF4;
    const uint32_t w = threadIdx.x / 64u;
    for (uint32_t q = threadIdx.x & 63u; q < tot; q += 64u) {
      const uint32_t j = w * per + q / kUnitF4, f = q % kUnitF4;
      st<0>(dst + ((size_t)(s * J + j) * R + r) * kUnitF4 + f, z);
    }
  }
}

// Unconstrained reference: grid-stride float4 sweep.
template <int POL>
__global__ __launch_bounds__(256) void k_sweep(v4f* __restrict__ dst, size_t n) {
  const v4f z = {0.f, 1.f, 0.f, 0.f};
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) st<POL>(dst + i, z);
}

// Expansion of 32-byte per-lane bitmap records (7 words of the 196-bit
// observation string + coins, as the step kernel stages them in LDS) into
// the [B][2][98] fp32 tensor in sweep order: thread t of the grid writes
// float4 x = t, t + stride, ...  (a split design: the step kernel writes the
// records, this kernel is a pure store stream).
template <int PER>
__global__ __launch_bounds__(256) void k_expand(const uint32_t* __restrict__ rec, v4f* __restrict__ dst, uint32_t nf4) {
  const uint32_t stride = gridDim.x * 256u;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const uint32_t x = blockIdx.x * 256u + threadIdx.x + (uint32_t)k * stride;
    if (x >= nf4) return;
    const uint32_t o = x / (uint32_t)kRowF4;
    const uint32_t c = x - o * (uint32_t)kRowF4;
    const uint32_t word = rec[8u * o + (c >> 3)];
    const uint32_t coins = rec[8u * o + 7u];
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
    dst[x] = v;
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

int main() {
  const size_t lanes = (size_t)1 << 20;
  const size_t bytes = lanes * 784;
  const size_t n = bytes / 16;
  const uint32_t waves = (uint32_t)(lanes / 64);
  v4f* a;
  CK(hipMalloc(&a, bytes));
  CK(hipMemset(a, 0, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 20;
  auto timed = [&](const char* name, int grid, int block, auto launch) -> int {
    for (int w = 0; w < 3; ++w) launch();
    CK(hipGetLastError());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("{\"kernel\": \"%s\", \"grid\": %d, \"block\": %d, \"bytes\": %.0f, \"us\": %.2f, \"GBps\": %.1f}\n",
                name, grid, block, (double)bytes, ms * 1e3 / reps, (double)bytes / (ms * 1e-3 / reps) / 1e9);
    std::fflush(stdout);
    return 0;
  };
  char name[96];
#define WAVE(T, POL, XCD, S)                                                                      \
  std::snprintf(name, sizeof name, "wave_t%d_pol%d_xcd%d_S%d", T, POL, (int)XCD, S);              \
  timed(name, (int)(waves / (T / 64)), T,                                                        \
        [&] { k_wave_chunks<T, POL, XCD, false><<<waves / (T / 64), T>>>(a, waves, S); })
  WAVE(256, 1, false, 0);
  WAVE(256, 0, false, 0);
  WAVE(256, 0, true, 0);
  WAVE(256, 2, true, 0);
  WAVE(256, 3, true, 0);
  WAVE(64, 0, true, 0);
  WAVE(64, 2, true, 0);
  WAVE(128, 0, true, 0);
  WAVE(512, 0, true, 0);
  WAVE(1024, 0, true, 0);
  for (int S : {1, 2, 4, 8, 16, 32, 64, 128, 256}) {
    WAVE(256, 0, true, S);
  }
  for (int S : {4, 16, 64, 256, 1024}) {
    WAVE(64, 0, true, S);
  }
  for (uint32_t R : {256u, 512u, 1024u, 2048u, 4096u}) {
    const int g = (int)(lanes / 256);
    std::snprintf(name, sizeof name, "unit8_coop_R%u", R);
    timed(name, g, 256, [&] { k_unit_strided<8, 32, true, false><<<g, 256>>>(a, R); });
    std::snprintf(name, sizeof name, "unit8_wave_R%u", R);
    timed(name, g, 256, [&] { k_unit_strided<8, 32, false, false><<<g, 256>>>(a, R); });
    std::snprintf(name, sizeof name, "unit8_coop_xr_R%u", R);
    timed(name, g, 256, [&] { k_unit_strided<8, 32, true, true><<<g, 256>>>(a, R); });
    std::snprintf(name, sizeof name, "unit4_coop_R%u", R);
    timed(name, g, 256, [&] { k_unit_strided<4, 64, true, false><<<g, 256>>>(a, R); });
    std::snprintf(name, sizeof name, "unit16_coop_R%u", R);
    timed(name, g, 256, [&] { k_unit_strided<16, 16, true, false><<<g, 256>>>(a, R); });
  }
  WAVE(256, 0, true, 0);
#undef WAVE
#define BLOCK(T, POL, XCD, S)                                                                     \
  std::snprintf(name, sizeof name, "block_t%d_pol%d_xcd%d_S%d", T, POL, (int)XCD, S);             \
  timed(name, (int)(lanes / T), T, [&] { k_block_chunks<T, POL, XCD><<<lanes / T, T>>>(a, S); })
  BLOCK(256, 0, true, 0);
  BLOCK(256, 2, true, 0);
  BLOCK(1024, 0, true, 0);
  BLOCK(1024, 2, true, 0);
  BLOCK(1024, 2, false, 0);
  BLOCK(512, 0, true, 0);
#undef BLOCK
  {
    uint32_t* rec;
    CK(hipMalloc(&rec, lanes * 32));
    CK(hipMemset(rec, 0x5A, lanes * 32));
    const uint32_t nf4 = (uint32_t)n;
    const int g1 = (int)((n + 255) / 256), g2 = (int)((n + 511) / 512), g4 = (int)((n + 1023) / 1024);
    timed("expand_per1", g1, 256, [&] { k_expand<1><<<g1, 256>>>(rec, a, nf4); });
    timed("expand_per2", g2, 256, [&] { k_expand<2><<<g2, 256>>>(rec, a, nf4); });
    timed("expand_per4", g4, 256, [&] { k_expand<4><<<g4, 256>>>(rec, a, nf4); });
    CK(hipFree(rec));
  }
  for (int grid : {65536, 131072}) {
    timed("sweep_plain", grid, 256, [&] { k_sweep<0><<<grid, 256>>>(a, n); });
    timed("sweep_nt", grid, 256, [&] { k_sweep<1><<<grid, 256>>>(a, n); });
  }
  CK(hipFree(a));
  return 0;
}
