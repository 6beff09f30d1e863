// hbm_probe.hip -- measured HBM ceilings for the roofline discussion
// (DESIGN.md section 5): a pure streaming write of the obs buffer size, the
// same with non-temporal stores, and a float4 copy.  Measurement tool only.
//   hipcc --offload-arch=gfx950 -O3 -o tools/hbm_probe tools/hbm_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float v4f __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void k_write(v4f* __restrict__ dst, size_t n) {
  const v4f z = {0.f, 1.f, 0.f, 0.f};
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    if (NT)
      __builtin_nontemporal_store(z, dst + i);
    else
      dst[i] = z;
  }
}

// The step kernel's store pattern with no compute: every wave writes its own
// 50,176-byte chunk as 49 consecutive 1 KiB store instructions.
__global__ __launch_bounds__(256) void k_write_chunks(v4f* __restrict__ dst, size_t n) {
  const v4f z = {0.f, 1.f, 0.f, 0.f};
  const size_t wave = ((size_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const size_t lane = threadIdx.x & 63;
  v4f* base = dst + wave * 3136;
  if ((wave + 1) * 3136 > n) return;
  for (int j = 0; j < 49; ++j) __builtin_nontemporal_store(z, base + 64 * j + lane);
}

// Block-cooperative chunks: a block of T threads owns T rows (T x 784 B) and
// iteration j writes T consecutive float4 (T x 16 B contiguous).
template <int T, bool NT>
__global__ __launch_bounds__(T) void k_write_block_chunks(v4f* __restrict__ dst, size_t n) {
  const v4f z = {0.f, 1.f, 0.f, 0.f};
  v4f* base = dst + (size_t)blockIdx.x * T * 49;
  if (((size_t)blockIdx.x + 1) * T * 49 > n) return;
  for (int j = 0; j < 49; ++j) {
    if (NT)
      __builtin_nontemporal_store(z, base + T * j + threadIdx.x);
    else
      base[T * j + threadIdx.x] = z;
  }
}

__global__ __launch_bounds__(256) void k_copy(v4f* __restrict__ dst, const v4f* __restrict__ src, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) dst[i] = src[i];
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      std::printf("%s: %s\n", #x, hipGetErrorString(e));                   \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main() {
  const size_t bytes = (size_t)784 << 20;  // 2^20 lanes x 784 B
  const size_t n = bytes / 16;
  v4f *a, *b;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMemset(a, 0, bytes));
  CK(hipMemset(b, 0, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 20;
  for (int grid : {2048, 4096, 16384}) {
    for (int kind = 0; kind < 3; ++kind) {
      for (int w = 0; w < 3; ++w) {
        if (kind == 0) k_write<false><<<grid, 256>>>(a, n);
        if (kind == 1) k_write<true><<<grid, 256>>>(a, n);
        if (kind == 2) k_copy<<<grid, 256>>>(a, b, n);
      }
      CK(hipEventRecord(e0));
      for (int r = 0; r < reps; ++r) {
        if (kind == 0) k_write<false><<<grid, 256>>>(a, n);
        if (kind == 1) k_write<true><<<grid, 256>>>(a, n);
        if (kind == 2) k_copy<<<grid, 256>>>(a, b, n);
      }
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double moved = (kind == 2 ? 2.0 : 1.0) * (double)bytes;
      const char* names[3] = {"write", "write_nt", "copy"};
      std::printf("{\"kernel\": \"%s\", \"grid\": %d, \"bytes\": %.0f, \"us\": %.2f, \"GBps\": %.1f}\n", names[kind],
                  grid, moved, ms * 1e3 / reps, moved / (ms * 1e-3 / reps) / 1e9);
    }
  }
  {
    const int grid = (int)(n / 3136 / 4);  // 4 waves per block, one chunk per wave
    for (int w = 0; w < 3; ++w) k_write_chunks<<<grid, 256>>>(a, n);
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) k_write_chunks<<<grid, 256>>>(a, n);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("{\"kernel\": \"write_chunks_nt\", \"grid\": %d, \"bytes\": %.0f, \"us\": %.2f, \"GBps\": %.1f}\n", grid,
                (double)bytes, ms * 1e3 / reps, (double)bytes / (ms * 1e-3 / reps) / 1e9);
  }
  auto timed = [&](const char* name, int grid, auto launch) -> int {
    for (int w = 0; w < 3; ++w) launch();
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("{\"kernel\": \"%s\", \"grid\": %d, \"bytes\": %.0f, \"us\": %.2f, \"GBps\": %.1f}\n", name, grid,
                (double)bytes, ms * 1e3 / reps, (double)bytes / (ms * 1e-3 / reps) / 1e9);
    return 0;
  };
  {
    const int g256 = (int)(n / (256 * 49)), g512 = (int)(n / (512 * 49)), g1024 = (int)(n / (1024 * 49));
    timed("block256_chunks_nt", g256, [&] { k_write_block_chunks<256, true><<<g256, 256>>>(a, n); });
    timed("block256_chunks", g256, [&] { k_write_block_chunks<256, false><<<g256, 256>>>(a, n); });
    timed("block512_chunks_nt", g512, [&] { k_write_block_chunks<512, true><<<g512, 512>>>(a, n); });
    timed("block1024_chunks_nt", g1024, [&] { k_write_block_chunks<1024, true><<<g1024, 1024>>>(a, n); });
    timed("block1024_chunks", g1024, [&] { k_write_block_chunks<1024, false><<<g1024, 1024>>>(a, n); });
  }
  CK(hipFree(a));
  CK(hipFree(b));
  return 0;
}
