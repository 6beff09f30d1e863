// w3_module_check.hip -- runs k_min<0> of the k_slot reproducer
// (tools/slot_inline_repro.hip) from separately compiled code objects, to
// tell whether the record-word-3 defect is in the IR
// that LLVM's SLP vectorizer leaves or in the AMDGPU backend's lowering of
// it.  The code objects are built by tools/w3_modules.sh from the device IR
// of the reproducer with and without SLP, each through llc at -O0..-O3 (and
// the SLP IR once more after opt's scalarizer).  Cases and expected records
// come from the reproducer's own k_gen / k_lane (the per-lane rules, bit-
// exact with the oracle).  Investigation tool, not product code.
//
//   tools/w3_modules.sh  (builds build/w3/*.co and build/w3/w3_module_check)
//   build/w3/w3_module_check 20000 build/w3/kmin_slp_O3.co ...
#define REPRO_NO_MAIN 1
#include "slot_inline_repro.hip"

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 20000;
  uint4 *recs, *work;
  uint32_t* acts;
  Result* ra;
  CHECK(hipMalloc(&recs, n * sizeof(uint4)));
  CHECK(hipMalloc(&work, n * sizeof(uint4)));
  CHECK(hipMalloc(&acts, n * sizeof(uint32_t)));
  CHECK(hipMalloc(&ra, n * sizeof(Result)));
  k_gen<<<(n + 255) / 256, 256>>>(n, recs, acts);
  k_lane<<<(n + 255) / 256, 256>>>(n, recs, acts, ra);
  CHECK(hipDeviceSynchronize());
  std::vector<uint32_t> ha(n);
  std::vector<Result> want(n);
  std::vector<uint4> hr(n);
  CHECK(hipMemcpy(ha.data(), acts, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(want.data(), ra, n * sizeof(Result), hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(hr.data(), recs, n * sizeof(uint4), hipMemcpyDeviceToHost));
  std::printf("{\"cases\":%d,\"modules\":{", n);
  for (int m = 2; m < argc; ++m) {
    hipModule_t mod;
    hipFunction_t fn;
    CHECK(hipModuleLoad(&mod, argv[m]));
    CHECK(hipModuleGetFunction(&fn, mod, "_Z5k_minILi0EEvN4coup8SlotArgsE"));
    CHECK(hipMemcpy(work, recs, n * sizeof(uint4), hipMemcpyDeviceToDevice));
    for (int i = 0; i < n; ++i) {
      SlotArgs sa;
      std::memset(&sa, 0, sizeof(sa));
      sa.dst_state = work + i;
      sa.action = (int)ha[i];
      sa.store = 1;
      size_t sz = sizeof(sa);
      void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &sa, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
      CHECK(hipModuleLaunchKernel(fn, 1, 1, 1, 64, 1, 1, 0, nullptr, nullptr, cfg));
    }
    CHECK(hipDeviceSynchronize());
    std::vector<uint4> got(n);
    CHECK(hipMemcpy(got.data(), work, n * sizeof(uint4), hipMemcpyDeviceToHost));
    int bad = 0, first = -1, by_word[4] = {0, 0, 0, 0};
    int by[18] = {0};
    for (int i = 0; i < n; ++i) {
      const uint4 e = want[i].rec, g = got[i];
      const bool d[4] = {e.x != g.x, e.y != g.y, e.z != g.z, e.w != g.w};
      if (d[0] || d[1] || d[2] || d[3]) {
        ++bad;
        for (int k = 0; k < 4; ++k) by_word[k] += d[k];
        by[ha[i] < 18u ? ha[i] : 0]++;
        if (first < 0) first = i;
      }
    }
    std::printf("%s\"%s\":{\"mismatch\":%d,\"by_word\":[%d,%d,%d,%d],\"by_action\":[", m > 2 ? "," : "", argv[m], bad,
                by_word[0], by_word[1], by_word[2], by_word[3]);
    for (int x = 0; x < 18; ++x) std::printf("%s%d", x ? "," : "", by[x]);
    std::printf("]");
    if (first >= 0)
      std::printf(",\"first\":{\"case\":%d,\"act\":%u,\"rec\":[%u,%u,%u,%u],\"want\":[%u,%u,%u,%u],\"got\":[%u,%u,%u,%u]}",
                  first, ha[first], hr[first].x, hr[first].y, hr[first].z, hr[first].w, want[first].rec.x,
                  want[first].rec.y, want[first].rec.z, want[first].rec.w, got[first].x, got[first].y, got[first].z,
                  got[first].w);
    std::printf("}");
    CHECK(hipModuleUnload(mod));
  }
  std::printf("}}\n");
  return 0;
}
