// Small device-resident batches through the C-ABI from C++ (no Python in the loop): per-call cost
// back to back, synchronised latency, and the same call captured once in a hipGraph and replayed.
// Full path: classify + grouping (perm + counts), MAC swap in place, 65 backends / 65537 slots.
// NBG_SMALL=0 in the environment selects the two-launch path for comparison.
// Build: hipcc -O2 -std=c++17 -o tools/small_bench tools/small_bench.cpp -Lnetbricks_amd -lnbgpu \
//          -Wl,-rpath,'$ORIGIN/../netbricks_amd'
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../include/nbgpu.h"

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      std::exit(1);                                                                      \
    }                                                                                    \
  } while (0)
#define NB(x)                                                                            \
  do {                                                                                   \
    int r_ = (x);                                                                        \
    if (r_ != 0) {                                                                       \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, nbg_last_error());  \
      std::exit(1);                                                                      \
    }                                                                                    \
  } while (0)

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main() {
  std::vector<std::string> names;
  for (int i = 0; i < 65; ++i) names.push_back("backend-" + std::to_string(i));
  std::vector<const char*> np;
  std::vector<uint32_t> nl;
  for (auto& s : names) {
    np.push_back(s.data());
    nl.push_back(static_cast<uint32_t>(s.size()));
  }
  nbg_maglev* h = nullptr;
  NB(nbg_maglev_create(np.data(), nl.data(), 65, 65537, 0, &h));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* small = std::getenv("NBG_SMALL");
  std::printf("{\"path\": \"%s\", \"results\": {", small && std::atoi(small) == 0 ? "two-launch" : "default");
  const uint64_t sizes[] = {32, 64, 128, 256, 512, 1024, 2048, 4096, 16384, 65536};
  for (size_t si = 0; si < sizeof(sizes) / sizeof(sizes[0]); ++si) {
    const uint64_t n = sizes[si];
    std::vector<uint32_t> off(n);
    std::vector<uint16_t> len(n);
    const uint64_t bytes = nbg_trace_layout(n, 0, 7 + n, off.data(), len.data());
    std::vector<uint8_t> buf(bytes);
    NB(nbg_trace_fill(buf.data(), off.data(), len.data(), n, 7 + n, 65536, 0));
    uint8_t* d_pkts;
    uint16_t* d_be;
    uint32_t *d_perm, *d_cnt;
    CK(hipMalloc(&d_pkts, bytes));
    CK(hipMalloc(&d_be, n * 2));
    CK(hipMalloc(&d_perm, n * 4));
    CK(hipMalloc(&d_cnt, 66 * 4));
    CK(hipMemcpy(d_pkts, buf.data(), bytes, hipMemcpyHostToDevice));
    auto call = [&] {
      NB(nbg_maglev_classify_device(h, d_pkts, nullptr, nullptr, 64, 60, n, NBG_SWAP_MACS, d_be, d_perm, d_cnt, s));
    };
    for (int i = 0; i < 50; ++i) call();
    CK(hipStreamSynchronize(s));
    const int K = 2000;
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < K; ++i) call();
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double b2b = ms * 1e3 / K;
    std::vector<double> lat;
    for (int i = 0; i < 200; ++i) {
      const auto t0 = std::chrono::steady_clock::now();
      call();
      CK(hipStreamSynchronize(s));
      lat.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    // the same call captured once and replayed (single-launch batches only: the library refuses to
    // capture the multi-launch path)
    const bool small_path = n <= 2048 && !(small && std::atoi(small) == 0);
    if (!small_path) {
      std::printf("%s\"%llu\": {\"back_to_back_us\": %.2f, \"latency_us_median\": %.2f, \"mpps_back_to_back\": %.1f}",
                  si ? ", " : "", static_cast<unsigned long long>(n), b2b, median(lat), n / b2b);
      CK(hipFree(d_pkts));
      CK(hipFree(d_be));
      CK(hipFree(d_perm));
      CK(hipFree(d_cnt));
      continue;
    }
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    call();
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int i = 0; i < 50; ++i) CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < K; ++i) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double gb2b = ms * 1e3 / K;
    std::vector<double> glat;
    for (int i = 0; i < 200; ++i) {
      const auto t0 = std::chrono::steady_clock::now();
      CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      glat.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    // check the graph replay still matches a direct call (counts of the last replay)
    std::vector<uint32_t> cnt(66);
    CK(hipMemcpy(cnt.data(), d_cnt, 66 * 4, hipMemcpyDeviceToHost));
    uint64_t total = 0;
    for (uint32_t c : cnt) total += c;
    std::printf("%s\"%llu\": {\"back_to_back_us\": %.2f, \"latency_us_median\": %.2f, \"graph_back_to_back_us\": %.2f, "
                "\"graph_latency_us_median\": %.2f, \"mpps_back_to_back\": %.1f, \"counts_sum_ok\": %s}",
                si ? ", " : "", static_cast<unsigned long long>(n), b2b, median(lat), gb2b, median(glat),
                n / b2b, total == n ? "true" : "false");
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    CK(hipFree(d_pkts));
    CK(hipFree(d_be));
    CK(hipFree(d_perm));
    CK(hipFree(d_cnt));
  }
  std::printf("}}\n");
  nbg_maglev_destroy(h);
  return 0;
}
