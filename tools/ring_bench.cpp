// The persistent RX ring (nbg_ring_*) against one launch per batch, fed from C++ (no Python in the
// producer loop, so the producer stays ahead of the kernel): C2 batches of 1M 64-B slots, 8 rotating
// inputs and outputs, 65 backends / 65537 slots, read only ("ro") or in place ("ip").
//   launch: K x nbg_maglev_classify_device_ex (no grouping) on one stream, HIP events around all K
//   ring:   the producer posts whenever a slot is free and stamps every change of the completed
//           count; the steady-state time per batch is the slope of completions over the middle
//           three quarters of the run (the ramp and the drain excluded), the wall figure includes both
// Prints one JSON line.
// Build: hipcc -O2 -std=c++17 -o tools/ring_bench tools/ring_bench.cpp -Lnetbricks_amd -lnbgpu \
//          -Wl,-rpath,'$ORIGIN/../netbricks_amd'
// Usage: ring_bench [ro|ip] [batches] [packets] [ahead|chunk]
//   chunk: the producer refills 32 slots at a time (whenever 32 are free) instead of one per completion
//   ahead: every batch is posted before the first completion is awaited (batches <= NBG_RING_SLOTS;
//          the producer out of the loop), the time per batch from the completions as above
// With an NBG_SPROBE build of libnbgpu.so the ring kernel's counters are printed too.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <algorithm>
#include <utility>
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

using Clock = std::chrono::steady_clock;

int main(int argc, char** argv) {
  const bool inplace = argc > 1 && std::strcmp(argv[1], "ip") == 0;
  const int K = argc > 2 ? std::atoi(argv[2]) : 512;
  const uint64_t n = argc > 3 ? std::strtoull(argv[3], nullptr, 10) : (1u << 20);
  const bool ahead = argc > 4 && std::strcmp(argv[4], "ahead") == 0;
  const bool chunk = argc > 4 && std::strcmp(argv[4], "chunk") == 0;
  if (ahead && K > static_cast<int>(NBG_RING_SLOTS)) {
    std::fprintf(stderr, "ahead: at most %u batches\n", NBG_RING_SLOTS);
    return 2;
  }
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
  constexpr int B = 8;
  std::vector<uint8_t*> pk(B);
  std::vector<uint16_t*> be(B);
  {
    std::vector<uint32_t> off(n);
    std::vector<uint16_t> len(n);
    const uint64_t bytes = nbg_trace_layout(n, 0, 900, off.data(), len.data());
    std::vector<uint8_t> buf(bytes);
    for (int i = 0; i < B; ++i) {
      NB(nbg_trace_fill(buf.data(), off.data(), len.data(), n, 900 + i, 65536, 0));
      CK(hipMalloc(&pk[i], bytes));
      CK(hipMalloc(&be[i], n * 2));
      CK(hipMemcpy(pk[i], buf.data(), bytes, hipMemcpyHostToDevice));
    }
  }
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const uint32_t flags = inplace ? NBG_SWAP_MACS : 0u;
  // one launch per batch
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 16; ++i)
    NB(nbg_maglev_classify_device_ex(h, pk[i % B], nullptr, nullptr, 64, 60, n, flags, be[i % B], nullptr, nullptr,
                                     nullptr, s));
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < K; ++i)
    NB(nbg_maglev_classify_device_ex(h, pk[i % B], nullptr, nullptr, 64, 60, n, flags, be[i % B], nullptr, nullptr,
                                     nullptr, s));
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double launch_us = ms * 1e3 / K;
  // the ring
  nbg_ring* r = nullptr;
  NB(nbg_ring_start(h, 64, 60, flags, 2000, s, &r));
  uint64_t t = 0;
  for (int i = 0; i < 16; ++i) NB(nbg_ring_post(r, pk[i % B], n, be[i % B], &t));
  NB(nbg_ring_wait(r, t, 10000));
  const uint64_t base = t + 1;
  std::vector<std::pair<double, uint64_t>> stamps;
  stamps.reserve(K + 1);
  uint64_t posted = 0, done = 0;
  const auto t0 = Clock::now();
  while (done < static_cast<uint64_t>(K)) {
    const bool refill = !chunk || posted - done <= NBG_RING_SLOTS - 32;
    while (refill && posted < static_cast<uint64_t>(K) && (ahead || posted - done < NBG_RING_SLOTS)) {
      NB(nbg_ring_post(r, pk[posted % B], n, be[posted % B], &t));
      ++posted;
    }
    uint64_t c = 0;
    NB(nbg_ring_poll(r, &c));
    c -= base;
    if (c != done) {
      stamps.emplace_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count(), c);
      done = c;
    }
  }
  const double wall = std::chrono::duration<double, std::micro>(Clock::now() - t0).count();
  NB(nbg_ring_stop(r));
  std::string dbg;
  using DbgFn = int (*)(unsigned int*, uint64_t);
  if (auto fn = reinterpret_cast<DbgFn>(dlsym(RTLD_DEFAULT, "nbg_debug_ringdbg"))) {
    std::vector<unsigned int> d(1024 * 20);
    if (fn(d.data(), d.size()) == 0) {
      unsigned long long s[4] = {0, 0, 0, 0};
      unsigned mx3 = 0;
      for (int b = 0; b < 256; ++b) {
        for (int i = 0; i < 4; ++i) s[i] += d[b * 20 + i];
        mx3 = std::max(mx3, d[b * 20 + 3]);
      }
      char tmp[256];
      std::snprintf(tmp, sizeof tmp,
                    ", \"prefetches\": %llu, \"taken\": %llu, \"empty_prefetches\": %llu, \"idle_entries\": %llu, "
                    "\"max_idle_entries_per_block\": %u",
                    s[0], s[1], s[2], s[3], mx3);
      dbg = tmp;
    }
  }
  using SpFn = int (*)(unsigned long long*, uint64_t);
  if (auto fn = reinterpret_cast<SpFn>(dlsym(RTLD_DEFAULT, "nbg_debug_sprobe"))) {
    // per block: mean interval between the 16 probed unit steps (wave 0, 100 MHz ticks), and the
    // spread of that over blocks and XCDs (block b on XCD b % 8 under round-robin dispatch)
    std::vector<unsigned long long> t(4096 * 20);
    if (fn(t.data(), t.size()) == 0) {
      constexpr int kBlocks = 255;  // the ring's classify blocks (block 255 is the relay)
      std::vector<double> m(kBlocks);
      double xcd[8] = {0}, worst = 0;
      int slow = 0;
      for (int b = 0; b < kBlocks; ++b) {
        const unsigned long long* w = &t[(b * 8) * 20];
        m[b] = (static_cast<double>(w[17]) - static_cast<double>(w[2])) / 15.0 / 100.0;
        xcd[b % 8] += m[b] / (b % 8 == 7 ? 31.0 : 32.0);
        for (int k = 2; k < 17; ++k) {
          const double iv = (static_cast<double>(w[k + 1]) - static_cast<double>(w[k])) / 100.0;
          worst = std::max(worst, iv);
          slow += iv > 5.0;
        }
      }
      std::vector<double> srt = m;
      std::sort(srt.begin(), srt.end());
      char tmp[512];
      std::snprintf(tmp, sizeof tmp,
                    ", \"step_us_by_block\": [%.2f, %.2f, %.2f, %.2f, %.2f], \"step_us_by_xcd\": [%.2f, %.2f, %.2f, "
                    "%.2f, %.2f, %.2f, %.2f, %.2f], \"worst_step_us\": %.2f, \"steps_over_5us\": %d",
                    srt[0], srt[25], srt[127], srt[229], srt[254], xcd[0], xcd[1], xcd[2], xcd[3], xcd[4], xcd[5],
                    xcd[6], xcd[7], worst, slow);
      dbg += tmp;
    }
  }
  const uint64_t lo = K / 8, hi = K - K / 8;
  size_t i0 = 0, i1 = 0;
  while (i0 < stamps.size() && stamps[i0].second < lo) ++i0;
  while (i1 < stamps.size() && stamps[i1].second < hi) ++i1;
  const double slope = (stamps[i1].first - stamps[i0].first) / static_cast<double>(stamps[i1].second - stamps[i0].second);
  // the slope over each eighth of the run (a drift over time shows here)
  {
    char tmp[64];
    dbg += ", \"slope_by_eighth\": [";
    for (int e = 0; e < 8; ++e) {
      const uint64_t a = K * e / 8, z = K * (e + 1) / 8 - 1;
      size_t j0 = 0, j1 = 0;
      while (j0 < stamps.size() && stamps[j0].second < a + 1) ++j0;
      while (j1 < stamps.size() && stamps[j1].second < z) ++j1;
      const double sl = j1 < stamps.size() && j0 < j1
                            ? (stamps[j1].first - stamps[j0].first) / static_cast<double>(stamps[j1].second - stamps[j0].second)
                            : 0.0;
      std::snprintf(tmp, sizeof tmp, "%s%.2f", e ? ", " : "", sl);
      dbg += tmp;
    }
    dbg += "]";
  }
  std::printf("{\"variant\": \"%s\", \"n_pkts\": %llu, \"batches\": %d, \"launch_us\": %.2f, \"ring_us_per_batch\": %.2f, "
              "\"ring_wall_us_per_batch\": %.2f, \"ring_gpps\": %.1f, \"launch_gpps\": %.1f, \"ahead\": %s%s}\n",
              inplace ? "in_place" : "read_only", static_cast<unsigned long long>(n), K, launch_us, slope, wall / K,
              n / slope / 1e3, n / launch_us / 1e3, ahead ? "true" : "false", dbg.c_str());
  nbg_maglev_destroy(h);
  for (int i = 0; i < B; ++i) {
    CK(hipFree(pk[i]));
    CK(hipFree(be[i]));
  }
  return 0;
}
