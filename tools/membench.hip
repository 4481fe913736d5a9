// Memory-pattern ceilings on MI355X for the Maglev classify kernel's access shapes.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/membench tools/membench.hip
// Usage: membench [rotating buffers, default 8] [iterations, default 100]
// Each pattern streams N rotating 64 MiB buffers (8: 512 MiB, 2x the 256 MiB Infinity Cache; 32:
// 2 GiB, 8x), so the ceilings can be taken at the same working set as the timed kernels.  Under
// rocprofv3 --pmc every dispatch of a pattern moves a known byte count (printed per pattern): the
// FETCH_SIZE / WRITE_SIZE calibration for these access shapes (tools/runs/r04_membench_pmc.sh).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ inline void nt_store(uint4* p, uint4 v) {
  u32x4 w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
}

__device__ inline uint4 nt_load(const uint4* p) {
  const u32x4 w = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(w.x, w.y, w.z, w.w);
}

constexpr size_t kBytes = 64ull << 20;
int kBufs = 8;

// 16 B written through the L2 (sc1): the persistent ring's in-place window stores (stg16_wt)
__device__ inline void wt_store(uint4* p, uint4 v) {
  const u32x4 w = {v.x, v.y, v.z, v.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(p), "v"(w) : "memory");
}

// U uint4 per thread, contiguous 1 KiB per wave-instruction; MODE: 0 read, 1 rw full, 2 rw chunk0, 3 copy
template <int U, int MODE, bool NTL = false>
__global__ __launch_bounds__(256) void pattern(uint4* __restrict__ buf, uint4* __restrict__ dst, uint32_t* sink) {
  const size_t base = (static_cast<size_t>(blockIdx.x) * 256 * U) + threadIdx.x;
  uint4 v[U];
#pragma unroll
  for (int k = 0; k < U; ++k) v[k] = NTL ? nt_load(&buf[base + k * 256]) : buf[base + k * 256];
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < U; ++k) {
    acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    if (MODE == 1) buf[base + k * 256] = make_uint4(v[k].y, v[k].x, v[k].z, v[k].w);
    if (MODE == 2 && (threadIdx.x & 3) == 0) buf[base + k * 256] = make_uint4(v[k].y, v[k].x, v[k].z, v[k].w);
    if (MODE == 3) dst[base + k * 256] = v[k];
    if (MODE == 4 && (threadIdx.x & 3) == 0) dst[(base + k * 256) >> 2] = v[k];  // dense 16 B per 64-B packet
    if (MODE == 5) nt_store(&buf[base + k * 256], make_uint4(v[k].y, v[k].x, v[k].z, v[k].w));
    if (MODE == 6 && (threadIdx.x & 3) == 0)
      nt_store(&buf[base + k * 256], make_uint4(v[k].y, v[k].x, v[k].z, v[k].w));
    if (MODE == 7) wt_store(&buf[base + k * 256], make_uint4(v[k].y, v[k].x, v[k].z, v[k].w));
    if (MODE == 8 && (threadIdx.x & 3) < 2)  // the first 32-B sector of every 64-B slot (chunks 0..1)
      nt_store(&buf[base + k * 256], make_uint4(v[k].y, v[k].x, v[k].z, v[k].w));
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// persistent grid-stride variant with U loads in flight
template <int U, int MODE>
__global__ __launch_bounds__(256) void pattern_p(uint4* __restrict__ buf, uint4* __restrict__ dst, uint32_t* sink,
                                                 size_t n16) {
  uint32_t acc = 0;
  for (size_t base = static_cast<size_t>(blockIdx.x) * 256 * U + threadIdx.x; base < n16;
       base += static_cast<size_t>(gridDim.x) * 256 * U) {
    uint4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = buf[base + k * 256];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
      if (MODE == 1) buf[base + k * 256] = make_uint4(v[k].y, v[k].x, v[k].z, v[k].w);
      if (MODE == 2 && (threadIdx.x & 3) == 0) buf[base + k * 256] = make_uint4(v[k].y, v[k].x, v[k].z, v[k].w);
      if (MODE == 3) dst[base + k * 256] = v[k];
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}


// IMIX descriptor windows: 4 lanes per packet read its 64-B window at off[p] (64-B aligned,
// scattered over ~375 MB); MODE 0 read, 1 in-place full-window nt rewrite, 2 + dense 12 B/pkt out
template <int MODE, bool NTL = false>
__global__ __launch_bounds__(256) void windows(uint8_t* __restrict__ buf, const uint32_t* __restrict__ off,
                                               uint8_t* __restrict__ dst, uint32_t* sink, uint32_t n) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, part = lane & 3u, quad = lane >> 2;
  const uint32_t wbase = blockIdx.x * 256u + wave * 64u;
  const uint32_t own = wbase + lane < n ? off[wbase + lane] : 0u;
  uint4 v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t o = static_cast<uint32_t>(__shfl(static_cast<int>(own), k * 16 + quad));
    v[k] = NTL ? nt_load(reinterpret_cast<const uint4*>(buf + o + part * 16u))
               : *reinterpret_cast<const uint4*>(buf + o + part * 16u);
  }
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    const uint32_t o = static_cast<uint32_t>(__shfl(static_cast<int>(own), k * 16 + quad));
    if (MODE == 1) nt_store(reinterpret_cast<uint4*>(buf + o + part * 16u), make_uint4(v[k].y, v[k].x, v[k].z, v[k].w));
    if ((MODE == 3 && part == 0u) || (MODE == 4 && part < 2u))  // 16 B / the first 32-B sector per window
      nt_store(reinterpret_cast<uint4*>(buf + o + part * 16u), make_uint4(v[k].y, v[k].x, v[k].z, v[k].w));
    if (MODE == 2 && part == 0u) {
      uint32_t* m = reinterpret_cast<uint32_t*>(dst + static_cast<size_t>(wbase + k * 16 + quad) * 12u);
      m[0] = v[k].y; m[1] = v[k].x; m[2] = v[k].z;
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <typename F>
float time_it(F f, int iters) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 8; ++i) f(i);
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) f(i);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f / iters;
}

int main(int argc, char** argv) {
  if (argc > 1) kBufs = std::max(1, std::atoi(argv[1]));
  const int iters = argc > 2 ? std::max(1, std::atoi(argv[2])) : 100;
  std::printf("rotating buffers: %d x 64 MiB = %d MiB; %d iterations per pattern\n", kBufs, kBufs * 64, iters);
  std::vector<uint4*> bufs(kBufs);
  for (auto& p : bufs) {
    CK(hipMalloc(&p, kBytes));
    CK(hipMemset(p, 1, kBytes));
  }
  uint4* dst;
  CK(hipMalloc(&dst, kBytes));
  uint32_t* sink;
  CK(hipMalloc(&sink, 64));
  const size_t n16 = kBytes / 16;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  auto report = [&](const char* name, float us, double rd, double wr) {
    std::printf("%-34s %8.2f us  read %6.0f GB/s  write %6.0f GB/s  total %6.0f GB/s\n", name, us, rd / us / 1e3,
                wr / us / 1e3, (rd + wr) / us / 1e3);
  };
#define RUN(U, MODE, NAME, RD, WR)                                                                      \
  {                                                                                                     \
    const int grid = static_cast<int>(n16 / (256 * U));                                                 \
    float us = time_it([&](int i) { pattern<U, MODE><<<grid, 256>>>(bufs[i % kBufs], dst, sink); }, iters); \
    report(NAME, us, RD, WR);                                                                           \
  }
#define RUNP(U, MODE, BPC, NAME, RD, WR)                                                                          \
  {                                                                                                               \
    const int grid = cus * BPC;                                                                                   \
    float us = time_it([&](int i) { pattern_p<U, MODE><<<grid, 256>>>(bufs[i % kBufs], dst, sink, n16); }, iters); \
    report(NAME, us, RD, WR);                                                                                     \
  }
  const double B = static_cast<double>(kBytes);
  for (int rep = 0; rep < 1; ++rep) {
    RUN(1, 0, "read U1", B, 0);
    RUN(4, 0, "read U4", B, 0);
    RUN(8, 0, "read U8", B, 0);
    RUN(16, 0, "read U16", B, 0);
    RUNP(4, 0, 4, "read persistent U4 x4/CU", B, 0);
    RUNP(8, 0, 4, "read persistent U8 x4/CU", B, 0);
    RUNP(8, 0, 8, "read persistent U8 x8/CU", B, 0);
    RUN(4, 1, "rw full U4", B, B);
    RUN(8, 1, "rw full U8", B, B);
    RUNP(8, 1, 4, "rw full persistent U8 x4/CU", B, B);
    RUN(4, 2, "rw chunk0 (16B/64B) U4", B, B / 4);
    RUN(8, 2, "rw chunk0 (16B/64B) U8", B, B / 4);
    RUN(4, 4, "read + dense 16B/pkt out U4", B, B / 4);
    RUN(4, 5, "rw full nt-store U4", B, B);
    RUN(4, 6, "rw chunk0 nt-store U4", B, B / 4);
    {  // the same shapes with non-temporal loads (the product's packet loads since round 2)
      const int grid = static_cast<int>(n16 / (256 * 4));
      report("read U4 nt-load", time_it([&](int i) { pattern<4, 0, true><<<grid, 256>>>(bufs[i % kBufs], dst, sink); }, iters), B, 0);
      report("rw full nt-load nt-store U4", time_it([&](int i) { pattern<4, 5, true><<<grid, 256>>>(bufs[i % kBufs], dst, sink); }, iters), B, B);
      report("rw 32B sector (chunks 0-1) nt-load nt-store U4", time_it([&](int i) { pattern<4, 8, true><<<grid, 256>>>(bufs[i % kBufs], dst, sink); }, iters), B, B / 2);
      report("rw chunk0 (16B) nt-load nt-store U4", time_it([&](int i) { pattern<4, 6, true><<<grid, 256>>>(bufs[i % kBufs], dst, sink); }, iters), B, B / 4);
      report("rw full nt-load sc1-store U4 (ring)", time_it([&](int i) { pattern<4, 7, true><<<grid, 256>>>(bufs[i % kBufs], dst, sink); }, iters), B, B);
      report("read nt-load + dense 16B/pkt out U4", time_it([&](int i) { pattern<4, 4, true><<<grid, 256>>>(bufs[i % kBufs], dst, sink); }, iters), B, B / 4);
      // four 64 MiB buffers' worth in one launch (the multi-batch launch's read ceiling), rotating over
      // 8 such 256 MiB buffers (2 GiB: a 256 MiB buffer reused back to back would fit the Infinity Cache)
      std::vector<uint4*> big(8);
      for (auto& p : big) {
        CK(hipMalloc(&p, 4 * kBytes));
        CK(hipMemset(p, 1, 4 * kBytes));
      }
      const int g4 = static_cast<int>(4 * n16 / (256 * 4));
      report("read 256 MiB in one launch U4 nt-load", time_it([&](int i) { pattern<4, 0, true><<<g4, 256>>>(big[i % 8], dst, sink); }, iters), 4 * B, 0);
      // the same rewrite shapes without a launch ramp every 64 MiB (the persistent ring's regime)
      report("rw full nt-load nt-store, 256 MiB per launch", time_it([&](int i) { pattern<4, 5, true><<<g4, 256>>>(big[i % 8], dst, sink); }, iters), 4 * B, 4 * B);
      report("rw 32B sector nt, 256 MiB per launch", time_it([&](int i) { pattern<4, 8, true><<<g4, 256>>>(big[i % 8], dst, sink); }, iters), 4 * B, 2 * B);
      report("rw full nt-load sc1-store, 256 MiB per launch", time_it([&](int i) { pattern<4, 7, true><<<g4, 256>>>(big[i % 8], dst, sink); }, iters), 4 * B, 4 * B);
      for (auto& p : big) CK(hipFree(p));
    }
    RUN(4, 3, "copy U4", B, B);
    RUN(8, 3, "copy U8", B, B);
    std::printf("--\n");
  }
  {
    // IMIX 7:4:1 of 60/572/1496-B frames at 64-B aligned offsets (tools/ mirror of tracegen mode 1)
    const uint32_t n = 1u << 20;
    std::vector<uint32_t> off(n);
    uint64_t x = 0x1234567ull, pos = 0;
    for (uint32_t i = 0; i < n; ++i) {
      x = x * 6364136223846793005ull + 1442695040888963407ull;
      const uint32_t r = static_cast<uint32_t>(x >> 33) % 12u;
      const uint32_t len = r < 7 ? 60 : (r < 11 ? 572 : 1496);
      off[i] = static_cast<uint32_t>(pos);
      pos += (len + 63) & ~63u;
    }
    std::vector<uint8_t*> ib(std::min(kBufs, 32));
    for (auto& p : ib) {
      CK(hipMalloc(&p, pos + 64));
      CK(hipMemset(p, 1, pos + 64));
    }
    uint32_t* d_off;
    CK(hipMalloc(&d_off, n * 4ull));
    CK(hipMemcpy(d_off, off.data(), n * 4ull, hipMemcpyHostToDevice));
    uint8_t* mo;
    CK(hipMalloc(&mo, n * 12ull));
    const int grid = static_cast<int>(n / 256);
    const double W = 64.0 * n, D = 4.0 * n;
    std::printf("IMIX buffer %.1f MB, 1M windows\n", pos / 1e6);
    float us = time_it([&](int i) { windows<0><<<grid, 256>>>(ib[i % ib.size()], d_off, mo, sink, n); }, iters);
    report("imix windows read", us, W + D, 0);
    us = time_it([&](int i) { windows<1><<<grid, 256>>>(ib[i % ib.size()], d_off, mo, sink, n); }, iters);
    report("imix windows rw nt (in place)", us, W + D, W);
    us = time_it([&](int i) { windows<2><<<grid, 256>>>(ib[i % ib.size()], d_off, mo, sink, n); }, iters);
    report("imix windows read + 12B/pkt out", us, W + D, 12.0 * n);
    us = time_it([&](int i) { windows<0, true><<<grid, 256>>>(ib[i % ib.size()], d_off, mo, sink, n); }, iters);
    report("imix windows read nt-load", us, W + D, 0);
    us = time_it([&](int i) { windows<1, true><<<grid, 256>>>(ib[i % ib.size()], d_off, mo, sink, n); }, iters);
    report("imix windows rw nt-load nt-store", us, W + D, W);
    us = time_it([&](int i) { windows<3, true><<<grid, 256>>>(ib[i % ib.size()], d_off, mo, sink, n); }, iters);
    report("imix windows rw 16B (chunk 0) nt", us, W + D, W / 4);
    us = time_it([&](int i) { windows<4, true><<<grid, 256>>>(ib[i % ib.size()], d_off, mo, sink, n); }, iters);
    report("imix windows rw 32B sector nt", us, W + D, W / 2);
  }
  return 0;
}
