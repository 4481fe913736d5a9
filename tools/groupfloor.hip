// Floors for the group kernel's launch shape (measurement only): what a 512-thread-block grid over a
// 1M-packet batch costs before any grouping work.  Run under rocprofv3 --kernel-trace --stats (the
// kernel durations are the figures); hipEvent medians are printed as well.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/groupfloor tools/groupfloor.hip
//   empty      256 blocks x 512 threads, no memory access
//   bload      each thread loads its 8 packets' u16 backends (the group kernel's round-major layout)
//              and folds them into one word stored per block (the load latency alone)
//   io         bload + perm[i] = i for the same packets (u32 coalesced stores: the kernel's bytes)
//   io_lds     io through an LDS counting pass: 8 LDS atomics per thread, 3 block barriers
//   rows       bload + every block sums the 256 x 33 packed partition rows (the kScanDirect prologue)
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

constexpr uint32_t kN = 1u << 20, kBlk = 512, kRounds = 8, kParts = kN / (kBlk * kRounds), kHw = 33;

__global__ __launch_bounds__(kBlk) void empty_kernel(uint32_t* sink) {
  if (threadIdx.x == 0x7fffffffu) sink[0] = 1;
}

__device__ __forceinline__ uint32_t bload(const uint16_t* be, uint32_t* pre) {
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint32_t wb = blockIdx.x * (kBlk * kRounds) + wave * 64u * kRounds;
  uint32_t acc = 0;
#pragma unroll
  for (uint32_t r = 0; r < kRounds; ++r) {
    pre[r] = be[wb + r * 64u + lane];
    acc += pre[r];
  }
  return acc;
}

__global__ __launch_bounds__(kBlk) void bload_kernel(const uint16_t* be, uint32_t* sink) {
  uint32_t pre[kRounds];
  const uint32_t acc = bload(be, pre);
  if (acc == 0xffffffffu) sink[blockIdx.x] = acc;
}

__global__ __launch_bounds__(kBlk) void io_kernel(const uint16_t* be, uint32_t* perm, uint32_t* sink) {
  uint32_t pre[kRounds];
  const uint32_t acc = bload(be, pre);
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint32_t wb = blockIdx.x * (kBlk * kRounds) + wave * 64u * kRounds;
#pragma unroll
  for (uint32_t r = 0; r < kRounds; ++r) perm[wb + r * 64u + lane] = wb + r * 64u + lane + (pre[r] >> 16);
  if (acc == 0xffffffffu) sink[blockIdx.x] = acc;
}

__global__ __launch_bounds__(kBlk) void io_lds_kernel(const uint16_t* be, uint32_t* perm, uint32_t* sink) {
  __shared__ uint32_t cnt[128];
  __shared__ uint32_t slot[kBlk * kRounds];
  uint32_t pre[kRounds];
  if (threadIdx.x < 128) cnt[threadIdx.x] = 0;
  __syncthreads();
  bload(be, pre);
  uint32_t rk[kRounds];
#pragma unroll
  for (uint32_t r = 0; r < kRounds; ++r) rk[r] = atomicAdd(&cnt[pre[r] & 127u], 1u);
  __syncthreads();
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
#pragma unroll
  for (uint32_t r = 0; r < kRounds; ++r) slot[(wave * kRounds + r) * 64u + lane] = rk[r] + cnt[pre[r] & 127u];
  __syncthreads();
  const uint32_t base = blockIdx.x * (kBlk * kRounds);
#pragma unroll
  for (uint32_t r = 0; r < kRounds; ++r) perm[base + r * kBlk + threadIdx.x] = base + slot[r * kBlk + threadIdx.x];
  (void)sink;
}

__global__ __launch_bounds__(kBlk) void rows_kernel(const uint16_t* be, const uint32_t* rows, uint32_t* sink) {
  __shared__ uint32_t tot[2 * kHw];
  uint32_t pre[kRounds];
  if (threadIdx.x < 2 * kHw) tot[threadIdx.x] = 0;
  __syncthreads();
  uint32_t acc = bload(be, pre);
  constexpr uint32_t L = kBlk / kHw, kU = 18;
  const uint32_t t = threadIdx.x;
  if (t < kHw * L) {
    const uint32_t w = t % kHw, j = t / kHw;
    uint32_t h[kU], lo = 0, hi = 0;
#pragma unroll
    for (uint32_t k = 0; k < kU; ++k) h[k] = rows[min(j + k * L, kParts - 1u) * kHw + w];
#pragma unroll
    for (uint32_t k = 0; k < kU; ++k) {
      const bool v = j + k * L < kParts;
      lo += v ? h[k] & 0xffffu : 0u;
      hi += v ? h[k] >> 16 : 0u;
    }
    atomicAdd(&tot[2 * w], lo);
    atomicAdd(&tot[2 * w + 1], hi);
  }
  __syncthreads();
  acc += tot[threadIdx.x & 63u];
  if (acc == 0xffffffffu) sink[blockIdx.x] = acc;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 200;
  uint16_t* be;
  uint32_t *perm, *rows, *sink;
  CK(hipMalloc(&be, kN * 2));
  CK(hipMalloc(&perm, kN * 4));
  CK(hipMalloc(&rows, kParts * kHw * 4));
  CK(hipMalloc(&sink, 4096 * 4));
  std::vector<uint16_t> hb(kN);
  uint64_t s = 88172645463325252ull;
  for (auto& x : hb) {
    s ^= s << 13, s ^= s >> 7, s ^= s << 17;
    x = static_cast<uint16_t>(s % 65);
  }
  CK(hipMemcpy(be, hb.data(), kN * 2, hipMemcpyHostToDevice));
  CK(hipMemset(rows, 1, kParts * kHw * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto time = [&](const char* name, auto launch) {
    std::vector<float> ms;
    for (int i = 0; i < iters; ++i) {
      CK(hipEventRecord(e0, 0));
      launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t = 0;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    std::printf("%-8s event median %7.2f us (min %7.2f)\n", name, ms[ms.size() / 2] * 1e3, ms[0] * 1e3);
  };
  const dim3 g(kParts), b(kBlk);
  time("empty", [&] { hipLaunchKernelGGL(empty_kernel, g, b, 0, 0, sink); });
  time("bload", [&] { hipLaunchKernelGGL(bload_kernel, g, b, 0, 0, be, sink); });
  time("io", [&] { hipLaunchKernelGGL(io_kernel, g, b, 0, 0, be, perm, sink); });
  time("io_lds", [&] { hipLaunchKernelGGL(io_lds_kernel, g, b, 0, 0, be, perm, sink); });
  time("rows", [&] { hipLaunchKernelGGL(rows_kernel, g, b, 0, 0, be, rows, sink); });
  CK(hipDeviceSynchronize());
  return 0;
}
