// Probe: dynamic LDS limits for 1024-thread workgroups on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(1024) void fill(uint32_t* out, uint32_t words) {
  extern __shared__ uint32_t lds[];
  for (uint32_t i = threadIdx.x; i < words; i += blockDim.x) lds[i] = i * 2654435761u;
  __syncthreads();
  uint32_t bad = 0;
  for (uint32_t i = threadIdx.x; i < words; i += blockDim.x) bad += lds[(i * 7919u) % words] != ((i * 7919u) % words) * 2654435761u;
  atomicAdd(out, bad);
}
int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  printf("sharedMemPerBlock %zu maxSharedMemoryPerMultiProcessor %zu sharedMemPerBlockOptin %zu\n", p.sharedMemPerBlock,
         p.maxSharedMemoryPerMultiProcessor, p.sharedMemPerBlockOptin);
  uint32_t* d;
  (void)hipMalloc(&d, 4);
  for (uint32_t kb : {48u, 64u, 96u, 128u, 144u, 160u}) {
    const uint32_t bytes = kb * 1024;
    hipError_t ea = hipFuncSetAttribute(reinterpret_cast<const void*>(fill), hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    (void)hipGetLastError();
    (void)hipMemset(d, 0, 4);
    hipLaunchKernelGGL(fill, dim3(1), dim3(1024), bytes, 0, d, bytes / 4);
    hipError_t el = hipGetLastError();
    hipError_t es = hipDeviceSynchronize();
    uint32_t bad = 0;
    (void)hipMemcpy(&bad, d, 4, hipMemcpyDeviceToHost);
    printf("%3u KB: attr=%s launch=%s sync=%s bad=%u\n", kb, hipGetErrorString(ea), hipGetErrorString(el),
           hipGetErrorString(es), bad);
  }
  return 0;
}
