#!/bin/bash
# Measurement build (tools/ab/lib_hrprobe.so, never the product): the host-batch server's blocks stamp
# each ticket with the GPU wall clock (100 MHz) at claim, descriptor seen, body start, body end and
# completion word; nbg_host_ring_stop writes the stamps of the first tickets to $NBG_PROBE_OUT
# (tools/hrprobe_stats.py summarises them).
set -e
cd "$(dirname "$0")/../.."
python3 tools/abpatch.py hrprobe \
  maglev_kernels.hip '__global__ __launch_bounds__(kSmallNT) void host_ring_kernel(HostRingArgs r) {' \
'__device__ unsigned long long g_hr_probe[1u << 18][5];
__global__ __launch_bounds__(kSmallNT) void host_ring_kernel(HostRingArgs r) {' \
  maglev_kernels.hip '      const uint32_t t = __hip_atomic_fetch_add(r.claim, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);' \
'      const uint32_t t = __hip_atomic_fetch_add(r.claim, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long pr_claim = wall_clock64();' \
  maglev_kernels.hip '      s_ticket = t;
      s_go = go;' \
'      s_ticket = t;
      s_go = go;
      if (go) {
        g_hr_probe[t & ((1u << 18) - 1u)][0] = pr_claim;
        g_hr_probe[t & ((1u << 18) - 1u)][1] = wall_clock64();
      }' \
  maglev_kernels.hip '    const GroupArgs g = hd.g;
    switch (hd.variant & 15u) {' \
'    const GroupArgs g = hd.g;
    if (tid == 0) g_hr_probe[t & ((1u << 18) - 1u)][2] = wall_clock64();
    switch (hd.variant & 15u) {' \
  maglev_kernels.hip '    __threadfence_system();  // this thread'"'"'s outputs are visible to the host
    __syncthreads();
    if (tid == 0) __hip_atomic_store(hd.done, hd.done_val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);' \
'    if (tid == 0) g_hr_probe[t & ((1u << 18) - 1u)][3] = wall_clock64();
    __threadfence_system();  // this thread'"'"'s outputs are visible to the host
    __syncthreads();
    if (tid == 0) __hip_atomic_store(hd.done, hd.done_val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (tid == 0) g_hr_probe[t & ((1u << 18) - 1u)][4] = wall_clock64();' \
  maglev_kernels.hip 'extern "C" uint64_t nbg_debug_lds_beside_ring(void) { return nbg::group_lds_beside_ring(); }' \
'extern "C" uint64_t nbg_debug_lds_beside_ring(void) { return nbg::group_lds_beside_ring(); }
extern "C" int nbg_probe_dump(const char* path, uint32_t n) {
  static unsigned long long h[1u << 18][5];
  n = n < (1u << 18) ? n : (1u << 18);
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(nbg::g_hr_probe), sizeof(h)) != hipSuccess) return -5;
  FILE* f = std::fopen(path, "wb");
  if (!f) return -5;
  std::fwrite(h, 40, n, f);
  std::fclose(f);
  return 0;
}' \
  nbgpu_api.hip '  (void)hipHostFree(r->host);
  (void)hipFree(r->claim);
  delete r;' \
'  if (const char* po = std::getenv("NBG_PROBE_OUT")) {
    extern int nbg_probe_dump_fwd(const char*, uint32_t);
    (void)nbg_probe_dump_fwd(po, static_cast<uint32_t>(r->next.load()));
  }
  (void)hipHostFree(r->host);
  (void)hipFree(r->claim);
  delete r;' \
  nbgpu_api.hip 'int nbg_host_ring_stop(nbg_host_ring* r) {' \
'extern "C" int nbg_probe_dump(const char* path, uint32_t n);
int nbg_probe_dump_fwd(const char* p, uint32_t n) { return nbg_probe_dump(p, n); }
int nbg_host_ring_stop(nbg_host_ring* r) {'
mkdir -p tools/ab/hrprobe && cp tools/ab/lib_hrprobe.so tools/ab/hrprobe/libnbgpu.so
echo built tools/ab/hrprobe/libnbgpu.so
