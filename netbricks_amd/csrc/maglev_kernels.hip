// CDNA4 (gfx950) kernels for the Maglev flow-steering hot path.
//
// classify_kernel — one lane per packet (4 packets per lane per tile):
//   parse::<MacHeader> (offset 14, framework/src/headers/mac.rs:96-106)
//   swap_addresses      (headers/mac.rs:140-145)            -> 12-B store
//   ipv4_extract_flow   (utils/flow.rs:53-62)
//   FNV-1a 64 over the packed little-endian Flow (utils/flow.rs:10-18,105-110)
//   lut[hash % M]       (test/maglev/src/nf.rs:78-81)       -> u16 store
//   per-tile histogram of backends + decoupled look-back over tiles, giving every
//   tile its exclusive per-backend prefix (the stable FIFO order of group_by.rs:46-51).
// scatter_kernel — per tile, wave ballot multisplit ranks + per-wave LDS counters,
//   writes perm[] = packet indices grouped by backend in arrival order.
//
// Integer-only; no MFMA.  HBM-bound: 64 B read + 12 B + 2 B written per packet in
// classify, 2 B read + 4 B written in scatter.
#include <hip/hip_runtime.h>

#include "nbgpu_internal.h"

namespace nbg {

namespace {

constexpr uint32_t kSentinel = NBG_SENTINEL;
constexpr uint32_t kEth = 14;
constexpr uint32_t kFlagAggregate = 1;
constexpr uint32_t kFlagPrefix = 2;
constexpr uint32_t kSpinLimit = 1u << 22;

// LUT placement / width variants.
enum LutMode { kLdsU8 = 0, kLdsU16 = 1, kGlobalU8 = 2, kGlobalU16 = 3 };

// h = h ^ b; h *= 0x100000001b3 on (lo, hi) 32-bit halves:
// h * (2^40 + 0x1b3) = lo*0x1b3 + 2^32 * (mulhi(lo,0x1b3) + hi*0x1b3 + (lo << 8))  (mod 2^64)
__device__ __forceinline__ void fnv_step(uint32_t& lo, uint32_t& hi, uint32_t b) {
  lo ^= b;
  const uint32_t nhi = __umulhi(lo, 0x1b3u) + hi * 0x1b3u + (lo << 8);
  lo = lo * 0x1b3u;
  hi = nhi;
}

// x mod 65537 with 2^16 == -1 (mod 65537): alternating 16-bit digit sum.
__device__ __forceinline__ uint32_t mod_f4(uint32_t lo, uint32_t hi) {
  uint32_t r = (lo & 0xffffu) + (hi & 0xffffu) + 131074u - (lo >> 16) - (hi >> 16);  // [4, 262144]
  r = (r & 0xffffu) + 65537u - (r >> 16);                                          // [65533, 131072]
  return r >= 65537u ? r - 65537u : r;
}

// Barrett: mu = floor(2^64 / m); q underestimates floor(h/m) by at most one.
__device__ __forceinline__ uint32_t mod_barrett(uint32_t lo, uint32_t hi, uint32_t m, uint64_t mu) {
  const uint64_t h = (static_cast<uint64_t>(hi) << 32) | lo;
  const uint64_t q = __umul64hi(h, mu);
  uint64_t r = h - q * m;
  if (r >= m) r -= m;
  return static_cast<uint32_t>(r);
}

// FNV over Flow{src_ip, dst_ip, src_port, dst_port, proto} (LE fields of BE-read values):
// byte order = p[15],p[14],p[13],p[12], p[19..16], p[ps+1],p[ps], p[ps+3],p[ps+2], p[9]
// where p = frame + 14.
__device__ __forceinline__ void fnv_flow(uint32_t& lo, uint32_t& hi, uint32_t src_be, uint32_t dst_be, uint32_t ports_be,
                                         uint32_t proto) {
  // src_be / dst_be / ports_be are the wire bytes packed little-endian (byte k at bits 8k).
  lo = 0x84222325u;  // 0xcbf29ce484222325
  hi = 0xcbf29ce4u;
  fnv_step(lo, hi, src_be >> 24);
  fnv_step(lo, hi, (src_be >> 16) & 0xffu);
  fnv_step(lo, hi, (src_be >> 8) & 0xffu);
  fnv_step(lo, hi, src_be & 0xffu);
  fnv_step(lo, hi, dst_be >> 24);
  fnv_step(lo, hi, (dst_be >> 16) & 0xffu);
  fnv_step(lo, hi, (dst_be >> 8) & 0xffu);
  fnv_step(lo, hi, dst_be & 0xffu);
  fnv_step(lo, hi, (ports_be >> 8) & 0xffu);
  fnv_step(lo, hi, ports_be & 0xffu);
  fnv_step(lo, hi, ports_be >> 24);
  fnv_step(lo, hi, (ports_be >> 16) & 0xffu);
  fnv_step(lo, hi, proto);
}

template <int LUTM>
__device__ __forceinline__ uint32_t lut_get(const ClassifyArgs& a, const uint8_t* lut_lds, uint32_t idx) {
  if constexpr (LUTM == kLdsU8) return lut_lds[idx];
  if constexpr (LUTM == kLdsU16) return reinterpret_cast<const uint16_t*>(lut_lds)[idx];
  if constexpr (LUTM == kGlobalU8) return static_cast<const uint8_t*>(a.lut)[idx];
  return static_cast<const uint16_t*>(a.lut)[idx];
}

template <int LUTM, bool F4>
__device__ __forceinline__ uint32_t lookup(const ClassifyArgs& a, const uint8_t* lut_lds, uint32_t lo, uint32_t hi) {
  const uint32_t idx = F4 ? mod_f4(lo, hi) : mod_barrett(lo, hi, a.m, a.mu);
  return lut_get<LUTM>(a, lut_lds, idx);
}

// Byte-wise path: any alignment, any length, any IHL.  Returns the bin (nb = sentinel).
template <int LUTM, bool F4>
__device__ __forceinline__ uint32_t classify_slow(const ClassifyArgs& a, const uint8_t* lut_lds, uint8_t* p,
                                               uint32_t len) {
  if (len < kEth) return a.nb;  // Packet::parse_header assert (interface/packet.rs:392-399)
  if (a.swap) {                 // transform runs before group_by over the batch
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const uint8_t d = p[k], s = p[k + 6];
      p[k] = s;
      p[k + 6] = d;
    }
  }
  const uint8_t* q = p + kEth;
  const uint32_t plen = len - kEth;
  if (plen < 20) return a.nb;
  const uint32_t ps = (q[0] & 0xfu) * 4u;
  if (plen < ps + 4) return a.nb;
  const uint32_t src = q[12] | (q[13] << 8) | (q[14] << 16) | (static_cast<uint32_t>(q[15]) << 24);
  const uint32_t dst = q[16] | (q[17] << 8) | (q[18] << 16) | (static_cast<uint32_t>(q[19]) << 24);
  const uint32_t ports =
      q[ps] | (q[ps + 1] << 8) | (q[ps + 2] << 16) | (static_cast<uint32_t>(q[ps + 3]) << 24);
  uint32_t lo, hi;
  fnv_flow(lo, hi, src, dst, ports, q[9]);
  return lookup<LUTM, F4>(a, lut_lds, lo, hi);
}

__device__ __forceinline__ unsigned long long pack_desc(uint32_t epoch, uint32_t flag, uint32_t v) {
  return (static_cast<unsigned long long>((epoch << 2) | flag) << 32) | v;
}

template <int LUTM, bool F4, bool GROUP>
__global__ __launch_bounds__(kBlock) void classify_kernel(ClassifyArgs a) {
  extern __shared__ __align__(16) uint8_t smem[];
  __shared__ uint32_t s_tile;
  __shared__ uint32_t s_part[kBlock];
  const uint32_t nbins = a.nb + 1;
  const uint32_t hist_bytes = (nbins * 4u + 15u) & ~15u;
  uint32_t* hist = reinterpret_cast<uint32_t*>(smem);
  uint8_t* lut_lds = smem + hist_bytes;
  const uint32_t tid = threadIdx.x;

  if constexpr (LUTM == kLdsU8 || LUTM == kLdsU16) {
    const uint4* src = static_cast<const uint4*>(a.lut);
    uint4* dst = reinterpret_cast<uint4*>(lut_lds);
    for (uint32_t k = tid; k < a.lut_lds_bytes / 16u; k += kBlock) dst[k] = src[k];
  }

  for (uint32_t iter = 0;; ++iter) {
    if constexpr (GROUP) {
      if (tid == 0) s_tile = static_cast<uint32_t>(atomicAdd(&a.ticket[0], 1ull));
      for (uint32_t b = tid; b < nbins; b += kBlock) hist[b] = 0;
    }
    __syncthreads();
    const uint32_t tile = GROUP ? s_tile : blockIdx.x + iter * gridDim.x;
    if (tile >= a.n_tiles) {
      if constexpr (GROUP) {
        // Every block has taken its last ticket once it gets here; the last block to
        // arrive resets both counters for the next launch on the stream.
        if (tid == 0 && atomicAdd(&a.ticket[1], 1ull) == gridDim.x - 1) {
          atomicExch(&a.ticket[0], 0ull);
          atomicExch(&a.ticket[1], 0ull);
        }
      }
      break;
    }

    // ---- issue every packet's header loads first (48 B per packet, 12 in flight per lane)
    uint4 c0[kPktsPerThread], c1[kPktsPerThread], c2[kPktsPerThread];
    uint8_t* pp[kPktsPerThread];
    uint32_t plen[kPktsPerThread];
    bool fast[kPktsPerThread];
    const uint32_t base = tile * kTile;
#pragma unroll
    for (int k = 0; k < kPktsPerThread; ++k) {
      const uint32_t i = base + k * kBlock + tid;
      const bool valid = i < a.n_pkts;
      const uint32_t ii = valid ? i : 0;
      pp[k] = a.pkts + (a.off ? static_cast<size_t>(a.off[ii]) : static_cast<size_t>(ii) * a.stride);
      plen[k] = a.len ? a.len[ii] : a.fixed_len;
      fast[k] = valid && ((reinterpret_cast<uintptr_t>(pp[k]) & 15u) == 0) && plen[k] >= 48u;
      if (fast[k]) {
        const uint4* v = reinterpret_cast<const uint4*>(pp[k]);
        c0[k] = v[0];
        c1[k] = v[1];
        c2[k] = v[2];
      }
    }
    // ---- hash, swap, lookup
#pragma unroll
    for (int k = 0; k < kPktsPerThread; ++k) {
      const uint32_t i = base + k * kBlock + tid;
      if (i >= a.n_pkts) continue;
      uint32_t bin;
      // bytes 12..15 = c0.w: byte 14 = version/IHL
      if (fast[k] && ((c0[k].w >> 16) & 0xfu) == 5u) {
        // frame bytes: src 26..29 = c1.z>>16 | c1.w<<16 ; dst 30..33 = c1.w>>16 | c2.x<<16
        //              ports 34..37 = c2.x>>16 | c2.y<<16 ; proto 23 = c1.y>>24
        const uint32_t src = (c1[k].z >> 16) | (c1[k].w << 16);
        const uint32_t dst = (c1[k].w >> 16) | (c2[k].x << 16);
        const uint32_t ports = (c2[k].x >> 16) | (c2[k].y << 16);
        uint32_t lo, hi;
        fnv_flow(lo, hi, src, dst, ports, c1[k].y >> 24);
        bin = lookup<LUTM, F4>(a, lut_lds, lo, hi);
        if (a.swap) {
          const uint32_t w0 = c0[k].x, w1 = c0[k].y, w2 = c0[k].z;
          uint32_t* o = reinterpret_cast<uint32_t*>(pp[k]);
          // new bytes 0..5 = old 6..11, new 6..11 = old 0..5
          o[0] = (w1 >> 16) | (w2 << 16);
          o[1] = (w2 >> 16) | (w0 << 16);
          o[2] = (w0 >> 16) | (w1 << 16);
        }
      } else {
        bin = classify_slow<LUTM, F4>(a, lut_lds, pp[k], plen[k]);
      }
      a.backend[i] = static_cast<uint16_t>(bin == a.nb ? kSentinel : bin);
      if constexpr (GROUP) atomicAdd(&hist[bin], 1u);
    }

    if constexpr (GROUP) {
      __syncthreads();
      // ---- decoupled look-back, one lane per bin
      const bool last = tile == a.n_tiles - 1;
      for (uint32_t b = tid; b < nbins; b += kBlock) {
        const uint32_t agg = hist[b];
        unsigned long long* d = a.desc + static_cast<size_t>(tile) * nbins + b;
        uint32_t excl = 0;
        if (tile == 0) {
          __hip_atomic_store(d, pack_desc(a.epoch, kFlagPrefix, agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          __hip_atomic_store(d, pack_desc(a.epoch, kFlagAggregate, agg), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
          for (int64_t j = static_cast<int64_t>(tile) - 1; j >= 0; --j) {
            const unsigned long long* pd = a.desc + static_cast<size_t>(j) * nbins + b;
            unsigned long long w;
            uint32_t spins = 0;
            for (;;) {
              w = __hip_atomic_load(pd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              const uint32_t tag = static_cast<uint32_t>(w >> 32);
              if ((tag >> 2) == a.epoch && (tag & 3u)) break;
              if (++spins >= kSpinLimit) {
                atomicOr(a.err, 1u);
                w = pack_desc(a.epoch, kFlagPrefix, 0);
                break;
              }
              __builtin_amdgcn_s_sleep(1);
            }
            excl += static_cast<uint32_t>(w);
            if (((w >> 32) & 3u) == kFlagPrefix) break;
          }
          __hip_atomic_store(d, pack_desc(a.epoch, kFlagPrefix, excl + agg), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        }
        a.tile_prefix[static_cast<size_t>(tile) * nbins + b] = excl;
        if (last) hist[b] = excl + agg;  // grand totals
      }
      if (last) {
        // ---- group sizes and exclusive group bases (one block, once per call)
        __syncthreads();
        const uint32_t chunk = (nbins + kBlock - 1) / kBlock;
        const uint32_t lo = tid * chunk, hi = min(lo + chunk, nbins);
        uint32_t s = 0;
        for (uint32_t b = lo; b < hi; ++b) s += hist[b];
        s_part[tid] = s;
        __syncthreads();
        if (tid == 0) {
          uint32_t acc = 0;
          for (int t = 0; t < kBlock; ++t) {
            const uint32_t v = s_part[t];
            s_part[t] = acc;
            acc += v;
          }
        }
        __syncthreads();
        uint32_t acc = s_part[tid];
        for (uint32_t b = lo; b < hi; ++b) {
          a.group_base[b] = acc;
          a.counts[b] = hist[b];
          acc += hist[b];
        }
      }
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(kBlock) void scatter_kernel(ScatterArgs a) {
  extern __shared__ __align__(16) uint32_t cnt[];  // [4 waves][nbins]
  const uint32_t nbins = a.nb + 1;
  const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u;
  const uint32_t tile = blockIdx.x;
  for (uint32_t k = tid; k < 4u * nbins; k += kBlock) cnt[k] = 0;
  __syncthreads();

  const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint32_t bins[kPktsPerThread], ranks[kPktsPerThread];
  uint32_t* mycnt = cnt + wave * nbins;
  // wave w owns packets [tile*kTile + w*256, +256) in 4 rounds of 64
#pragma unroll
  for (int r = 0; r < kPktsPerThread; ++r) {
    const uint32_t i = tile * kTile + wave * (64u * kPktsPerThread) + r * 64u + lane;
    const bool valid = i < a.n_pkts;
    uint32_t bin = 0;
    if (valid) {
      const uint32_t v = a.backend[i];
      bin = v == kSentinel ? a.nb : v;
    }
    unsigned long long eq = __ballot(valid);
    for (uint32_t bit = 0; bit < a.bits; ++bit) {
      const bool set = (bin >> bit) & 1u;
      const unsigned long long bb = __ballot(set);
      eq &= set ? bb : ~bb;
    }
    uint32_t rank = 0;
    if (valid) {
      const uint32_t prior = mycnt[bin];
      rank = prior + __popcll(eq & lt);
      if ((eq & lt) == 0) mycnt[bin] = prior + __popcll(eq);
    }
    bins[r] = bin;
    ranks[r] = rank;
  }
  __syncthreads();
  for (uint32_t b = tid; b < nbins; b += kBlock) {
    uint32_t acc = a.group_base[b] + a.tile_prefix[static_cast<size_t>(tile) * nbins + b];
#pragma unroll
    for (uint32_t w = 0; w < 4; ++w) {
      const uint32_t c = cnt[w * nbins + b];
      cnt[w * nbins + b] = acc;
      acc += c;
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kPktsPerThread; ++r) {
    const uint32_t i = tile * kTile + wave * (64u * kPktsPerThread) + r * 64u + lane;
    if (i < a.n_pkts) a.perm[mycnt[bins[r]] + ranks[r]] = i;
  }
}

template <int LUTM, bool F4, bool GROUP>
int launch_one(const ClassifyArgs& a, int grid, size_t lds, hipStream_t s) {
  auto fn = classify_kernel<LUTM, F4, GROUP>;
  if (lds > 64 * 1024) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                            static_cast<int>(lds)) != hipSuccess)
      (void)hipGetLastError();  // not required on gfx950; never leave a sticky error behind
  }
  hipLaunchKernelGGL(fn, dim3(grid), dim3(kBlock), lds, s, a);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(NBG_EIO, "classify launch: %s", hipGetErrorString(e));
  return NBG_OK;
}

template <int LUTM>
int launch_mode(const ClassifyArgs& a, bool group, int grid, size_t lds, hipStream_t s) {
  const bool f4 = a.m == 65537u;
  if (f4) return group ? launch_one<LUTM, true, true>(a, grid, lds, s) : launch_one<LUTM, true, false>(a, grid, lds, s);
  return group ? launch_one<LUTM, false, true>(a, grid, lds, s) : launch_one<LUTM, false, false>(a, grid, lds, s);
}

size_t classify_lds(uint32_t nb, uint32_t lut_lds_bytes) {
  return ((static_cast<size_t>(nb + 1) * 4 + 15) & ~size_t(15)) + lut_lds_bytes;
}

}  // namespace

int launch_classify(const ClassifyArgs& a, bool wide_lut, bool lds_lut, int grid, void* stream) {
  const bool group = a.desc != nullptr;
  const size_t lds = classify_lds(a.nb, lds_lut ? a.lut_lds_bytes : 0);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (lds_lut) return wide_lut ? launch_mode<kLdsU16>(a, group, grid, lds, s) : launch_mode<kLdsU8>(a, group, grid, lds, s);
  return wide_lut ? launch_mode<kGlobalU16>(a, group, grid, lds, s) : launch_mode<kGlobalU8>(a, group, grid, lds, s);
}

int launch_scatter(const ScatterArgs& a, uint32_t n_tiles, void* stream) {
  const size_t lds = static_cast<size_t>(a.nb + 1) * 4 * 4;
  if (lds > 64 * 1024) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(scatter_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)) != hipSuccess)
      (void)hipGetLastError();
  }
  hipLaunchKernelGGL(scatter_kernel, dim3(n_tiles), dim3(kBlock), lds, static_cast<hipStream_t>(stream), a);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(NBG_EIO, "scatter launch: %s", hipGetErrorString(e));
  return NBG_OK;
}

// Resident workgroups for the classify kernel: CUs x blocks/CU as limited by LDS
// (the LDS-staged LUT amortises its staging over the tiles a resident block takes).
int max_classify_grid(bool /*wide_lut*/, bool lds_lut, uint32_t lds_bytes, int device, int* grid) {
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0)
    return set_error(NBG_ENODEV, "hipDeviceGetAttribute(CU count) failed");
  const size_t lds = classify_lds(0, lds_lut ? lds_bytes : 0) + 2048;  // + static LDS
  int per_cu = lds_lut ? static_cast<int>((160 * 1024) / lds) : 8;
  if (per_cu < 1) per_cu = 1;
  if (per_cu > 8) per_cu = 8;
  *grid = cus * per_cu;
  return NBG_OK;
}

}  // namespace nbg
