// CDNA4 (gfx950) kernels for the Maglev flow-steering hot path.
//
// classify_kernel — per packet (test/maglev/src/nf.rs:92-106):
//   parse::<MacHeader>   offset 14 (framework/src/headers/mac.rs:96-106, feature "performance")
//   swap_addresses       headers/mac.rs:140-145
//   ipv4_extract_flow    utils/flow.rs:53-62
//   FNV-1a 64 over the packed little-endian Flow (utils/flow.rs:10-18,105-110)
//   lut[hash % M]        test/maglev/src/nf.rs:78-81
//   + a per-tile backend histogram for the group_by FIFO order (operators/group_by.rs:46-51).
//   Loads are cooperative: a wave reads 64 packets' 64-B header windows as 16-B chunks
//   (4 lanes per window, contiguous 1 KiB per instruction for the 64-B slot layout),
//   transposes them through LDS to one packet per lane, and the lane holding chunk 0
//   applies the MAC swap in registers and writes the window back with full-line stores.
// scan_kernel — (many backends only) per backend bin, exclusive scan of the partition
//   histograms over partitions, and the bin totals (64 bins per block, coalesced rows).
// group_kernel — per partition: the per-bin prefix over earlier partitions and the group
//   bases, then per 4096-packet chunk wave ballot multisplit ranks (stable), a local counting
//   sort in LDS, and coalesced stores of perm[] = packet indices grouped by backend.
//
// Integer/byte work only; no MFMA.  HBM-bound.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>

#include "nbgpu_internal.h"

namespace nbg {

namespace {

constexpr uint32_t kSentinel = NBG_SENTINEL;
constexpr uint32_t kEth = 14;

// LUT placement / width variants.
enum LutMode { kLdsU8 = 0, kLdsU16 = 1, kGlobalU8 = 2, kGlobalU16 = 3, kLdsU8Tail = 4, kIdx = 5 };
// kIdx (NBG_LUT_TILED): no lookup; the classify kernel emits the LUT index (bit 31 set, so it
// cannot be mistaken for the would-panic bin) and the tiled lookup resolves it later.

// Packet layouts: fixed slots (general), fixed slots known by the host to be 16-B aligned with
// owned windows, no length array and frames >= 48 B (every chunk readable, no per-lane
// predicates), and descriptors (offset + length arrays).
enum Layout { kFixed = 0, kLean = 1, kDesc = 2 };

// h = h ^ b; h *= 0x100000001b3 on (lo, hi) 32-bit halves:
// h * (2^40 + 0x1b3) = lo*0x1b3 + 2^32 * ((hi*0x1b3 mod 2^32) + (lo << 8))  (mod 2^64)
// -> one v_mad_u64_u32 (lo*0x1b3 + (hi*0x1b3) << 32), one v_mul_lo_u32, one shift-add.
__device__ __forceinline__ void fnv_step(uint32_t& lo, uint32_t& hi, uint32_t b) {
  lo ^= b;
  const uint64_t t = static_cast<uint64_t>(lo) * 0x1b3u + (static_cast<uint64_t>(hi * 0x1b3u) << 32);
  hi = static_cast<uint32_t>(t >> 32) + (lo << 8);
  lo = static_cast<uint32_t>(t);
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

// FNV over Flow{src_ip, dst_ip, src_port, dst_port, proto} (LE fields of BE-read values).
// src/dst/ports are the wire bytes packed little-endian (wire byte k at bits 8k), so the
// hashed byte order is src[3..0], dst[3..0], ports[1],ports[0], ports[3],ports[2], proto.
__device__ __forceinline__ void fnv_flow(uint32_t& lo, uint32_t& hi, uint32_t src, uint32_t dst, uint32_t ports,
                                         uint32_t proto) {
  lo = 0x84222325u;  // 0xcbf29ce484222325
  hi = 0xcbf29ce4u;
  fnv_step(lo, hi, src >> 24);
  fnv_step(lo, hi, (src >> 16) & 0xffu);
  fnv_step(lo, hi, (src >> 8) & 0xffu);
  fnv_step(lo, hi, src & 0xffu);
  fnv_step(lo, hi, dst >> 24);
  fnv_step(lo, hi, (dst >> 16) & 0xffu);
  fnv_step(lo, hi, (dst >> 8) & 0xffu);
  fnv_step(lo, hi, dst & 0xffu);
  fnv_step(lo, hi, (ports >> 8) & 0xffu);
  fnv_step(lo, hi, ports & 0xffu);
  fnv_step(lo, hi, ports >> 24);
  fnv_step(lo, hi, (ports >> 16) & 0xffu);
  fnv_step(lo, hi, proto);
}

template <int LUTM>
__device__ __forceinline__ uint32_t lut_get(const ClassifyArgs& a, const uint8_t* lut_lds, uint32_t idx) {
  if constexpr (LUTM == kLdsU8) return lut_lds[idx];
  if constexpr (LUTM == kLdsU16) return reinterpret_cast<const uint16_t*>(lut_lds)[idx];
  if constexpr (LUTM == kGlobalU8) return static_cast<const uint8_t*>(a.lut)[idx];
  if constexpr (LUTM == kLdsU8Tail) return idx < 65536u ? lut_lds[idx] : a.lut_tail;  // streaming kernel
  if constexpr (LUTM == kIdx) return idx | 0x80000000u;
  return static_cast<const uint16_t*>(a.lut)[idx];
}

template <int LUTM, bool F4>
__device__ __forceinline__ uint32_t lookup(const ClassifyArgs& a, const uint8_t* lut_lds, uint32_t lo, uint32_t hi) {
  const uint32_t idx = F4 ? mod_f4(lo, hi) : mod_barrett(lo, hi, a.m, a.mu);
  return lut_get<LUTM>(a, lut_lds, idx);
}

// DIR-24-8 lookup_entry (test/lpm/src/nf.rs:88-98) of a host-order IPv4 address.
__device__ __forceinline__ uint32_t lpm_lookup(const uint16_t* tbl24, const uint16_t* tbl_long, uint32_t ip) {
  const uint32_t t = tbl24[ip >> 8];
  return (t & 0x8000u) ? tbl_long[((t & 0x7fffu) << 8) + (ip & 0xffu)] : t;
}

// One byte of global memory, loaded and waited for inside one asm statement: the compiler's wait
// pass never sees it pending (see classify_slow's SYNC).
__device__ __forceinline__ uint32_t ld_byte_sync(const uint8_t* p) {
  uint32_t v;
  asm volatile(
      "global_load_ubyte %0, %1, off\n\t"
      "s_waitcnt vmcnt(0)"
      : "=v"(v)
      : "v"(p)
      : "memory");
  return v;
}

// Byte-wise path: any alignment, any length, any IHL.  Returns the bin (nb = sentinel);
// CHAIN also sets the lpm gate (sentinel when test/lpm cannot parse the packet).
// SYNC (the streaming kernels): every byte is read by ld_byte_sync.  Compiler-visible loads here
// would stay pending, as far as the compiler's wait pass knows, across the unit loop's back-edge,
// and it then puts vmcnt(0) waits on the main path wherever the register allocator reuses their
// VGPRs, draining the LDS-DMA tile ring every step (measured: 2x per-step time in the lagged-
// grouping kernel).  A synchronous byte load costs a full memory round trip, but only packets off
// the fast path (none in the C2/C3/C5 traces) take this path.
// WT (the persistent ring kernel): the MAC bytes are stored write-through (sc1), so that they are in
// HBM once the store retires (nbg_ring completion, no L2 write-back in a kernel that never ends).
template <int LUTM, bool F4, bool CHAIN, bool SYNC = false, bool WT = false>
__device__ __forceinline__ uint32_t classify_slow(const ClassifyArgs& a, const uint8_t* lut_lds, uint8_t* p,
                                                  uint32_t len, uint32_t pkt, uint32_t& gate) {
  auto rd = [](const uint8_t* x) -> uint32_t {
    if constexpr (SYNC) return ld_byte_sync(x);
    return *x;
  };
  auto wr = [](uint8_t* x, uint8_t v) {
    if constexpr (WT)  // global (not flat): a flat store would also count in lgkmcnt
      __hip_atomic_store((__attribute__((address_space(1))) uint8_t*)(x), v, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    else *x = v;
  };
  gate = kSentinel;
  if (len < kEth) return a.nb;  // Packet::parse_header assert (interface/packet.rs:392-399)
  const uint8_t* q = p + kEth;
  const uint32_t plen = len - kEth;
  if constexpr (CHAIN) {
    // test/lpm: parse::<IpHeader> asserts payload_size >= 20 (packet.rs:392-399, ip.rs:53-56);
    // the gate is the group index of its group_by(lpm_groups) (test/lpm/src/nf.rs:216-221)
    if (plen < 20) return a.nb;
    const uint32_t ip = (rd(q + 12) << 24) | (rd(q + 13) << 16) | (rd(q + 14) << 8) | rd(q + 15);
    gate = lpm_lookup(a.tbl24, a.tbl_long, ip);
    if (gate >= a.lpm_groups) return a.nb;
  } else if (a.swap) {  // transform runs before group_by over the batch (chain: two swaps cancel)
    uint8_t* o = a.mac_out ? a.mac_out + static_cast<size_t>(pkt) * 12u : p;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const uint8_t d = static_cast<uint8_t>(rd(p + k)), s = static_cast<uint8_t>(rd(p + k + 6));
      wr(o + k, s);
      wr(o + k + 6, d);
    }
  }
  if (plen < 20) return a.nb;  // slice OOB in ipv4_extract_flow
  const uint32_t ps = (rd(q) & 0xfu) * 4u;
  if (plen < ps + 4) return a.nb;
  const uint32_t src = rd(q + 12) | (rd(q + 13) << 8) | (rd(q + 14) << 16) | (rd(q + 15) << 24);
  const uint32_t dst = rd(q + 16) | (rd(q + 17) << 8) | (rd(q + 18) << 16) | (rd(q + 19) << 24);
  const uint32_t ports = rd(q + ps) | (rd(q + ps + 1) << 8) | (rd(q + ps + 2) << 16) | (rd(q + ps + 3) << 24);
  uint32_t lo, hi;
  fnv_flow(lo, hi, src, dst, ports, rd(q + 9));
  return lookup<LUTM, F4>(a, lut_lds, lo, hi);
}

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
// Packet windows are read once: the streaming policy.  Round 1 measured it neutral on C2's 4-stream
// path (then served by this kernel); round 2, with C2 on the streaming kernel, it cut C3 from 48.9 to
// 44.8 us and C5 from 28.3 to 26.5 us per batch at 3 streams (profiles/r02_c3_c5_ntloads_ab.txt).
__device__ __forceinline__ uint4 ldg16(const uint8_t* p) {
  const u32x4_t w = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
  return make_uint4(w.x, w.y, w.z, w.w);
}
// Non-temporal 16-B store: in-place window write-back streams ~10 % faster with nt (tools/membench).
__device__ __forceinline__ void stg16_nt(uint8_t* p, uint4 v) {
  const u32x4_t w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, reinterpret_cast<u32x4_t*>(p));
}

// Write-through 16-B store (sc1: the line leaves L2 for HBM; MI355X_MICROARCH.md visibility table):
// the persistent ring kernel's outputs, visible to any later launch or copy once the store retires.
// Inline asm (the compiler cannot emit sc1 on a 64-bit-addressed 16-B store); s_nop 1 keeps the
// compiler's next instruction off the data VGPRs while the store reads them.
__device__ __forceinline__ void stg16_wt(void* p, uint4 v) {
  const u32x4_t w = {v.x, v.y, v.z, v.w};
  asm volatile(
      "global_store_dwordx4 %0, %1, off sc1\n\t"
      "s_nop 1"
      :
      : "v"(p), "v"(w)
      : "memory");
}

// Workgroup barrier for LDS-only hand-offs: wait for this wave's LDS operations, then s_barrier.
// Unlike __syncthreads() it does not wait for outstanding global stores (the release fence drains
// vmcnt), which would put HBM write latency on the group kernel's critical path.
__device__ __forceinline__ void lds_sync() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0) only
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// One wave's 64-packet tile in registers: lane = (quad, part) holds 16-B chunk `part` of
// packet k*16+quad (k = 0..3) — for 64-B slots each wave-instruction reads 1 KiB contiguous.
// Every load is issued unconditionally (a lane with nothing to read loads 16 B at the batch
// base) and nothing selects on its value: a predicated load merged with a default forces the
// compiler to wait for it inside the branch, serialising the four loads.  The chunk of a lane
// whose cflag bit is clear is never used.
struct TileRegs {
  uint4 ch[4];
  uint32_t cflag;  // bit k: chunk k was really read and the packet is long enough for the fast path
};

// Per-lane metadata of its own packet (descriptor mode: offset + length; else fixed).
struct TileMeta {
  uint32_t off, len;
};

// DESC (descriptor mode): off[] and len[] are both present and read unconditionally (clamped
// index), so the loads can stay in flight; otherwise only len[] may be present.
template <int LAYOUT>
__device__ __forceinline__ TileMeta load_meta(const ClassifyArgs& a, uint32_t wbase, uint32_t lane) {
  const uint32_t p = min(wbase + lane, a.n_pkts - 1u);  // clamped: the value of a lane past the end is unused
  TileMeta m;
  if constexpr (LAYOUT == kLean) {
    m.off = 0u;
    m.len = a.fixed_len;
  } else if constexpr (LAYOUT == kDesc) {
    m.off = a.off[p];
    m.len = a.len[p];
  } else {
    m.off = 0u;
    m.len = a.len ? a.len[p] : a.fixed_len;
  }
  return m;
}

// Fixed slots: the wave's tile base is wave-uniform (scalar 64-bit math) and lane offsets are
// 32-bit (stride < 2^24 is checked on the host), keeping 64-bit multiplies out of the VALU path.
template <int LAYOUT>
__device__ __forceinline__ const uint8_t* pkt_addr(const ClassifyArgs& a, uint32_t wbase, uint32_t idx_in_tile,
                                                   uint32_t off) {
  if constexpr (LAYOUT == kDesc) return a.pkts + off;
  return a.pkts + static_cast<size_t>(wbase) * a.stride + __umul24(idx_in_tile, a.stride);
}

template <int LAYOUT>
__device__ __forceinline__ void load_tile(const ClassifyArgs& a, uint32_t wbase, const TileMeta& m, uint32_t part,
                                          uint32_t quad, TileRegs& t) {
  constexpr bool DESC = LAYOUT == kDesc;
  const uint8_t* addr[4];
  t.cflag = 0;
  if constexpr (LAYOUT == kLean) {
    // every chunk of every packet is readable; only the batch tail is masked
    const uint8_t* tb = a.pkts + static_cast<size_t>(wbase) * a.stride + __umul24(quad, a.stride) + part * 16u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool pv = wbase + k * 16u + quad < a.n_pkts;
      addr[k] = pv ? tb + k * 16u * a.stride : a.pkts;
      t.cflag |= static_cast<uint32_t>(pv) << k;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) t.ch[k] = ldg16(addr[k]);
    return;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t src = k * 16u + quad;
    const uint32_t p = wbase + src;
    const bool pv = p < a.n_pkts;
    const uint32_t o = DESC ? static_cast<uint32_t>(__shfl(static_cast<int>(m.off), src)) : 0u;
    const uint32_t l = a.len ? static_cast<uint32_t>(__shfl(static_cast<int>(m.len), src)) : a.fixed_len;
    const uint8_t* base = pkt_addr<LAYOUT>(a, wbase, src, o);
    const bool aligned = (reinterpret_cast<uintptr_t>(base) & 15u) == 0;
    // chunk readable/writable: inside the frame, or the window is owned by this packet.  (Read only,
    // chunk 3 is unused, but skipping its load measured 0.7 us slower for C5: profiles/r04_c5_ablation.txt)
    const bool inwin = a.win_owned || (part * 16u + 16u <= l);
    const bool rd = pv && aligned && inwin;
    addr[k] = rd ? base + part * 16u : a.pkts;
    if (rd && l >= 48u) t.cflag |= 1u << k;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) t.ch[k] = ldg16(addr[k]);
}

// One transposed 64-packet tile of classify_kernel (its loads in `cur`, its chunks 0..2 in the
// wave's LDS rows `xp`): classify each lane's packet, write back, count.  Packets off the fast
// path are classified after this tile's loads, stores and gathers are all issued (`slow`): their
// byte-wise loads would otherwise make the compiler wait for every outstanding load.
template <int LUTM, bool F4, bool HIST, bool CHAIN, int LAYOUT>
__device__ __forceinline__ void classify_tile(const ClassifyArgs& a, const uint8_t* lut_lds, const uint8_t* xp,
                                              uint32_t* hist, uint32_t lane, uint32_t part, uint32_t quad,
                                              uint32_t wbase, const TileMeta& meta, const TileRegs& cur) {
  constexpr bool desc = LAYOUT == kDesc;
  const uint32_t p_own = wbase + lane;
  // compute lane: one packet (issues the LUT / LPM gathers)
  uint32_t bin = a.nb, gate = kSentinel, iplo = 0;
  bool resolve = false;  // CHAIN fast path: `gate` holds the raw tbl24 entry until consumed
  bool slow = false;
  uint8_t* pown = const_cast<uint8_t*>(pkt_addr<LAYOUT>(a, wbase, lane, meta.off));
  if (p_own < a.n_pkts) {
    const uint8_t* x = xp + lane * kXStride;
    const uint32_t w3 = *reinterpret_cast<const uint32_t*>(x + 12);
    const bool aligned = LAYOUT == kLean || (reinterpret_cast<uintptr_t>(pown) & 15u) == 0;
    const bool longf = LAYOUT == kLean || meta.len >= 48u;
    // same decision as the loader lanes: chunks 0..2 were loaded (and, if swapping, get written)
    if (aligned && longf && ((w3 >> 16) & 0xfu) == 5u) {
      const uint4 c1 = *reinterpret_cast<const uint4*>(x + 16);
      const uint2 c2 = *reinterpret_cast<const uint2*>(x + 32);
      // frame bytes: src 26..29, dst 30..33, ports 34..37, proto 23
      const uint32_t src = (c1.z >> 16) | (c1.w << 16);
      const uint32_t dst = (c1.w >> 16) | (c2.x << 16);
      const uint32_t ports = (c2.x >> 16) | (c2.y << 16);
      uint32_t lo, hi;
      if constexpr (CHAIN) {  // tbl24 gather issued here, resolved after the LUT gather
        const uint32_t ip = __builtin_bswap32(src);
        gate = a.tbl24[ip >> 8];
        iplo = ip & 0xffu;
        resolve = true;
      }
      fnv_flow(lo, hi, src, dst, ports, c1.y >> 24);
      bin = lookup<LUTM, F4>(a, lut_lds, lo, hi);
    } else {
      slow = true;
    }
  }
  // MAC swap in the loader lanes + window write-back (fast-path packets only).  Never in the chain
  // (lpm's and maglev's swaps cancel; the host clears a.swap): compiled out there, so the tile's
  // registers are dead after the transpose
  if (!CHAIN && a.swap) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      // the quad's chunk-0 lane holds bytes 12..15 (IHL) of this packet
      const uint32_t w3 = static_cast<uint32_t>(__shfl(static_cast<int>(cur.ch[k].w), lane & ~3u));
      const bool fast = ((cur.cflag >> k) & 1u) && ((w3 >> 16) & 0xfu) == 5u;
      const uint32_t src = k * 16u + quad;
      const uint32_t o = desc ? static_cast<uint32_t>(__shfl(static_cast<int>(meta.off), src)) : 0u;
      if (!fast) continue;
      uint8_t* base = const_cast<uint8_t*>(pkt_addr<LAYOUT>(a, wbase, src, o));
      uint4 v = cur.ch[k];
      if (part == 0u) {
        const uint32_t w0 = v.x, w1 = v.y, w2 = v.z;
        // new bytes 0..5 = old 6..11, new 6..11 = old 0..5
        v = make_uint4((w1 >> 16) | (w2 << 16), (w2 >> 16) | (w0 << 16), (w0 >> 16) | (w1 << 16), v.w);
      }
      if (a.mac_out) {
        // egress rewrite record: the 12 swapped bytes, dense (packet bytes untouched)
        if (part == 0u) {
          uint32_t* mo = reinterpret_cast<uint32_t*>(a.mac_out + static_cast<size_t>(wbase + src) * 12u);
          mo[0] = v.x;
          mo[1] = v.y;
          mo[2] = v.z;
        }
      } else if (part == 0u || a.wb_full) {
        stg16_nt(base + part * 16u, v);  // chunks 1..3 unchanged: makes the write whole lines
      }
    }
  }
  // consume the gathers
  if (p_own < a.n_pkts) {
    if (slow) bin = classify_slow<LUTM, F4, CHAIN>(a, lut_lds, pown, meta.len, p_own, gate);
    if constexpr (CHAIN) {
      if (resolve && (gate & 0x8000u)) gate = a.tbl_long[((gate & 0x7fffu) << 8) + iplo];
      a.gate[p_own] = static_cast<uint16_t>(gate);
      if (gate >= a.lpm_groups) bin = a.nb;  // test/lpm would panic: never reaches maglev
    }
    if constexpr (LUTM == kIdx) {
      a.idx_out[p_own] = (bin & 0x80000000u) ? (bin & 0x7fffffffu) : 0xffffffffu;
    } else {
      a.backend[p_own] = static_cast<uint16_t>(bin == a.nb ? kSentinel : bin);
      if constexpr (HIST) atomicAdd(&hist[bin], 1u);
    }
  }
}

// classify_kernel: each wave walks `tiles_per_wave` consecutive 64-packet tiles.  L2-gathered LUT:
// 256-thread blocks, one tile per wave, 8 blocks per CU (occupancy hides the latency; a software
// pipeline measured no faster there and cost 18 VGPRs).  LDS-staged LUT: one
// 1024-thread block per CU, up to 4 tiles per wave with two tiles' loads in flight (below).  Per
// tile: loads, LDS transpose, hash + gathers, then the write-back stores (vmcnt retires in issue
// order: stores issued before the gathers would delay their use), then the slow-path packets.
// One LDS histogram per block (two barriers per launch) is flushed once into the block's partition
// row (the block's 64 * waves * tiles_per_wave packets divide part_pkts).
// The kernel body; `bid` is the block's index within its batch (classify_desc_multi_kernel runs
// several batches' blocks in one grid).
template <int LUTM, bool F4, bool HIST, bool CHAIN, int LAYOUT, int NT>
__device__ __forceinline__ void classify_body(const ClassifyArgs& a, const uint32_t bid) {
  extern __shared__ __align__(16) uint8_t smem[];
  constexpr uint32_t kW = NT / 64u;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t part = lane & 3u, quad = lane >> 2;
  const uint32_t nbins = a.nb + 1;
  constexpr bool kLdsLut = LUTM == kLdsU8 || LUTM == kLdsU16;
  const uint32_t lut_bytes = kLdsLut ? a.lut_lds_bytes : 0u;
  uint8_t* lut_lds = smem;
  uint8_t* xp = smem + lut_bytes + wave * (64u * kXStride);
  uint32_t* hist = reinterpret_cast<uint32_t*>(smem + lut_bytes + kW * 64u * kXStride);  // per block
  const uint32_t tpw = a.tiles_per_wave;
  const uint32_t t0 = (bid * kW + wave) * tpw;  // first 64-packet tile of this wave

  // LDS-staged LUT: one 1024-thread block per CU (4 waves per SIMD) leaves VGPRs for kPf tiles'
  // loads in flight beside the tile being classified (a ring of kPf + 1 register tiles; the tile
  // loop is unrolled so that the ring stays in registers).  The first tiles' loads are issued
  // before the LUT staging, so that its latency hides under theirs.
  constexpr uint32_t kPf = kLdsLut ? 2u : 0u;
  constexpr uint32_t kRing = kPf + 1u;
  constexpr uint32_t kMaxTpw = kLdsLut ? kChunk / (64u * kW) : 1u;
  TileMeta rm[kRing];
  TileRegs rt[kRing];
  if constexpr (kLdsLut) {
#pragma unroll
    for (uint32_t j = 0; j < kPf; ++j) {
      const uint32_t wb = (t0 + j) * 64u;
      if (j < tpw && wb < a.n_pkts) {
        rm[j] = load_meta<LAYOUT>(a, wb, lane);
        load_tile<LAYOUT>(a, wb, rm[j], part, quad, rt[j]);
      }
    }
    constexpr int kS = 8;  // 16 B per thread per slot: up to 128 KiB per 1024-thread block
    const uint32_t nvec = lut_bytes / 16u;
    const uint4* src = static_cast<const uint4*>(a.lut);
    uint4 lt[kS];
#pragma unroll
    for (int j = 0; j < kS; ++j) {
      const uint32_t k = j * NT + tid;
      lt[j] = k < nvec ? src[k] : make_uint4(0, 0, 0, 0);
    }
    uint4* dst = reinterpret_cast<uint4*>(lut_lds);
#pragma unroll
    for (int j = 0; j < kS; ++j) {
      const uint32_t k = j * NT + tid;
      if (k < nvec) dst[k] = lt[j];
    }
  }
  if constexpr (HIST) {
    for (uint32_t b = tid; b < nbins; b += NT) hist[b] = 0;
  }
  if constexpr (HIST || kLdsLut) lds_sync();

  // transpose: chunks 0..2 of each packet of a tile -> LDS [packet][kXStride B]
  auto transpose = [&](const TileRegs& cur) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (part < 3u) *reinterpret_cast<uint4*>(xp + (k * 16u + quad) * kXStride + part * 16u) = cur.ch[k];
    }
  };


  if constexpr (kPf > 0) {
    // tile i sits in ring slot i % kRing; after its transpose, tile i + kPf is loaded into the
    // slot tile i - 1 used
#pragma unroll
    for (uint32_t i = 0; i < kMaxTpw; ++i) {
      const uint32_t wbase = (t0 + i) * 64u;
      if (i >= tpw || wbase >= a.n_pkts) break;  // wave-uniform
      transpose(rt[i % kRing]);
      const uint32_t j = i + kPf, wb = (t0 + j) * 64u;
      if (j < tpw && wb < a.n_pkts) {
        rm[j % kRing] = load_meta<LAYOUT>(a, wb, lane);
        load_tile<LAYOUT>(a, wb, rm[j % kRing], part, quad, rt[j % kRing]);
      }
      classify_tile<LUTM, F4, HIST, CHAIN, LAYOUT>(a, lut_lds, xp, hist, lane, part, quad, wbase, rm[i % kRing],
                                                           rt[i % kRing]);
    }
  } else if (LAYOUT == kDesc && tpw > 1u && tpw <= 4u) {
    // descriptor layouts, 2..4 tiles per wave (NBG_TPW, measurement): the descriptors of all of the
    // wave's tiles are loaded up front (measured no faster than one tile per wave for C3 / C5:
    // profiles/r04_c5_ablation.txt), unconditionally (clamped), so every tile after the first
    // issues its window loads at once instead of after a descriptor round trip of its own
    constexpr uint32_t kMetaTiles = 4;
    TileMeta mq[kMetaTiles];
#pragma unroll
    for (uint32_t j = 0; j < kMetaTiles; ++j) mq[j] = load_meta<LAYOUT>(a, (t0 + j) * 64u, lane);
#pragma unroll
    for (uint32_t i = 0; i < kMetaTiles; ++i) {
      const uint32_t wbase = (t0 + i) * 64u;
      if (i >= tpw || wbase >= a.n_pkts) break;  // wave-uniform
      __builtin_amdgcn_s_setprio(kLoadPrio);
      TileRegs cur;
      load_tile<LAYOUT>(a, wbase, mq[i], part, quad, cur);
      __builtin_amdgcn_s_setprio(0);
      transpose(cur);
      classify_tile<LUTM, F4, HIST, CHAIN, LAYOUT>(a, lut_lds, xp, hist, lane, part, quad, wbase, mq[i], cur);
    }
  } else {
    for (uint32_t i = 0; i < tpw; ++i) {
      const uint32_t wbase = (t0 + i) * 64u;
      if (wbase >= a.n_pkts) break;  // wave-uniform
      // The tile's loads are issued at raised wave priority, so a newly started wave gets its HBM
      // requests out ahead of resident waves' hash/gather work (bench +2 % in place, +4 % records).
      __builtin_amdgcn_s_setprio(kLoadPrio);
      const TileMeta meta = load_meta<LAYOUT>(a, wbase, lane);
      TileRegs cur;
      load_tile<LAYOUT>(a, wbase, meta, part, quad, cur);
      __builtin_amdgcn_s_setprio(0);
      transpose(cur);
      classify_tile<LUTM, F4, HIST, CHAIN, LAYOUT>(a, lut_lds, xp, hist, lane, part, quad, wbase, meta, cur);
    }
  }

  if constexpr (HIST) {
    // one flush per block into its partition row (the block's packets never straddle two):
    // 4096-packet rows take ~16 blocks' adds, so they rarely contend
    lds_sync();
    const uint32_t p = bid * kW * tpw * 64u / a.part_pkts;
    if (a.hist16) {  // two bins per word: half the atomics, and half the rows' bytes for the group kernel
      const uint32_t hw = (nbins + 1) >> 1;
      uint32_t* row = a.part_hist + static_cast<size_t>(p) * hw;
      for (uint32_t w = tid; w < hw; w += NT) {
        const uint32_t h = hist[2 * w] | (2 * w + 1 < nbins ? hist[2 * w + 1] << 16 : 0u);
        if (h) atomicAdd(&row[w], h);
      }
    } else {
      uint32_t* row = a.part_hist + static_cast<size_t>(p) * nbins;
      for (uint32_t b = tid; b < nbins; b += NT) {
        const uint32_t h = hist[b];
        if (h) atomicAdd(&row[b], h);
      }
    }
  }
}


template <int LUTM, bool F4, bool HIST, bool CHAIN, int LAYOUT, int NT = kBlock>
__global__ __launch_bounds__(NT, CHAIN ? 1 : 2048 / NT) void classify_kernel(ClassifyArgs a) {
  classify_body<LUTM, F4, HIST, CHAIN, LAYOUT, NT>(a, blockIdx.x);
}

// Several descriptor batches in one grid (several RX queues' bursts per launch): the launch's ramp
// and tail are paid once for all of them.  The batch of a block is found by a wave-uniform scan of
// blk_base (monotone; an empty batch owns no block).
template <int LUTM, bool F4, bool HIST, bool CHAIN>
__global__ __launch_bounds__(kBlock, CHAIN ? 1 : 2048 / kBlock) void classify_desc_multi_kernel(ClassifyArgs a,
                                                                                                 DescBatches db) {
  uint32_t j = 0;
#pragma unroll
  for (uint32_t k = 1; k < kMaxMulti; ++k) j = (k < db.n && blockIdx.x >= db.blk_base[k]) ? k : j;
  ClassifyArgs b = a;
  b.pkts = db.pkts[j];
  b.off = db.off[j];
  b.len = db.len[j];
  b.backend = db.backend[j];
  b.gate = db.gate[j];
  b.part_hist = db.part_hist[j];
  b.n_pkts = db.n_pkts[j];
  classify_body<LUTM, F4, HIST, CHAIN, kDesc, kBlock>(b, blockIdx.x - db.blk_base[j]);
}

// Loads at a 32-bit byte offset from a kernel-argument base: the compiler can then use the
// SGPR-base + 32-bit VGPR-offset form (one VGPR per address instead of two).
__device__ __forceinline__ uint32_t ld_u32(const uint32_t* base, uint32_t byte_off) {
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(base) + byte_off);
}
// Raw buffer resource over `bytes` bytes at p (gfx9 descriptor word 3: CK_BUFFER_RESOURCE_3RD_DWORD):
// a load past `bytes` returns 0 without touching memory, so the group kernel's loads need neither an
// index clamp nor a 64-bit address per lane (one 32-bit offset, constant parts in the instruction).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t raw_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, static_cast<int>(bytes), 0x00020000);
}
__device__ __forceinline__ uint32_t ld_u16(const uint16_t* base, uint32_t byte_off) {
  return *reinterpret_cast<const uint16_t*>(reinterpret_cast<const uint8_t*>(base) + byte_off);
}

// Inclusive scan over the 64 lanes of a wave with DPP moves (no LDS round trips): shifts by
// 1, 2, 4, 8 inside each 16-lane row, then row 0's / rows 0-1's totals broadcast into the rows
// above (row_bcast:15 into rows 1 and 3, row_bcast:31 into rows 2 and 3).  Lanes a move does not
// write keep the `old` operand, 0.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x111, 0xf, 0xf, false));
  x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x112, 0xf, 0xf, false));
  x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x114, 0xf, 0xf, false));
  x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x118, 0xf, 0xf, false));
  x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x142, 0xa, 0xf, false));
  x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x143, 0xc, 0xf, false));
  return x;
}

// Block-wide exclusive scan of one value per thread (blocks of NT threads); returns the
// exclusive prefix and the total.
template <uint32_t NT>
__device__ __forceinline__ uint32_t block_excl_scan_n(uint32_t v, uint32_t* s_wave, uint32_t& total) {
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t x = wave_incl_scan(v);
  if (lane == 63u) s_wave[wave] = x;
  lds_sync();
  uint32_t wpre = 0, tot = 0;
#pragma unroll
  for (uint32_t w = 0; w < NT / 64; ++w) {
    const uint32_t t = s_wave[w];
    if (w < wave) wpre += t;
    tot += t;
  }
  lds_sync();
  total = tot;
  return wpre + x - v;
}

// Stable rank of this lane among the lanes of its wave with the same `bin` (valid lanes only), and
// how many lanes hold that bin: one ballot per bin bit plus one for validity, no loop over lanes.
template <int BITS>
__device__ __forceinline__ void wave_match_rank(uint32_t bin, bool valid, uint32_t lane, uint32_t& rank,
                                                uint32_t& count) {
  const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const uint32_t mv = valid ? ~0u : 0u;
  const unsigned long long bv = __builtin_amdgcn_ballot_w64(valid);
  uint32_t elo = ~(static_cast<uint32_t>(bv) ^ mv), ehi = ~(static_cast<uint32_t>(bv >> 32) ^ mv);
#pragma unroll
  for (int bit = 0; bit < BITS; ++bit) {
    const uint32_t m = static_cast<uint32_t>(__builtin_amdgcn_sbfe(static_cast<int>(bin), bit, 1));  // 0 or ~0
    const unsigned long long bb = __builtin_amdgcn_ballot_w64(m != 0);
    elo &= ~(static_cast<uint32_t>(bb) ^ m);
    ehi &= ~(static_cast<uint32_t>(bb >> 32) ^ m);
  }
  rank = __popc(elo & static_cast<uint32_t>(lt)) + __popc(ehi & static_cast<uint32_t>(lt >> 32));
  count = __popc(elo) + __popc(ehi);
}

// N (2..4) consecutive bin bits b .. b + N - 1 of a wave ballot multisplit, four VALU operations per
// bit: the lane's bit as 0 / ~0 (v_bfe), the wave's ballot of it (v_cmp into an SGPR pair), and per
// 32-lane half acc |= ballot ^ bit in one v_bitop3 (truth table 0xde over (ballot, acc, bit)).  The
// compiler's own form of the accumulation took ~6 operations per bit (v_lshlrev + v_cmp for the
// ballot, two v_xor, v_or3), and the group kernel's ranks are VALU-bound (profiles/r05_group_pmc.txt).
// The N compares are one asm statement and the bitop3s follow in others: a VALU read of an SGPR that a
// VALU just wrote needs wait states on gfx950, which the compiler's hazard pass inserts between
// statements (one s_nop per group instead of one per bit).
template <int N>
__device__ __forceinline__ void mismatch_bits(uint32_t bin, int b, uint32_t& mlo, uint32_t& mhi) {
  static_assert(N >= 2 && N <= 4, "2 to 4 bits per group");
  uint32_t m[4];
  unsigned long long q[4];
#pragma unroll
  for (int k = 0; k < N; ++k) m[k] = static_cast<uint32_t>(__builtin_amdgcn_sbfe(static_cast<int>(bin), b + k, 1));
  if constexpr (N == 4)
    asm("v_cmp_ne_u32_e64 %0, 0, %4\n\tv_cmp_ne_u32_e64 %1, 0, %5\n\t"
        "v_cmp_ne_u32_e64 %2, 0, %6\n\tv_cmp_ne_u32_e64 %3, 0, %7"
        : "=&s"(q[0]), "=&s"(q[1]), "=&s"(q[2]), "=&s"(q[3])
        : "v"(m[0]), "v"(m[1]), "v"(m[2]), "v"(m[3]));
  else if constexpr (N == 3)
    asm("v_cmp_ne_u32_e64 %0, 0, %3\n\tv_cmp_ne_u32_e64 %1, 0, %4\n\tv_cmp_ne_u32_e64 %2, 0, %5"
        : "=&s"(q[0]), "=&s"(q[1]), "=&s"(q[2])
        : "v"(m[0]), "v"(m[1]), "v"(m[2]));
  else
    asm("v_cmp_ne_u32_e64 %0, 0, %2\n\tv_cmp_ne_u32_e64 %1, 0, %3" : "=&s"(q[0]), "=&s"(q[1]) : "v"(m[0]), "v"(m[1]));
#pragma unroll
  for (int k = 0; k < N; ++k) {
    asm("v_bitop3_b32 %0, %1, %0, %2 bitop3:0xde" : "+v"(mlo) : "s"(static_cast<uint32_t>(q[k])), "v"(m[k]));
    asm("v_bitop3_b32 %0, %1, %0, %2 bitop3:0xde" : "+v"(mhi) : "s"(static_cast<uint32_t>(q[k] >> 32)), "v"(m[k]));
  }
}

// All BITS bin bits (7 or 10): groups of 4, then the remaining 3 or 2
template <int BITS>
__device__ __forceinline__ void mismatch_all(uint32_t bin, uint32_t& mlo, uint32_t& mhi) {
  static_assert(BITS % 4 >= 2 || BITS % 4 == 0, "groups of 2 to 4 bits");
#pragma unroll
  for (int b = 0; b + 4 <= BITS; b += 4) mismatch_bits<4>(bin, b, mlo, mhi);
  if constexpr (BITS % 4 == 3) mismatch_bits<3>(bin, BITS - 3, mlo, mhi);
  if constexpr (BITS % 4 == 2) mismatch_bits<2>(bin, BITS - 2, mlo, mhi);
}

// ---- streaming classify (fixed 64-B-aligned slots, u8 LUT <= 65537 entries) -------------------
//
// One 512-thread block per CU (persistent).  The block stages the LUT in LDS once with LDS-DMA
// (entries 0..65535; entry 65536 of a 65537-slot table is the kernel argument lut_tail), so the
// per-packet lookup is an LDS read instead of an L2 gather (a 1M-packet batch of L2 gathers costs
// ~3.3 us of L2 request throughput).  Each wave then streams 64-packet tiles through a
// private ring of kRing LDS buffers: every packet's row lands packet-major by global_load_lds_dwordx4
// straight from HBM — no VGPRs held by loads in flight, no transpose — while the wave classifies the
// tile kStreamAhead tiles behind.  Tiles are interleaved so that the whole grid sweeps the batch
// sequentially; the block's backend histogram is flushed once per unit of W tiles.
//
// LDS-DMA writes are ordered for the issuing wave's ds_read only by its own covering vmcnt
// (MI355X_MICROARCH.md item 7).  hipcc does not count the inline-asm loads, so each tile is waited
// for with a counted s_waitcnt vmcnt(4 * tiles issued after it): other VM operations issued in
// between (stores, flush atomics, the compiler's slow-path loads) only make that wait conservative.
constexpr int kStreamNT = 512;                 // threads per block (8 waves)
constexpr int kStreamW = kStreamNT / 64;
constexpr int kRing = 2;                       // LDS tile buffers per wave
[[maybe_unused]] constexpr int kStreamAhead = kRing - 1;  // tiles in flight while one is classified
static_assert(kRing >= 2 && kRing <= 3, "classify_stream_kernel tracks the counts of three tiles at most");
// LDS bytes per packet: 48 (chunks 0..2, all the classify reads) for read-only and records; 64 (the
// whole slot) for the in-place swap, which then writes every line back whole from LDS (measured:
// 48-B rows read faster, whole-line write-back beats 16-B partial-line stores)
template <int MODE>
constexpr uint32_t row_of() { return MODE == 1 ? 64u : 48u; }
template <int MODE>
constexpr uint32_t stream_row_of() { return row_of<MODE>(); }
constexpr uint32_t kLutLds = 65536;            // LUT bytes staged in LDS

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return static_cast<uint32_t>(
      reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) void*)(p)));
}

// 16 B per active lane from `src` into LDS at m0 + lane * 16 (lds_base wave-uniform).
__device__ __forceinline__ void glds16(const void* src, uint32_t lds_base) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds_base))
      : "memory");
}

// The same with the streaming (non-temporal) policy, for packet windows (read once).  Measured on
// classify_stream_kernel, 1M packets, one MI355X (tools/runs/gpu_ab_ms.sh, profiles/r02_tile_nt_ab.txt):
// one stream, read-only 14.6 -> 13.5 us, in place 27.5 -> 25.5, records 17.0 -> 16.6; three streams
// with grouping, read-only 16.1 -> 15.8, in place neutral, records 17.8 -> 18.9 (slower).  So nt for
// read-only and in place (NT = true), the default policy for records.  The LUT pieces keep the
// default policy: every CU of an XCD re-reads them from L2.
template <bool NT>
__device__ __forceinline__ void glds16_tile(const void* src, uint32_t lds_base) {
  if constexpr (NT) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off nt\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds_base))
        : "memory");
  } else {
    glds16(src, lds_base);
  }
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// Wait until tile i's four LDS-DMA loads landed: `ahead` tiles (0..5) were issued after it.
__device__ __forceinline__ void wait_tile(uint32_t ahead) {
  if (ahead >= 5) wait_vm<20>();
  else if (ahead == 4) wait_vm<16>();
  else if (ahead == 3) wait_vm<12>();
  else if (ahead == 2) wait_vm<8>();
  else if (ahead == 1) wait_vm<4>();
  else wait_vm<0>();
}

// Wait until at most n VM operations are outstanding (n above 31 waits for 31: stricter, still right).
__device__ __forceinline__ void wait_vm_n(uint32_t n) {
#define NBG_VMC(i) \
  case i:          \
    wait_vm<i>();  \
    break;
  switch (n) {
    NBG_VMC(0) NBG_VMC(1) NBG_VMC(2) NBG_VMC(3) NBG_VMC(4) NBG_VMC(5) NBG_VMC(6) NBG_VMC(7)
    NBG_VMC(8) NBG_VMC(9) NBG_VMC(10) NBG_VMC(11) NBG_VMC(12) NBG_VMC(13) NBG_VMC(14) NBG_VMC(15)
    NBG_VMC(16) NBG_VMC(17) NBG_VMC(18) NBG_VMC(19) NBG_VMC(20) NBG_VMC(21) NBG_VMC(22) NBG_VMC(23)
    NBG_VMC(24) NBG_VMC(25) NBG_VMC(26) NBG_VMC(27) NBG_VMC(28) NBG_VMC(29) NBG_VMC(30)
    default:
      wait_vm<31>();
      break;
  }
#undef NBG_VMC
}

// Issue tile `t` (64 packets from tile base `tb`) into the LDS buffer at `buf`: instruction k
// covers packets 16k..16k+15.  48-B rows: lane l < 48 fetches chunk l % 3 of packet 16k + l / 3;
// 64-B rows: lane l fetches chunk l % 4 of packet 16k + l / 4 (1 KiB contiguous).  Lanes past the
// batch end fetch the batch base (their rows are never read).
template <uint32_t kRow, bool NT>
__device__ __forceinline__ void issue_tile(const ClassifyArgs& a, uint32_t tb, uint32_t buf, uint32_t lane) {
  constexpr uint32_t kCh = kRow / 16u;
  if (kCh == 4u || lane < 16u * kCh) {
    const uint32_t pk = lane / kCh, ch = lane - pk * kCh;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      const uint32_t p = tb + k * 16u + pk;
      const uint8_t* src = p < a.n_pkts ? a.pkts + static_cast<size_t>(p) * a.stride + ch * 16u : a.pkts;
      glds16_tile<NT>(src, buf + k * (16u * kRow));
    }
  }
}

template <bool HIST>
__device__ __forceinline__ void stream_flush(const ClassifyArgs& a, uint32_t* hist, uint32_t nbins, uint32_t part,
                                             uint32_t lane) {
  if constexpr (HIST) {
    if (a.hist16) {
      const uint32_t hw = (nbins + 1) >> 1;
      uint32_t* row = a.part_hist + static_cast<size_t>(part) * hw;
      for (uint32_t w = lane; w < hw; w += 64) {
        const uint32_t h = hist[2 * w] | (2 * w + 1 < nbins ? hist[2 * w + 1] << 16 : 0u);
        if (h) atomicAdd(&row[w], h);
      }
    } else {
      uint32_t* row = a.part_hist + static_cast<size_t>(part) * nbins;
      for (uint32_t b = lane; b < nbins; b += 64) {
        const uint32_t h = hist[b];
        if (h) atomicAdd(&row[b], h);
      }
    }
    for (uint32_t b = lane; b < nbins; b += 64) hist[b] = 0;
  }
}

// Classify one tile from its LDS ring buffer `x` (row of this lane's packet) and write the results.
// Returns the bin to count (histogram) through `bin`; false when the lane has no packet.
template <bool F4, int MODE, uint32_t kRow = row_of<MODE>(), bool WT = false>
__device__ __forceinline__ bool stream_classify(const ClassifyArgs& a, const uint8_t* lut, const uint8_t* x,
                                                uint32_t p, uint32_t& bin_out, bool& slow_out) {
  const bool valid = p < a.n_pkts;
  const uint4 c0 = *reinterpret_cast<const uint4*>(x);
  const uint4 c1 = *reinterpret_cast<const uint4*>(x + 16);
  const uint2 c2 = *reinterpret_cast<const uint2*>(x + 32);
  const bool fast = valid && ((c0.w >> 16) & 0xfu) == 5u;  // lean layout: aligned, frames >= 48 B
  // frame bytes: src 26..29, dst 30..33, ports 34..37, proto 23
  const uint32_t src = (c1.z >> 16) | (c1.w << 16);
  const uint32_t dst = (c1.w >> 16) | (c2.x << 16);
  const uint32_t ports = (c2.x >> 16) | (c2.y << 16);
  uint32_t lo, hi;
  fnv_flow(lo, hi, src, dst, ports, c1.y >> 24);
  const uint32_t idx = F4 ? mod_f4(lo, hi) : mod_barrett(lo, hi, a.m, a.mu);
  const uint32_t e = lut[idx & 0xffffu];
  bin_out = (idx >> 16) ? a.lut_tail : e;
  if constexpr (MODE == 1) {
    static_assert(kRow == 64, "the in-place swap writes whole slots back from 64-B rows");
    // whole-line write-back from the tile's LDS rows: lane (quad, part) stores chunk `part` of packet
    // 16k + quad (1 KiB contiguous per instruction), chunk 0 with the MACs swapped; a packet off
    // the fast path keeps its chunk 0 for the byte-wise path
    const uint8_t* tile = x - (p & 63u) * kRow;
    const uint32_t part = p & 3u, quad = (p & 63u) >> 2;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      const uint32_t q = (p & ~63u) + k * 16u + quad;
      uint4 v = *reinterpret_cast<const uint4*>(tile + (k * 16u + quad) * kRow + part * 16u);
      // the quad's chunk-0 lane holds bytes 12..15 (IHL)
      const uint32_t w3 = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v.w), 0x00, 0xf, 0xf, false));
      const bool qfast = q < a.n_pkts && ((w3 >> 16) & 0xfu) == 5u;
      if (part == 0u)
        v = make_uint4((v.y >> 16) | (v.z << 16), (v.z >> 16) | (v.x << 16), (v.x >> 16) | (v.y << 16), v.w);
      if (qfast) {
        if constexpr (WT) stg16_wt(a.pkts + static_cast<size_t>(q) * a.stride + part * 16u, v);
        else stg16_nt(a.pkts + static_cast<size_t>(q) * a.stride + part * 16u, v);
      }
    }
  } else if constexpr (MODE == 2) {
    if (fast) {
      uint32_t* mo = reinterpret_cast<uint32_t*>(a.mac_out + static_cast<size_t>(p) * 12u);
      mo[0] = (c0.y >> 16) | (c0.z << 16);
      mo[1] = (c0.z >> 16) | (c0.x << 16);
      mo[2] = (c0.x >> 16) | (c0.y << 16);
    }
  }
  slow_out = valid && !fast;
  return valid;
}

// The packet's backend (and its slow path, after the tile's next loads are issued).
template <bool F4>
__device__ __forceinline__ uint32_t stream_finish(const ClassifyArgs& a, const uint8_t* lut, uint32_t p, uint32_t bin,
                                                  bool slow) {
  if (slow) {
    uint32_t gate;
    bin = classify_slow<kLdsU8Tail, F4, false, true>(a, lut, a.pkts + static_cast<size_t>(p) * a.stride, a.fixed_len,
                                                     p, gate);
  }
  a.backend[p] = static_cast<uint16_t>(bin == a.nb ? kSentinel : bin);
  return bin;
}

// 4 or 2 B per lane from `src` into LDS at m0 + lane * 4.
__device__ __forceinline__ void glds4(const void* src, uint32_t lds_base) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dword %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds_base))
      : "memory");
}
__device__ __forceinline__ void glds2(const void* src, uint32_t lds_base) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_ushort %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds_base))
      : "memory");
}


// Lagged grouping (NBG_GROUP_LAG, GB > 0: the multisplit's bin bits): besides classifying its batch,
// the launch groups the handle's pending batch `lg` (classified by the previous launch, whose
// partition rows are complete).  Block c owns partition c: a prologue sums the rows into the
// partition's per-bin perm bases (group base + prefix over earlier partitions, as group_kernel's),
// then at every unit step each wave ranks 64 packets of the next 512-packet piece of the partition
// (ballot multisplit), the unit's existing LDS barrier publishes the per-wave bin counts, and every
// lane stores perm[base + run + earlier waves' counts + rank] = its packet: the stable per-group FIFO
// order of group_by.rs:46-51.  Pieces beyond the unit steps run after them.  A piece's backends
// arrive by LDS-DMA with the tile of its step (counted in `seq`), so grouping never drains the tile
// ring.  The launch then zeroes the lag histogram buffer the launch after next accumulates into
// (three buffers rotate: classify into one, group from the previous one, zero the third).
constexpr uint32_t kLagPiece = 64u * kStreamW;  // packets per piece (one 64-packet rank per wave)
constexpr uint32_t kLagSlots = 3;                // backend pieces per wave: steps k, k+1, k+2

// LDS words of the lag state past the block histograms (hstride = (nbins + 3) & ~3):
// base[hs], tot[hs], run[2][hs], cnt[2][kStreamW][hs], pbs[2][hs] (a piece's bin starts),
// kStreamW * kLagSlots pieces of 64 dwords, the block scan's per-wave sums, and srt[2][kLagPiece]
// (pos, packet) pairs of a piece sorted by bin (dynamic LDS only: the kernel may take all 160 KiB)
__host__ __device__ constexpr uint32_t lag_lds_words(uint32_t hstride) {
  return hstride * (6u + 2u * kStreamW) + kStreamW * kLagSlots * 64u + kStreamW + 2u * kLagPiece * 2u;
}

// MODE: 0 = read only, 1 = MAC swap in place, 2 = swapped MACs as 12-B records (a.mac_out)
// sb: the batches of this launch (one for nbg_maglev_classify_device; up to kMaxMulti for
// nbg_maglev_classify_device_multi).  `a` carries what they share; per unit, the unit's batch
// supplies pkts, n_pkts, backend, mac_out and part_hist (a view of `a`).  GB > 0: one batch, plus
// the lagged grouping of lg (above).
template <bool F4, bool HIST, int MODE, int GB = 0>
__global__ __launch_bounds__(kStreamNT, 1) void classify_stream_kernel(ClassifyArgs a, StreamBatches sb, LagGroup lg) {
  constexpr uint32_t kRow = stream_row_of<MODE>(), kTileLds = 64u * kRow;
  static_assert(GB == 0 || HIST, "lagged grouping runs on the per-unit histogram barrier");
  extern __shared__ __align__(16) uint8_t smem[];
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t nbins = a.nb + 1;
  uint8_t* lut = smem;
  uint8_t* ring = smem + kLutLds + wave * (kRing * kTileLds);
  const uint32_t hstride = (nbins + 3) & ~3u;
  uint32_t* hist_base = reinterpret_cast<uint32_t*>(smem + kLutLds + kStreamW * kRing * kTileLds);
  const uint32_t ring_lds = __builtin_amdgcn_readfirstlane(lds_addr(ring));
  const uint32_t lut_lds = __builtin_amdgcn_readfirstlane(lds_addr(lut));
  // Interleaved units: unit u = tiles [u*W, u*W + W), one per wave; block b takes units b, b + G,
  // b + 2G, ...  At any moment the grid reads consecutive units: one sequential sweep of the batch
  // (contiguous per-wave runs read ~3k streams at a fixed stride and measured 10 % slower:
  // HBM channel imbalance).  The block's histogram is double-buffered per unit and flushed by one
  // wave behind one LDS-only barrier; a unit (W tiles = 512 packets) never straddles a partition.
  const uint32_t n_units = sb.unit_base[sb.n];
  const uint32_t G = gridDim.x, b = blockIdx.x;
  const uint32_t nt = b < n_units ? (n_units - b + G - 1) / G : 0u;  // units of this block (block-uniform)
  // position k: global unit b + k*G; its batch j (scalar search, block-uniform) and the unit's
  // first packet within the batch
  // A cursor over the batches: units [lo, hi) are batch j's.  Positions visit increasing units, so
  // a cursor only moves forward, at most n - 1 times per block: the kernel arguments are read at a
  // batch change only.  Measured (rocprof, 4 x 1M per launch, profiles/r02_multi_batch_rocprof.txt):
  // read-only 45.7 us with the cursor against 52.7 us with a per-unit search of the argument arrays.
  struct Cursor {
    uint32_t j, lo, hi;
    ClassifyArgs v;
  };
  auto load = [&](Cursor& c, uint32_t j) {
    c.j = j;
    c.lo = sb.unit_base[j];
    c.hi = sb.unit_base[j + 1];
    c.v = a;
    c.v.pkts = sb.pkts[j];
    c.v.n_pkts = sb.n_pkts[j];
    c.v.backend = sb.backend[j];
    c.v.mac_out = sb.mac_out[j];
    c.v.part_hist = sb.part_hist[j];
  };
  auto seek = [&](Cursor& c, uint32_t u) {
    if (u < c.hi) return;
    uint32_t jj = c.j + 1;
    while (jj + 1 < sb.n && u >= sb.unit_base[jj + 1]) ++jj;
    load(c, jj);
  };
  auto first_pkt = [&](const Cursor& c, uint32_t u) { return ((u - c.lo) * kStreamW + wave) * 64u; };
  Cursor cur, nxt;  // the unit being classified; the unit whose tile is issued
  load(cur, 0);
  load(nxt, 0);
  uint32_t* hist = hist_base;  // [2][hstride]
  // GB == 0: the wave's 64 backend words for the packed backend[] stores, past the histograms
  uint16_t* rep = reinterpret_cast<uint16_t*>(hist_base + 2u * hstride) + wave * 64u;

  // lagged grouping state (GB > 0): this block's partition [pbeg, pend) of the pending batch, its
  // 512-packet pieces, and the LDS words past the block histograms
  uint32_t* g_base = hist_base + 2 * hstride;   // [hstride] perm base of every bin for this partition
  uint32_t* g_tot = g_base + hstride;           // [hstride] prologue scratch: bin totals
  uint32_t* g_run = g_tot + hstride;            // [2][hstride] bin counts of earlier pieces
  uint32_t* g_cnt = g_run + 2 * hstride;        // [2][kStreamW][hstride] per-wave counts of a piece
  uint32_t* g_pbs = g_cnt + 2 * kStreamW * hstride;  // [2][hstride] where each bin starts in a sorted piece
  uint32_t* g_bk = g_pbs + 2 * hstride;         // [kStreamW][kLagSlots][64] backends (one dword per lane)
  uint32_t* s_wave = g_bk + kStreamW * kLagSlots * 64u;  // [kStreamW] block scan
  uint2* g_srt = reinterpret_cast<uint2*>(s_wave + kStreamW);  // [2][kLagPiece] (perm position, packet)
  const uint32_t bk_lds = GB > 0 ? __builtin_amdgcn_readfirstlane(lds_addr(g_bk + wave * kLagSlots * 64u)) : 0u;
  const bool g_own = GB > 0 && b < lg.n_parts;  // block-uniform
  const uint32_t pbeg = g_own ? b * lg.part_pkts : 0u;
  const uint32_t pend = g_own ? min(pbeg + lg.part_pkts, lg.n_pkts) : 0u;
  const uint32_t pieces = g_own && lg.perm ? (pend - pbeg + kLagPiece - 1) / kLagPiece : 0u;
  const bool pro = g_own && (lg.perm || b == 0);  // block-uniform; counts from block 0

  // Prologue loads (GB > 0): this partition's per-bin perm base (group base + prefix over earlier
  // partitions) is summed straight from the pending batch's partition rows (group_kernel's direct
  // scan): L threads per row word, each over rows j, j + L, ...  The first kPU rows of every thread
  // are loaded here, before the LUT pieces and the first tiles, so they retire first: the compiler's
  // waits for them (it does not see the LDS-DMA loads) never wait for the tile ring.
  constexpr uint32_t kPU = GB > 0 ? 32u : 1u;
  const uint32_t rw = lg.hist16 ? (nbins + 1) >> 1 : nbins;  // words per row
  const uint32_t pL = rw >= kStreamNT ? 1u : kStreamNT / rw;
  const uint32_t pw = tid % rw, pj = tid / rw;
  const bool pthr = pro && tid < rw * pL;
  uint32_t ph[kPU];
  if constexpr (GB > 0) {
    if (pthr) {
#pragma unroll
      for (uint32_t k = 0; k < kPU; ++k) ph[k] = ld_u32(lg.part_hist, (min(pj + k * pL, lg.n_parts - 1u) * rw + pw) * 4u);
    }
  }

  // LUT staging: lut_lds_bytes (a multiple of 1 KiB, <= 64 KiB) in 1-KiB pieces over the block's
  // waves (the device LUT is padded to whole pieces); the first tiles go out behind them
  const uint32_t pieces_lut = a.lut_lds_bytes >> 10;
  const uint32_t first = min(nt, static_cast<uint32_t>(kRing));
  // the LUT pieces first, then the first tiles (measured: tiles first, or the LUT through registers
  // off the LDS-DMA path, are both ~0.8 us slower per launch)
  for (uint32_t q = wave; q < pieces_lut; q += kStreamW)
    glds16(static_cast<const uint8_t*>(a.lut) + q * 1024u + lane * 16u, lut_lds + q * 1024u);
  // VM operations this wave issued after the LUT pieces (tile loads, and a lower bound of its
  // stores): waiting for tile k is vmcnt(seq - its count), so the stores issued after a tile do not
  // make the wait for it stricter (vmcnt counts stores too)
  uint32_t seq = 0, sA = 0, sB = 0, sC = 0;  // counts after tiles k, k+1, k+2
  // lagged grouping: piece q's 64 backends of this wave, one dword per lane (a 2-B LDS-DMA fills a
  // dword), into slot q % kLagSlots; issued just before the tile of step q, so waiting for that
  // tile covers it.  One instruction (counted) when the wave has packets in the piece.
  auto issue_piece = [&](uint32_t q) {
    if constexpr (GB > 0) {
      const uint32_t i0 = pbeg + q * kLagPiece + wave * 64u;
      if (q < pieces && i0 < pend) {
        const uint32_t i = min(i0 + lane, pend - 1u);
        glds2(lg.backend + i, bk_lds + (q % kLagSlots) * 256u);
        ++seq;
      }
    }
  };
  for (uint32_t k = 0; k < first; ++k) {
    const uint32_t u = b + k * G;
    seek(nxt, u);
    issue_piece(k);
    issue_tile<kRow, MODE != 2>(nxt.v, first_pkt(nxt, u), ring_lds + k * kTileLds, lane);
    seq += 4;
    (k == 0 ? sA : (k == 1 ? sB : sC)) = seq;
  }
  if constexpr (HIST)
    for (uint32_t i = tid; i < 2 * hstride; i += kStreamNT) hist[i] = 0;
  if constexpr (GB > 0) {
    if (pro) {  // the sums, while the LUT pieces and the first tiles are in flight
      for (uint32_t i = tid; i < hstride; i += kStreamNT) {
        g_base[i] = 0;
        g_tot[i] = 0;
        g_run[i] = 0;
      }
      lds_sync();
      const uint32_t c = b;
      if (pthr) {
        uint32_t pre_lo = 0, pre_hi = 0, all_lo = 0, all_hi = 0;
        auto add = [&](uint32_t q, uint32_t h) {
          const uint32_t lo = !lg.hist16 ? h : (h & 0xffffu), hi = lg.hist16 ? h >> 16 : 0u;
          const bool in = q < lg.n_parts;
          all_lo += in ? lo : 0u;
          all_hi += in ? hi : 0u;
          pre_lo += in && q < c ? lo : 0u;
          pre_hi += in && q < c ? hi : 0u;
        };
#pragma unroll
        for (uint32_t k = 0; k < kPU; ++k) add(pj + k * pL, ph[k]);
        for (uint32_t q = pj + kPU * pL; q < lg.n_parts; q += pL)  // rows past the first kPU (rare)
          add(q, ld_u32(lg.part_hist, (q * rw + pw) * 4u));
        const uint32_t b0 = lg.hist16 ? 2 * pw : pw;
        if (pre_lo) atomicAdd(&g_base[b0], pre_lo);
        if (all_lo) atomicAdd(&g_tot[b0], all_lo);
        if (lg.hist16 && b0 + 1 < nbins) {
          if (pre_hi) atomicAdd(&g_base[b0 + 1], pre_hi);
          if (all_hi) atomicAdd(&g_tot[b0 + 1], all_hi);
        }
      }
      lds_sync();
      // group bases: exclusive scan of the totals over bins (<= 2^GB bins: <= 512 = one per thread)
      static_assert((1u << GB) <= kStreamNT, "one bin per thread in the group-base scan");
      const uint32_t t = tid < nbins ? g_tot[tid] : 0u;
      uint32_t all;
      const uint32_t gb = block_excl_scan_n<kStreamNT>(t, s_wave, all);
      if (tid < nbins) {
        if (c == 0 && lg.counts) lg.counts[tid] = t;
        g_base[tid] += gb;
      }
    }
  }
  // this wave's LUT pieces are in when at most its tile loads are outstanding; then the barrier
  // makes every wave's pieces visible to every wave
  wait_tile(first);
  lds_sync();

  // Lagged grouping of piece q runs across three barriers, so that every barrier the unit loop already
  // has carries it (sync point s = the loop step, then tail barriers):
  //   before barrier q:  rank the wave's 64 packets (ballot multisplit), publish the wave's bin counts
  //   after barrier q:   each packet's perm position (base + earlier pieces + earlier waves + rank);
  //                      one wave: the next piece's running counts and this piece's bin starts (pbs)
  //   after barrier q+1: each packet's slot in the piece sorted by bin (pbs + earlier waves + rank)
  //   after barrier q+2: thread t stores sorted slot t: consecutive threads write consecutive perm
  //                      entries of one bin (coalesced), where lane-order stores scattered every lane
  uint32_t g_bin = 0, g_rank = 0;    // piece q (ranked, before barrier q)
  bool g_valid = false;
  uint32_t p_pos = 0, p_bin = 0, p_pre = 0;  // piece q-1 (positioned, after barrier q-1)
  bool p_valid = false;
  auto piece_rank = [&](uint32_t q) {  // before barrier q
    if constexpr (GB > 0) {
      const uint32_t i = pbeg + q * kLagPiece + wave * 64u + lane;
      g_valid = i < pend;
      const uint32_t raw = g_bk[(wave * kLagSlots + q % kLagSlots) * 64u + lane] & 0xffffu;
      g_bin = g_valid ? (raw == NBG_SENTINEL ? a.nb : raw) : 0u;
      uint32_t count;
      wave_match_rank<GB>(g_bin, g_valid, lane, g_rank, count);
      uint32_t* row = g_cnt + ((q & 1u) * kStreamW + wave) * hstride;
      for (uint32_t j = lane; j < hstride; j += 64) row[j] = 0;
      __builtin_amdgcn_wave_barrier();
      if (g_valid) row[g_bin] = count;  // every lane of a bin stores the same count
    }
  };
  auto piece_sync = [&](uint32_t s) {  // after barrier s
    if constexpr (GB > 0) {
      // piece s-2: coalesced stores of its sorted slots
      if (s >= 2 && s - 2 < pieces) {
        const uint32_t q = s - 2, n_q = min(pend - (pbeg + q * kLagPiece), kLagPiece);
        const uint2 e = g_srt[(q & 1u) * kLagPiece + tid];
        if (tid < n_q && e.x < lg.n_pkts) lg.perm[e.x] = e.y;
        if (wave * 64u < n_q) ++seq;  // lane 0 stored
      }
      // piece s-1: its sorted slot
      if (s >= 1 && s - 1 < pieces && p_valid) {
        const uint32_t q = s - 1;
        const uint32_t slot = g_pbs[(q & 1u) * hstride + p_bin] + p_pre;
        g_srt[(q & 1u) * kLagPiece + slot] = make_uint2(p_pos, pbeg + q * kLagPiece + wave * 64u + lane);
      }
      // piece s: perm positions; one wave: running counts and bin starts
      if (s < pieces) {
        const uint32_t* cq = g_cnt + (s & 1u) * kStreamW * hstride;
        uint32_t pre = g_rank;
#pragma unroll
        for (uint32_t w = 0; w < kStreamW; ++w)
          if (w < wave) pre += cq[w * hstride + g_bin];
        p_pos = g_base[g_bin] + g_run[(s & 1u) * hstride + g_bin] + pre;
        p_bin = g_bin;
        p_pre = pre;
        p_valid = g_valid;
        if (wave == (s + kStreamW / 2) % kStreamW) {
          constexpr uint32_t kB = (1u << GB) / 64u;  // consecutive bins per lane
          uint32_t pc[kB], tot = 0;
#pragma unroll
          for (uint32_t i = 0; i < kB; ++i) {
            const uint32_t bn = lane * kB + i;
            uint32_t v = 0;
            if (bn < nbins) {
#pragma unroll
              for (uint32_t w = 0; w < kStreamW; ++w) v += cq[w * hstride + bn];
              g_run[((s + 1) & 1u) * hstride + bn] = g_run[(s & 1u) * hstride + bn] + v;
            }
            pc[i] = v;
            tot += v;
          }
          uint32_t st = wave_incl_scan(tot) - tot;
#pragma unroll
          for (uint32_t i = 0; i < kB; ++i) {
            const uint32_t bn = lane * kB + i;
            if (bn < nbins) g_pbs[(s & 1u) * hstride + bn] = st;
            st += pc[i];
          }
        }
      } else {
        p_valid = false;
      }
    }
  };

  for (uint32_t k = 0; k < nt; ++k) {
    const uint32_t u = b + k * G;
    seek(cur, u);
    const ClassifyArgs& aj = cur.v;
    const uint32_t tb = first_pkt(cur, u);
    wait_vm_n(seq - sA);  // kStreamAhead tiles (and their stores) stay in flight
    const uint32_t p = tb + lane;
    uint32_t bin = 0;
    bool slow = false;
    const bool valid = tb < aj.n_pkts && stream_classify<F4, MODE, kRow>(aj, lut, ring + (k % kRing) * kTileLds + lane * kRow,
                                                                    p, bin, slow);
    // tile k + kRing into the buffer just read (its ds_reads are consumed above): while the next
    // tile is classified, kStreamAhead tiles stay in flight
    uint32_t sN = 0;
    if (k + kRing < nt) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const uint32_t u2 = u + kRing * G;
      seek(nxt, u2);
      issue_piece(k + kRing);
      issue_tile<kRow, MODE != 2>(nxt.v, first_pkt(nxt, u2), ring_lds + (k % kRing) * kTileLds, lane);
      seq += 4;
      sN = seq;
    }
    if constexpr (GB == 0) {
      // backend[]: a whole tile's 128 B go out as 16-B stores of lanes 0..7 (through the wave's LDS
      // words, as the ring kernel does) instead of 64 2-B stores: in place 93.2-93.8 against
      // 94.0-94.5 us per 4 x 1M launch (profiles/r05_stream_pack_ab.txt)
      uint32_t be = 0;
      if (valid) {
        if (slow) {
          uint32_t gate;
          bin = classify_slow<kLdsU8Tail, F4, false, true>(aj, lut, aj.pkts + static_cast<size_t>(p) * aj.stride,
                                                           aj.fixed_len, p, gate);
        }
        be = bin == aj.nb ? kSentinel : bin;
        if constexpr (HIST) atomicAdd(&hist[(k & 1u) * hstride + bin], 1u);
      }
      if (tb + 64u <= aj.n_pkts && (reinterpret_cast<uintptr_t>(aj.backend) & 15u) == 0) {
        rep[lane] = static_cast<uint16_t>(be);
        asm volatile("" ::: "memory");  // the u16 writes before the 16-B reads of the same words
        __builtin_amdgcn_wave_barrier();
        const uint4 w = reinterpret_cast<const uint4*>(rep)[lane & 7u];
        if (lane < 8u) *reinterpret_cast<uint4*>(aj.backend + tb + lane * 8u) = w;
      } else if (valid) {
        aj.backend[p] = static_cast<uint16_t>(be);
      }
    } else if (valid) {
      bin = stream_finish<F4>(aj, lut, p, bin, slow);
      if constexpr (HIST) atomicAdd(&hist[(k & 1u) * hstride + bin], 1u);
    }
    if (tb < aj.n_pkts) ++seq;  // the backend store (one instruction; lane 0 has a packet)
    if (k < pieces) piece_rank(k);
    sA = sB;
    if constexpr (kRing == 2) {
      sB = sN;
    } else {
      sB = sC;
      sC = sN;
    }
    if constexpr (HIST) {
      // every wave's counts of unit k are in hist[k & 1]; one wave flushes it into the unit's
      // partition row and zeroes it.  The next barrier (unit k + 1) orders that before unit k + 2
      // counts into the same buffer.
      lds_sync();
      if (wave == k % kStreamW) {
        uint32_t* h = hist + (k & 1u) * hstride;
        stream_flush<HIST>(aj, h, nbins, ((u - cur.lo) * kStreamW * 64u) / a.part_pkts, lane);
      }
    }
    piece_sync(k);
  }
  if constexpr (GB > 0) {
    // sync points past the unit steps: pieces beyond them (a pending batch larger than this one),
    // then the last two pieces' sorted slots and stores
    {
      for (uint32_t s = nt; s < pieces + 2; ++s) {
        if (s < pieces) {
          issue_piece(s);
          wait_vm<0>();
          piece_rank(s);
        }
        lds_sync();
        piece_sync(s);
      }
    }
    for (uint32_t i = b * kStreamNT + tid; i < lg.zero_words; i += G * kStreamNT) lg.zero[i] = 0;
  }
}

// ---- persistent RX-ring classify (nbg_ring_*) ----------------------------------------------------
//
// One launch per ring for the whole run: the RX ring that never stops (ReceiveBatch polling its port,
// framework/src/operators/receive_batch.rs:26,52-61).  Same blocks, LUT staging, LDS-DMA tile ring
// and interleaved 512-packet units as classify_stream_kernel, but the unit sequence is open-ended:
// batch j covers units [ulo_j, uhi_j) of one sequence, block b takes units b, b + G, b + 2G, ... of
// it, and batches arrive through a descriptor ring in pinned host memory while the kernel runs.  So
// the LUT is staged once per ring and the tile pipeline runs across batch boundaries without a
// ramp.
//
//   Descriptors.  The control wave (the ninth) of every block keeps up to kRingCache batch
//   descriptors in LDS.  It prefetches the next kRingFetch slots of its replica of the device ring
//   (uncached HBM, filled from the host's ring by the relay block, ring_relay) by LDS-DMA; a slot is taken
//   once its seq and check match (a read that overlaps the relay rewriting the slot fails the check
//   and is retried).  The count of known batches is published through a step-parity LDS word behind
//   the unit barrier, so every wave sees the same count.  When the block has no tile to classify
//   (the next unit is in no known batch) it drains and the control wave polls the slot (and the
//   device stop word) with s_sleep between polls: the idle path.  No classify CU reads host memory.
//   Exit: stop set and nothing posted, or idle_ticks without a new batch (the exit condition every
//   wave reaches when the host goes away).
//
//   Completion.  Outputs are stored write-through (sc1: backend[] packed 16 B per lane, the in-place
//   windows 16 B per lane), so a store that retired is in HBM.  In-order vmcnt: once every wave has
//   waited for tile k (the unit barrier of step k), the stores of steps <= k - 3 retired.  The
//   control wave then publishes, per block, the count of batches all of whose units of this block
//   are complete (to uncached HBM, when the count changes); the relay reports the minimum to the host.
constexpr uint32_t kRingCache = 4;  // batch descriptors in LDS (from the current unit's batch on)
constexpr uint32_t kRingFetch = 2;  // ring slots per prefetch (one LDS-DMA dword load, 32 lanes)
constexpr uint32_t kRingCtlWords = kRingCache * 16u + kRingFetch * 16u + 4u + kStreamW * 32u + 16u;

__device__ __forceinline__ void glds4_sys(const void* src, uint32_t lds_base) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dword %1, off sc0 sc1\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds_base))
      : "memory");
}

__device__ __forceinline__ uint32_t rfl(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }


// The ring kernel's cursor over the known batches (block-uniform; loaded from the LDS descriptor cache)
struct RingCursor {
  uint32_t j;  // batch index (0xffffffff: none yet)
  uint64_t lo, hi;
  uint8_t* pkts;
  uint16_t* backend;
  uint32_t n;
};

__device__ __forceinline__ void ring_load(RingCursor& c, const uint32_t* cache, uint32_t j) {
  const uint32_t* e = cache + (j % kRingCache) * 16u;
  c.j = j;
  c.pkts = reinterpret_cast<uint8_t*>(static_cast<uintptr_t>(rfl(e[0])) | static_cast<uintptr_t>(rfl(e[1])) << 32);
  c.backend = reinterpret_cast<uint16_t*>(static_cast<uintptr_t>(rfl(e[2])) | static_cast<uintptr_t>(rfl(e[3])) << 32);
  c.lo = static_cast<uint64_t>(rfl(e[4])) | static_cast<uint64_t>(rfl(e[5])) << 32;
  c.hi = static_cast<uint64_t>(rfl(e[6])) | static_cast<uint64_t>(rfl(e[7])) << 32;
  c.n = rfl(e[8]);
}

// Move c forward to the batch holding unit u; false when u lies past the known batches.
__device__ __forceinline__ bool ring_seek(RingCursor& c, const uint32_t* cache, uint64_t u, uint32_t known) {
  while (u >= c.hi) {
    const uint32_t nj = c.j + 1u;
    if (static_cast<int32_t>(nj - known) >= 0) return false;
    ring_load(c, cache, nj);
  }
  return true;
}

// Take the staged descriptor d (every lane reads its 16 words) as batch known_w if it is that batch
// (seq and check match) and the cache has room past `base` (the oldest batch a cursor may still load).
__device__ __forceinline__ bool ring_take(const uint32_t* d, uint32_t* cache, uint32_t& known_w, uint32_t base,
                                          uint32_t lane) {
  const uint4 w0 = *reinterpret_cast<const uint4*>(d), w1 = *reinterpret_cast<const uint4*>(d + 4);
  const uint4 w2 = *reinterpret_cast<const uint4*>(d + 8), w3 = *reinterpret_cast<const uint4*>(d + 12);
  const uint64_t pk = w0.x | static_cast<uint64_t>(w0.y) << 32, be = w0.z | static_cast<uint64_t>(w0.w) << 32;
  const uint64_t lo = w1.x | static_cast<uint64_t>(w1.y) << 32, hi = w1.z | static_cast<uint64_t>(w1.w) << 32;
  const uint64_t ck = w3.z | static_cast<uint64_t>(w3.w) << 32;
  const bool ok = w2.y == known_w + 1u && ck == ring_check(pk, be, lo, hi, w2.x, w2.y) && known_w - base < kRingCache;
  if (!rfl(ok ? 1u : 0u)) return false;
  // copy the words just checked (d may be rewritten by a landing prefetch meanwhile)
  const uint4 q = (lane >> 2) == 0 ? w0 : ((lane >> 2) == 1 ? w1 : ((lane >> 2) == 2 ? w2 : w3));
  const uint32_t x = (lane & 3u) == 0 ? q.x : ((lane & 3u) == 1 ? q.y : ((lane & 3u) == 2 ? q.z : q.w));
  if (lane < 16) cache[(known_w % kRingCache) * 16u + lane] = x;
  ++known_w;
  return true;
}

// Batch j's descriptor in this block's replica of the ring.
__device__ __forceinline__ const RingDesc* ring_slot(const RingArgs& r, uint32_t j) {
  return r.desc + (blockIdx.x & (r.reps - 1u)) * r.slots + (j & (r.slots - 1u));
}

// Wave 0, idle: read ring slots (and the stop word) until a new batch is taken; true = exit (stop
// with nothing posted, or idle_ticks without a batch: then the error word is set).
__device__ __forceinline__ bool ring_poll(const RingArgs& r, uint32_t* stage, uint32_t* cache, uint32_t& known_w,
                                          uint32_t base, uint32_t lane) {
  const uint64_t t0 = wall_clock64();
  const uint32_t known0 = known_w;
  for (uint32_t nap = 1;; nap = min(2u * nap, 16u)) {
    for (;;) {  // every consecutive batch that is posted (and fits)
      const uint32_t* slot = reinterpret_cast<const uint32_t*>(ring_slot(r, known_w));
      if (lane < 16) stage[lane] = __hip_atomic_load(slot + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __builtin_amdgcn_wave_barrier();
      if (!ring_take(stage, cache, known_w, base, lane)) break;
    }
    if (known_w != known0) return false;
    if (rfl(__hip_atomic_load(r.dstop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM))) {
      // a batch posted before the stop is in its slot by now: look once more
      const uint32_t* slot = reinterpret_cast<const uint32_t*>(ring_slot(r, known_w));
      if (lane < 16) stage[lane] = __hip_atomic_load(slot + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __builtin_amdgcn_wave_barrier();
      return !ring_take(stage, cache, known_w, base, lane);
    }
    if (static_cast<uint64_t>(wall_clock64()) - t0 > r.idle_ticks) {
      if (lane == 0) __hip_atomic_store(&r.ctl->error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return true;
    }
    // back off to 16 x 512 clocks (~3.5 us) between polls of the (uncached) device ring
    for (uint32_t i = 0; i < nap; ++i) __builtin_amdgcn_s_sleep(8);
  }
}

// The ring's relay: wave 0 of the classify kernel's last block (the other waves of that block exit),
// so its PCIe reads of the host ring hold no classify CU.  (A separate one-wave kernel measured no
// good: blocks go to XCDs round-robin and never move, so the XCD that hosted it had one classify
// block too many for its CUs, and that block never became resident.)
// Loop: copy every newly posted host slot (seq and check match) into each replica of the uncached
// device ring; report the minimum of the blocks' completion counts to the host when it moves; on
// the host's stop, relay what was posted before it, then raise the device stop word and exit once
// every relayed batch is complete; on idle_ticks without a post or a completion, raise the device
// stop word and the host error word and exit (the exit every path reaches when the host goes away).
__device__ __forceinline__ void ring_relay(const RingArgs& r, uint32_t lane) {
  uint32_t known = 0, done = 0, nap = 1;
  bool stopping = false, stopped = false;
  uint64_t t_act = wall_clock64();
  for (;;) {
    bool moved = false;
    for (;;) {  // every consecutive posted slot
      const uint32_t* hs = reinterpret_cast<const uint32_t*>(r.hdesc + (known & (r.slots - 1u)));
      const uint32_t x = lane < 16u ? __hip_atomic_load(hs + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0u;
      uint32_t w[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) w[i] = __shfl(x, i);
      const uint64_t pk = w[0] | static_cast<uint64_t>(w[1]) << 32, be = w[2] | static_cast<uint64_t>(w[3]) << 32;
      const uint64_t lo = w[4] | static_cast<uint64_t>(w[5]) << 32, hi = w[6] | static_cast<uint64_t>(w[7]) << 32;
      const uint64_t ck = w[14] | static_cast<uint64_t>(w[15]) << 32;
      if (!(w[9] == known + 1u && ck == ring_check(pk, be, lo, hi, w[8], w[9]))) break;
      for (uint32_t q = lane >> 4; q < r.reps; q += 4u) {
        uint32_t* d = reinterpret_cast<uint32_t*>(r.desc + q * r.slots + (known & (r.slots - 1u)));
        __hip_atomic_store(d + (lane & 15u), __shfl(x, static_cast<int>(lane & 15u)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      }
      ++known;
      moved = true;
    }
    // completion: the slowest block
    uint32_t lag = 0;
    for (uint32_t b = lane; b < r.grid; b += 64u)
      lag = max(lag, known - __hip_atomic_load(r.prog + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) lag = max(lag, static_cast<uint32_t>(__shfl_xor(static_cast<int>(lag), o)));
    const uint32_t c = known - rfl(lag);
    if (c != done) {
      done = c;
      if (lane == 0) {
        __hip_atomic_store(r.dcomp, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // the gate kernels
        __hip_atomic_store(&r.ctl->completed, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      moved = true;
    }
    if (moved) {
      t_act = wall_clock64();
      nap = 1;
      continue;
    }
    if (stopped) {
      if (done == known) break;  // every relayed batch is complete; the blocks exit on the stop word
    } else if (rfl(__hip_atomic_load(&r.ctl->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM))) {
      if (stopping) {
        // the slots were read once more after the stop was seen: everything posted before it is
        // relayed; the descriptors are in memory before the stop word
        wait_vm<0>();
        if (lane == 0) __hip_atomic_store(r.dstop, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        stopped = true;
        continue;
      }
      stopping = true;
      continue;
    }
    if (static_cast<uint64_t>(wall_clock64()) - t_act > r.idle_ticks) {
      if (lane == 0) {
        __hip_atomic_store(r.dstop, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (done != known || !stopped) __hip_atomic_store(&r.ctl->error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      break;
    }
    for (uint32_t i = 0; i < nap; ++i) __builtin_amdgcn_s_sleep(4);
    nap = min(2u * nap, 8u);
  }
}

constexpr int kRingNT = kStreamNT + 64;  // the tile waves plus the control wave

template <bool F4, int MODE>
__global__ __launch_bounds__(kRingNT, 1) void classify_ring_kernel(ClassifyArgs a, RingArgs r) {
  static_assert(MODE == 0 || MODE == 1, "the ring classifies read only or in place");
  constexpr uint32_t kRow = stream_row_of<MODE>(), kTileLds = 64u * kRow;
  extern __shared__ __align__(16) uint8_t smem[];
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const uint32_t wave = rfl(tid >> 6);
  // the control wave (the last) fetches descriptors, publishes completion and polls when idle: its
  // PCIe reads are in no tile wave's vmcnt, so a slow read never holds a tile wait
  const bool ctl = wave == static_cast<uint32_t>(kStreamW);
  uint8_t* lut = smem;
  uint8_t* ring = smem + kLutLds + (ctl ? 0u : wave) * (kRing * kTileLds);
  uint32_t* cache = reinterpret_cast<uint32_t*>(smem + kLutLds + kStreamW * kRing * kTileLds);  // [kRingCache][16]
  uint32_t* stage = cache + kRingCache * 16u;   // [kRingFetch][16] the control wave's prefetch landing area
  uint32_t* known_l = stage + kRingFetch * 16u;  // [2] known batches, by step parity; [2] exit
  uint16_t* rep = reinterpret_cast<uint16_t*>(known_l + 4) + (ctl ? 0u : wave) * 64u;  // a tile wave's 64 backends
  const uint32_t ring_lds = rfl(lds_addr(ring)), lut_lds = rfl(lds_addr(lut)), stage_lds = rfl(lds_addr(stage));
  if (blockIdx.x == r.grid) {  // the relay block
    if (wave == 0) ring_relay(r, lane);
    return;
  }
  const uint32_t G = r.grid, b = blockIdx.x;
  const uint32_t pieces_lut = ctl ? 0u : a.lut_lds_bytes >> 10;
  for (uint32_t q = wave; q < pieces_lut; q += kStreamW)
    glds16(static_cast<const uint8_t*>(a.lut) + q * 1024u + lane * 16u, lut_lds + q * 1024u);
  if (tid < 4) known_l[tid] = 0;
  wait_vm<0>();
  lds_sync();

  // cursors (every wave keeps them): the unit being classified, and the unit whose tile is issued
  RingCursor cur{0xffffffffu, 0, 0, nullptr, nullptr, 0}, nxt = cur;
  const uint64_t Gu = G;
  uint32_t k = 0, iss = 0;                   // unit steps of this block classified / issued
  uint32_t seq = 0, sA = 0, sB = 0, sC = 0;  // VM operations issued; counts after tiles k, k+1, k+2
  // the control wave's descriptor state
  uint32_t known_w = 0, pf_base = 0, last_pf = 0, pub = 0;
  bool pf = false;
  uint32_t hA = 0xffffffffu, hB = 0xffffffffu, hC = 0xffffffffu;  // batch of the unit of steps k - 1, k - 2, k - 3
  // a step's backends are stored one step late, behind the next tile issue: the wait for a tile then
  // covers the write-through stores of four steps back, not three, so their longer acks stay off the
  // critical path
  uint4 pw = make_uint4(0, 0, 0, 0);
  uint16_t* pp = nullptr;
  bool pend = false;

// the tile of unit step `t` into ring buffer t % kRing (the issue cursor moves to its batch; the
// control wave only moves its cursor)
#define RING_ISSUE(t, ok)                                                                                    \
  {                                                                                                         \
    const uint64_t u_ = b + static_cast<uint64_t>(t) * Gu;                                                  \
    ok = ring_seek(nxt, cache, u_, known);                                                                  \
    if (ok) {                                                                                               \
      if (!ctl) {                                                                                           \
        ClassifyArgs v_ = a;                                                                                \
        v_.pkts = nxt.pkts;                                                                                 \
        v_.n_pkts = nxt.n;                                                                                  \
        issue_tile<kRow, true>(v_, static_cast<uint32_t>(((u_ - nxt.lo) * kStreamW + wave) * 64u),         \
                               ring_lds + (rfl(t) % kRing) * kTileLds, lane);                               \
        seq += 4;                                                                                           \
        const uint32_t d_ = (t) - k;                                                                        \
        if (d_ == 0) sA = seq;                                                                              \
        else if (d_ == 1) sB = seq;                                                                         \
        else sC = seq;                                                                                      \
      }                                                                                                     \
      ++iss;                                                                                                \
    }                                                                                                       \
  }
// batches < v complete for this block (the control wave; one system-scope store when the count moves)
#define RING_PUBLISH(v)                                                                                      \
  {                                                                                                         \
    const uint32_t v_ = (v);                                                                                \
    if (static_cast<int32_t>(v_ - pub) > 0) {                                                               \
      pub = v_;                                                                                             \
      if (lane == 0) __hip_atomic_store(r.prog + b, v_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);       \
    }                                                                                                       \
  }
// take what has landed of the control wave's prefetch (the LDS-DMA may still be in flight: a slot not
// yet landed, torn, or not yet posted fails ring_take's seq / check test and is fetched again)
#define RING_TAKE_STAGED(base)                                                                               \
  {                                                                                                         \
    uint32_t i_ = 0;                                                                                        \
    for (; i_ < kRingFetch && pf_base + i_ == known_w; ++i_)                                                \
      if (!ring_take(stage + i_ * 16u, cache, known_w, (base), lane)) break;                               \
    if (i_ == kRingFetch) pf = false;                                                                       \
  }

  for (;;) {
    const uint32_t known = rfl(known_l[k & 1u]);  // block-uniform: written before the last barrier
    for (bool ok = true; ok && iss < k + kRing;) RING_ISSUE(iss, ok)
    if (iss == k) {
      // nothing to classify: drain, then the control wave fetches descriptors (polling while none is
      // posted).  No issued unit waits for cur, so it takes nxt's place: the descriptor cache then
      // only keeps batches past the issue cursor (which has walked every known batch), and a block
      // with no unit in several small batches still gets room to take the next ones.
      cur = nxt;
      if (pend) {
        if (lane < 8u) stg16_wt(pp, pw);
        pend = false;
      }
      wait_vm<0>();
      lds_sync();
      if (ctl) {
        const uint32_t base = cur.j == 0xffffffffu ? 0u : cur.j;
        if (pf) {  // landed (vmcnt(0) above)
          RING_TAKE_STAGED(base)
          pf = false;
        }
        RING_PUBLISH(known)  // every unit of this block in batches < known is complete
        const bool ex = known_w == known && ring_poll(r, stage, cache, known_w, base, lane);
        if (lane == 0) {
          known_l[k & 1u] = known_w;
          known_l[2] = ex ? 1u : 0u;
        }
      }
      lds_sync();
      if (rfl(known_l[2])) break;
      continue;
    }
    const uint64_t u = b + static_cast<uint64_t>(k) * Gu;
    ring_seek(cur, cache, u, known);
    const uint32_t h0 = cur.j;
    if (ctl) {
      // descriptor prefetch: take what has landed, then fetch the next slots when the issue cursor
      // is within two batches of the known ones (again after 6 steps when they were not posted yet)
      if (pf) {
        const uint32_t kw0 = known_w;
        RING_TAKE_STAGED(cur.j)
        if (known_w == kw0 && k - last_pf >= 6u) {
          pf = false;
        }
      }
      if (!pf && known_w - cur.j < kRingCache && known_w - nxt.j <= 2u) {
        if (lane < 16u * kRingFetch) stage[lane] = 0u;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        pf_base = known_w;
        if (lane < 16u * kRingFetch)
          glds4_sys(reinterpret_cast<const uint32_t*>(ring_slot(r, known_w + lane / 16u)) + (lane & 15u), stage_lds);
        pf = true;
        last_pf = k;
      }
      if (lane == 0) known_l[(k + 1u) & 1u] = known_w;
    } else {
      wait_vm_n(seq - sA);
      ClassifyArgs v = a;
      v.pkts = cur.pkts;
      v.n_pkts = cur.n;
      v.backend = cur.backend;
      const uint32_t tb = static_cast<uint32_t>(((u - cur.lo) * kStreamW + wave) * 64u);
      const uint32_t p = tb + lane;
      uint32_t bin = 0;
      bool slow = false;
      const bool valid = tb < v.n_pkts && stream_classify<F4, MODE, kRow, true>(
                                              v, lut, ring + (k % kRing) * kTileLds + lane * kRow, p, bin, slow);
      if (iss == k + kRing) {  // the next tile into the buffer just read
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        bool ok;
        RING_ISSUE(iss, ok)
      }
      if (pend) {  // the previous step's backends
        if (lane < 8u) stg16_wt(pp, pw);
        ++seq;
        pend = false;
      }
      if (valid && slow) {
        uint32_t gate;
        bin = classify_slow<kLdsU8Tail, F4, false, true, true>(v, lut, v.pkts + static_cast<size_t>(p) * v.stride,
                                                               v.fixed_len, p, gate);
      }
      if (tb < v.n_pkts) {
        const uint16_t be = static_cast<uint16_t>(bin == a.nb ? kSentinel : bin);
        const uint32_t cnt = min(64u, v.n_pkts - tb);
        if (cnt == 64u) {  // 16 B per lane: lanes 0..7 store the wave's 128 B (next step)
          rep[lane] = be;
          asm volatile("" ::: "memory");  // the u16 writes before the 16-B reads of the same words
          __builtin_amdgcn_wave_barrier();
          pw = reinterpret_cast<const uint4*>(rep)[lane & 7u];
          pp = v.backend + tb + (lane & 7u) * 8u;
          pend = true;
        } else {
          if (valid)
            __hip_atomic_store((__attribute__((address_space(1))) uint16_t*)(v.backend + p), be, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
          ++seq;
        }
      }
    }
    lds_sync();
    // every tile wave has waited for tile k: the stores of steps <= k - 4 retired (the backends of
    // step k - 3 went out behind tile k's issue)
    if (ctl && hC != 0xffffffffu) RING_PUBLISH(hC)
    hC = hB;
    hB = hA;
    hA = h0;
    sA = sB;
    sB = sC;
    ++k;
  }
#undef RING_ISSUE
#undef RING_PUBLISH
#undef RING_TAKE_STAGED
  // the block's exit, once every wave's stores have retired: a gate kernel waiting for a batch this
  // ring will never complete (stop, idle exit) returns when every classify block has exited
  wait_vm<0>();
  lds_sync();
  if (tid == 0) __hip_atomic_fetch_add(r.dexit, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The gate of a ring batch's grouping (nbg_ring_group before the batch is complete): one wave that
// polls the relay's completion word in uncached HBM and returns once batch target - 1 is complete,
// or once every classify block has exited (the ring ended; the grouping then reads what backend[]
// holds, which no kernel writes any more).  Every path ends: the ring itself always ends (stop or
// idle_ms).  Launched ahead of the batch's hist / group kernels on the caller's stream, so the
// producer needs no host poll between the ring's completion and the grouping.
__global__ __launch_bounds__(64) void ring_gate_kernel(const uint32_t* dcomp, const uint32_t* dexit, uint32_t target,
                                                       uint32_t grid) {
  for (uint32_t nap = 1;; nap = min(2u * nap, 4u)) {
    const uint32_t c = rfl(__hip_atomic_load(dcomp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    if (static_cast<int32_t>(c - target) >= 0) return;
    if (rfl(__hip_atomic_load(dexit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) >= grid) return;
    for (uint32_t i = 0; i < nap; ++i) __builtin_amdgcn_s_sleep(2);
  }
}

// ---- streaming classify for descriptor layouts (IMIX: u32 offsets + u16 lengths, owned windows) ----
//
// Configs C5 (the lpm -> maglev chain: u8 LUT in LDS, tbl24 gathered) and the IMIX read-only /
// record layouts (u8 LUT in LDS or the u16 LUT gathered).  Same block structure as
// classify_stream_kernel (one block per CU, interleaved units, per-unit block histogram).  Per wave,
// everything global arrives by LDS-DMA: the descriptors of a tile (off[64], len[64]) issued four
// tiles ahead, the packet windows of a tile from its descriptors three tiles ahead, and the per-packet
// gather (tbl24 or LUT entry, 2 B per lane) one tile ahead — so iteration k hashes tile k+1 and
// issues its gather, then finishes tile k, whose gather had a whole iteration to land.  The chain's
// second, dependent gather (tbl_long, routes longer than /24) is issued at the start of iteration k
// and waited for after tile k+1's hash and prefetches, so it never drains them.  Opt-in
// (NBG_STREAM_DESC): one block per CU holds all LDS, so several streams' kernels cannot co-run.
//
// vmcnt retires in issue order and hipcc does not count these loads, so the kernel keeps its own
// wave-uniform count of issued VM operations (`seq`): each load group records the count after it,
// and waiting for one is vmcnt(seq - recorded).  Every store instruction is issued by every lane
// (lanes with nothing to store write to a scratch sink), so the count of stores per tile is a
// known lower bound; uncounted operations (byte-wise path, histogram flush) only ever make a wait
// stricter.
// A 1- or 2-B LDS-DMA load still fills one dword per lane (measured: lane i's value at 4i), so the
// u16 lengths and gathered entries take 4 B of LDS per lane.
constexpr uint32_t kDescRing = 4;                   // descriptor slots per wave: tiles k .. k+3, then k+4 into k's
constexpr uint32_t kDescLds = 64u * 4u + 64u * 4u;  // off[64] then len[64] (dword per lane)
constexpr uint32_t kGatherLds = 64u * 4u;           // one dword per lane, two tiles

template <int MODE>
__host__ __device__ constexpr uint32_t desc_ring_tiles() { return MODE == 1 ? 4u : 3u; }

template <int MODE>
__host__ __device__ constexpr uint32_t desc_wave_lds() {
  return desc_ring_tiles<MODE>() * 64u * row_of<MODE>() + kDescRing * kDescLds + 3u * kGatherLds;
}

// A hashed tile waiting for its gather.
struct DescTile {
  uint32_t fast;   // packet on the fast path (valid, 16-B aligned, >= 48 B, IHL 5)
  uint32_t bin;    // u8 LUT: the entry (LDS lookup)
  uint32_t iplo;   // chain: low byte of the source address (tbl_long index)
  uint32_t r0, r1, r2;  // records: the swapped MAC words
};


// LUTM: kLdsU8Tail (u8 LUT staged in LDS) or kGlobalU16 (u16 LUT gathered from L2).
// MODE: 0 = read only (always with CHAIN), 1 = in place (whole owned windows), 2 = 12-B records.
template <int LUTM, bool F4, bool HIST, int MODE, bool CHAIN>
__global__ __launch_bounds__(kStreamNT, 1) void classify_stream_desc_kernel(ClassifyArgs a) {
  constexpr uint32_t kRow = row_of<MODE>(), kTileLds = 64u * kRow;
  constexpr uint32_t kLut = LUTM == kLdsU8Tail ? kLutLds : 0u;
  constexpr uint32_t kPR = desc_ring_tiles<MODE>();
  constexpr bool kG = (CHAIN || LUTM == kGlobalU16) ;  // one 2-B gather per packet
  // store instructions per tile (a lower bound: the compiler may not split them further)
  constexpr uint32_t kS = 1u + (CHAIN ? 1u : 0u) + (MODE == 1 ? 4u : 0u) + (MODE == 2 ? 1u : 0u);
  extern __shared__ __align__(16) uint8_t smem[];
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t nbins = a.nb + 1;
  uint8_t* lut = smem;
  uint8_t* wbase = smem + kLut + wave * desc_wave_lds<MODE>();
  uint8_t* ring = wbase;
  uint8_t* dring = wbase + kPR * kTileLds;
  uint8_t* gbuf = dring + kDescRing * kDescLds;
  uint8_t* tlbuf = gbuf + 2u * kGatherLds;  // chain: tbl_long entries of the tile being finished
  const uint32_t hstride = (nbins + 3) & ~3u;
  uint32_t* hist = reinterpret_cast<uint32_t*>(smem + kLut + kStreamW * desc_wave_lds<MODE>());
  const uint32_t ring_lds = __builtin_amdgcn_readfirstlane(lds_addr(ring));
  const uint32_t dring_lds = __builtin_amdgcn_readfirstlane(lds_addr(dring));
  const uint32_t gbuf_lds = __builtin_amdgcn_readfirstlane(lds_addr(gbuf));
  const uint32_t tl_lds = __builtin_amdgcn_readfirstlane(lds_addr(tlbuf));
  const uint32_t lut_lds = __builtin_amdgcn_readfirstlane(lds_addr(lut));
  const uint32_t n_tiles = (a.n_pkts + 63u) >> 6;
  const uint32_t n_units = (n_tiles + kStreamW - 1) / kStreamW;
  const uint32_t G = gridDim.x, b = blockIdx.x;
  const uint32_t nt = b < n_units ? (n_units - b + G - 1) / G : 0u;
  auto tile_of = [&](uint32_t k) { return (b + k * G) * kStreamW + wave; };
  auto doff = [&](uint32_t k) {
    return reinterpret_cast<const uint32_t*>(dring + (k % kDescRing) * kDescLds);
  };
  auto dlen = [&](uint32_t k) {
    return reinterpret_cast<const uint32_t*>(dring + (k % kDescRing) * kDescLds + 256u);
  };
  uint8_t* sink = a.sink + lane * 16u;
  uint32_t seq = 0;  // VM operations this wave issued (counted ones)
  auto wait_seq = [&](uint32_t after) { wait_vm_n(seq - after); };
  // descriptors of step k: lane i fetches off/len of packet tile_of(k)*64 + i (clamped)
  auto issue_desc = [&](uint32_t k) {
    const uint32_t p = min(tile_of(k) * 64u + lane, a.n_pkts - 1u);
    const uint32_t d = dring_lds + (k % kDescRing) * kDescLds;
    glds4(a.off + p, d);
    glds2(a.len + p, d + 256u);
    seq += 2;
    return seq;
  };
  // packet windows of step k from its landed descriptors; a window off the 16-B grid is fetched
  // from the batch base (its lane takes the byte-wise path)
  auto issue_pk = [&](uint32_t k) {
    constexpr uint32_t kCh = kRow / 16u;
    const uint32_t* o = doff(k);
    const uint32_t buf = ring_lds + (k % kPR) * kTileLds;
    const uint32_t tb = tile_of(k) * 64u;
    if (kCh == 4u || lane < 16u * kCh) {
      const uint32_t pk = lane / kCh, ch = lane - pk * kCh;
      uint32_t off[4];
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j) off[j] = o[j * 16u + pk];
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t q = j * 16u + pk;
        const uint8_t* src = (tb + q < a.n_pkts && (off[j] & 15u) == 0) ? a.pkts + off[j] + ch * 16u : a.pkts;
        glds16_tile<MODE != 2>(src, buf + j * (16u * kRow));
      }
    }
    seq += 4;
    return seq;
  };
  // hash step k's packets (landed) and issue their gather; returns the count after the gather
  auto hash = [&](uint32_t k, DescTile& st) {
    const uint32_t p = tile_of(k) * 64u + lane;
    const uint8_t* x = ring + (k % kPR) * kTileLds + lane * kRow;
    const uint4 c0 = *reinterpret_cast<const uint4*>(x);
    const uint4 c1 = *reinterpret_cast<const uint4*>(x + 16);
    const uint2 c2 = *reinterpret_cast<const uint2*>(x + 32);
    const uint32_t off = doff(k)[lane], len = dlen(k)[lane] & 0xffffu;
    const bool fast = p < a.n_pkts && (off & 15u) == 0 && len >= 48u && ((c0.w >> 16) & 0xfu) == 5u;
    st.fast = fast;
    // frame bytes: src 26..29, dst 30..33, ports 34..37, proto 23
    const uint32_t src = (c1.z >> 16) | (c1.w << 16);
    const uint32_t dst = (c1.w >> 16) | (c2.x << 16);
    const uint32_t ports = (c2.x >> 16) | (c2.y << 16);
    uint32_t lo, hi;
    fnv_flow(lo, hi, src, dst, ports, c1.y >> 24);
    const uint32_t idx = F4 ? mod_f4(lo, hi) : mod_barrett(lo, hi, a.m, a.mu);
    if constexpr (LUTM == kLdsU8Tail) st.bin = (idx >> 16) ? a.lut_tail : lut[idx & 0xffffu];
    if constexpr (MODE == 2) {
      st.r0 = (c0.y >> 16) | (c0.z << 16);
      st.r1 = (c0.z >> 16) | (c0.x << 16);
      st.r2 = (c0.x >> 16) | (c0.y << 16);
    }
    const uint32_t g = gbuf_lds + (k & 1u) * kGatherLds;
    if constexpr (CHAIN) {
      const uint32_t ip = __builtin_bswap32(src);
      st.iplo = ip & 0xffu;
      if (kG) glds2(a.tbl24 + (fast ? (ip >> 8) : 0u), g);
    } else if constexpr (LUTM == kGlobalU16 && kG) {
      glds2(static_cast<const uint16_t*>(a.lut) + (fast ? idx : 0u), g);
    }
    if constexpr (kG) ++seq;
    return seq;
  };

  if constexpr (kLut) {
    const uint32_t pieces = a.lut_lds_bytes >> 10;
    for (uint32_t q = wave; q < pieces; q += kStreamW)
      glds16(static_cast<const uint8_t*>(a.lut) + q * 1024u + lane * 16u, lut_lds + q * 1024u);
  }
  if constexpr (HIST)
    for (uint32_t i = tid; i < 2 * hstride; i += kStreamNT) hist[i] = 0;
  // prologue: D(0..2) landed, P(0..2) and D(3) in flight
  uint32_t sP1 = 0, sP2 = 0, sP3 = 0, sD3 = 0, sD4 = 0, sG0 = 0, sG1 = 0, sP0 = 0;
  if (nt > 0) {
    for (uint32_t j = 0; j < 3 && j < nt; ++j) issue_desc(j);
    wait_vm<0>();  // the LUT pieces too
    sP0 = issue_pk(0);
    if (nt > 1) sP1 = issue_pk(1);
    if (nt > 2) sP2 = issue_pk(2);
    if (nt > 3) sD3 = issue_desc(3);
  }
  lds_sync();  // LUT and zeroed histograms visible to every wave
  DescTile cur{}, nxt{};
  if (nt > 0) {
    wait_seq(sP0);
    sG0 = hash(0, cur);
  }
  for (uint32_t k = 0; k < nt; ++k) {
    const uint32_t tb = tile_of(k) * 64u;
    const uint32_t p = tb + lane;
    const bool valid = p < a.n_pkts;
    // tile k's gather (issued one iteration ago)
    uint32_t gv = 0;
    if constexpr (kG) {
      wait_seq(sG0);
      gv = reinterpret_cast<const uint32_t*>(gbuf + (k & 1u) * kGatherLds)[lane] & 0xffffu;
    }
    uint32_t bin = LUTM == kLdsU8Tail ? cur.bin : gv;
    uint32_t gate = kSentinel;
    // chain: routes longer than /24 need a second, dependent gather (tbl_long); issued here, before
    // the next tile's work, and waited for after it, so it does not drain the prefetches
    bool lng = false, any_lng = false;
    uint32_t sTL = 0;
    if constexpr (CHAIN) {
      gate = gv;
      lng = cur.fast && (gv & 0x8000u);
      any_lng = kG && __builtin_amdgcn_ballot_w64(lng) != 0;
      if (any_lng) {
        glds2(a.tbl_long + (lng ? ((gv & 0x7fffu) << 8) + cur.iplo : 0u), tl_lds);
        sTL = ++seq;
      }
    }
    if (k + 1 < nt) {
      wait_seq(sP1);
      sG1 = hash(k + 1, nxt);
    }
    if (k + 3 < nt) {
      wait_seq(sD3);
      sP3 = issue_pk(k + 3);
    }
    if constexpr (CHAIN) {
      if (any_lng) {
        wait_seq(sTL);
        const uint32_t t = reinterpret_cast<const uint32_t*>(tlbuf)[lane] & 0xffffu;
        if (lng) gate = t;
      }
    }
    if constexpr (MODE == 1) {
      // whole owned windows back from LDS: lane (quad, part) stores chunk `part` of packet
      // 16j + quad, chunk 0 with the MACs swapped; lanes of other packets store to the sink
      const uint8_t* tile = ring + (k % kPR) * kTileLds;
      const uint32_t part = lane & 3u, quad = lane >> 2;
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t q = j * 16u + quad;
        uint4 v = *reinterpret_cast<const uint4*>(tile + q * kRow + part * 16u);
        const uint32_t qo = doff(k)[q], ql = dlen(k)[q] & 0xffffu;
        const uint32_t w3 =
            static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v.w), 0x00, 0xf, 0xf, false));
        const bool qfast = tb + q < a.n_pkts && (qo & 15u) == 0 && ql >= 48u && ((w3 >> 16) & 0xfu) == 5u;
        if (part == 0u)
          v = make_uint4((v.y >> 16) | (v.z << 16), (v.z >> 16) | (v.x << 16), (v.x >> 16) | (v.y << 16), v.w);
        stg16_nt(qfast ? a.pkts + qo + part * 16u : sink, v);
      }
    } else if constexpr (MODE == 2) {
      uint32_t* mo = reinterpret_cast<uint32_t*>(cur.fast ? a.mac_out + static_cast<size_t>(p) * 12u : sink);
      mo[0] = cur.r0;
      mo[1] = cur.r1;
      mo[2] = cur.r2;
    }
    if (valid && !cur.fast) {
      // byte-wise loads: their waits stay inside this branch
      bin = classify_slow<LUTM, F4, CHAIN>(a, lut, a.pkts + doff(k)[lane], dlen(k)[lane] & 0xffffu, p, gate);
      asm volatile("" : "+v"(bin), "+v"(gate)::"memory");
    }
    if constexpr (CHAIN) {
      if (cur.fast && gate >= a.lpm_groups) bin = a.nb;  // test/lpm would panic: never reaches maglev
      *(valid ? a.gate + p : reinterpret_cast<uint16_t*>(sink)) = static_cast<uint16_t>(gate);
    }
    *(valid ? a.backend + p : reinterpret_cast<uint16_t*>(sink)) = static_cast<uint16_t>(bin == a.nb ? kSentinel : bin);
    seq += kS;
    if constexpr (HIST) {
      if (valid) atomicAdd(&hist[(k & 1u) * hstride + bin], 1u);
      lds_sync();
      if (wave == k % kStreamW) {
        uint32_t* h = hist + (k & 1u) * hstride;
        stream_flush<HIST>(a, h, nbins, ((b + k * G) * kStreamW * 64u) / a.part_pkts, lane);
      }
    }
    if (k + 4 < nt) sD4 = issue_desc(k + 4);  // into tile k's descriptor slot, now free
    cur = nxt;
    sP1 = sP2;
    sP2 = sP3;
    sD3 = sD4;
    sG0 = sG1;
  }
}

// Many backends: the partition histograms come from this kernel instead of the classify kernel
// (whose per-block flush would cost about one global atomic per packet at ~1000 bins).  One
// 512-thread block per partition counts its packets' backends in LDS and stores the whole row.
// Blocks [j * hm.per, j * hm.per + h[j].n_parts) count batch j (a single batch: j = 0).
__global__ __launch_bounds__(kGBlock) void hist_kernel(HistMulti hm) {
  extern __shared__ __align__(16) uint32_t hs[];
  const uint32_t bj = blockIdx.x / hm.per;
  const HistArgs a = hm.h[bj];
  const uint32_t nbins = a.nb + 1, tid = threadIdx.x, c_lin = blockIdx.x - bj * hm.per;
  // the group kernel's XCD-aware partition order: partition c's backends, read here, are read again by
  // the group block of partition c on the same XCD, from its L2
  const uint32_t c = (a.n_parts % 8u == 0u && c_lin < a.n_parts) ? (c_lin % 8u) * (a.n_parts / 8u) + c_lin / 8u : c_lin;
  if (c >= a.n_parts) return;
  const uint32_t pbeg = c * a.part_pkts, pend = min(pbeg + a.part_pkts, a.n_pkts);
  for (uint32_t b = tid; b < nbins; b += kGBlock) hs[b] = 0;
  lds_sync();
  // one chunk per pass, every load unconditional (clamped) and in flight together
  for (uint32_t i0 = pbeg; i0 < pend; i0 += kChunk) {
    uint32_t v[kGRounds];
#pragma unroll
    for (int k = 0; k < kGRounds; ++k) v[k] = ld_u16(a.backend, min(i0 + k * kGBlock + tid, a.n_pkts - 1u) * 2u);
#pragma unroll
    for (int k = 0; k < kGRounds; ++k) {
      // min: the sentinel (0xFFFF) is bin nb; so is any other value > nb, which no classify writes
      // but a ring batch's backend[] can hold after a ring that ended before completing it
      if (i0 + k * kGBlock + tid < pend) atomicAdd(&hs[min(v[k], a.nb)], 1u);
    }
  }
  lds_sync();
  if (a.hist16) {  // half the row bytes the group kernel's direct prefix reads
    const uint32_t hw = (nbins + 1) >> 1;
    uint32_t* row = a.part_hist + static_cast<size_t>(c) * hw;
    for (uint32_t w = tid; w < hw; w += kGBlock) row[w] = hs[2 * w] | (2 * w + 1 < nbins ? hs[2 * w + 1] << 16 : 0u);
    return;
  }
  uint32_t* row = a.part_hist + static_cast<size_t>(c) * nbins;
  for (uint32_t b = tid; b < nbins; b += kGBlock) row[b] = hs[b];
}

// Many backends: exclusive scan of part_hist[.][bin] over partitions, and every bin's total.
// One block per 64 consecutive bins, one lane per bin; wave w scans partitions [32w, 32w + 32)
// in registers (each row segment is one coalesced 256-B load, all 32 in flight), and the waves'
// sums are combined through LDS.
constexpr uint32_t kScanBins = 64, kScanWaves = kMaxParts / 32;
__global__ __launch_bounds__(kScanWaves * 64) void scan_kernel(ScanMulti sm) {
  __shared__ uint32_t s_sum[kScanWaves][kScanBins];
  const ScanArgs a = sm.s[blockIdx.y];  // batch
  const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u;
  const uint32_t b = blockIdx.x * kScanBins + lane;
  const uint32_t bc = min(b, a.nbins - 1u), q0 = wave * 32u;
  uint32_t v[32];
#pragma unroll
  for (uint32_t k = 0; k < 32; ++k) v[k] = ld_u32(a.part_hist, (min(q0 + k, a.n_parts - 1u) * a.nbins + bc) * 4u);
  uint32_t run = 0;
#pragma unroll
  for (uint32_t k = 0; k < 32; ++k) {
    const uint32_t x = q0 + k < a.n_parts ? v[k] : 0u;
    v[k] = run;  // exclusive within this wave's partitions
    run += x;
  }
  s_sum[wave][lane] = run;
  __syncthreads();
  uint32_t off = 0, total = 0;
#pragma unroll
  for (uint32_t w = 0; w < kScanWaves; ++w) {
    const uint32_t t = s_sum[w][lane];
    off += w < wave ? t : 0u;
    total += t;
  }
  if (b < a.nbins) {
#pragma unroll
    for (uint32_t k = 0; k < 32; ++k)
      if (q0 + k < a.n_parts) a.part_prefix[static_cast<size_t>(q0 + k) * a.nbins + b] = off + v[k];
    if (wave == 0) a.totals[b] = total;
  }
}

// ---- LDS-tiled lookup (NBG_LUT_TILED; config C3's named variant) --------------------------------
// A u16 LUT larger than LDS (C3: 655373 entries = 1.25 MiB) is split into 64-KiB tiles of 32768
// entries.  After the classify kernel has written each packet's LUT index (kIdx):
//   tile_bucket_kernel  appends (packet, index in tile) to its tile's bucket: counts per tile in
//                       LDS, one global reservation per tile per block, then the scatter;
//   tile_lookup_kernel  one block per (tile, chunk of its bucket) stages the tile in LDS and
//                       resolves its chunk: backend[packet] = tile[index].
// Would-panic packets (index 0xffffffff) get the sentinel in the bucket kernel.  The measured
// alternative to the L2 gather that BASELINE config C3 names.
constexpr uint32_t kTileEntries = 32768;  // u16 entries per 64-KiB LUT tile
constexpr uint32_t kBucketNT = 256, kBucketPkts = 4096, kLookupNT = 512, kLookupChunk = 8192;

__global__ __launch_bounds__(kBucketNT) void tile_bucket_kernel(TileArgs a) {
  extern __shared__ __align__(16) uint32_t tcnt[];  // [n_tiles] counts, then reserved bases
  const uint32_t tid = threadIdx.x, p0 = blockIdx.x * kBucketPkts;
  for (uint32_t t = tid; t < a.n_tiles; t += kBucketNT) tcnt[t] = 0;
  __syncthreads();
  constexpr uint32_t kPer = kBucketPkts / kBucketNT;
  uint32_t idx[kPer], slot[kPer];
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) {
    const uint32_t p = p0 + k * kBucketNT + tid;
    idx[k] = a.idx[min(p, a.n_pkts - 1u)];
  }
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) {
    const uint32_t p = p0 + k * kBucketNT + tid;
    slot[k] = 0;
    if (p < a.n_pkts) {
      if (idx[k] == 0xffffffffu) a.backend[p] = static_cast<uint16_t>(kSentinel);
      else slot[k] = atomicAdd(&tcnt[idx[k] / kTileEntries], 1u);
    }
  }
  __syncthreads();
  for (uint32_t t = tid; t < a.n_tiles; t += kBucketNT)
    tcnt[t] = tcnt[t] ? atomicAdd(&a.cursor[t], tcnt[t]) : 0u;
  __syncthreads();
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) {
    const uint32_t p = p0 + k * kBucketNT + tid;
    if (p < a.n_pkts && idx[k] != 0xffffffffu) {
      const uint32_t t = idx[k] / kTileEntries;
      a.bucket[static_cast<size_t>(t) * a.bucket_cap + tcnt[t] + slot[k]] =
          (static_cast<uint64_t>(p) << 32) | (idx[k] - t * kTileEntries);
    }
  }
}

__global__ __launch_bounds__(kLookupNT) void tile_lookup_kernel(TileArgs a) {
  extern __shared__ __align__(16) uint16_t tlut[];  // one LUT tile
  const uint32_t t = blockIdx.y, tid = threadIdx.x;
  const uint32_t cnt = a.cursor[t];
  const uint32_t c0 = blockIdx.x * kLookupChunk;
  if (c0 >= cnt) return;  // block-uniform
  const uint32_t entries = min(kTileEntries, a.m - t * kTileEntries);
  const uint4* src = reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(a.lut) + t * kTileEntries);
  for (uint32_t v = tid; v < (entries + 7) / 8; v += kLookupNT) reinterpret_cast<uint4*>(tlut)[v] = src[v];
  __syncthreads();
  const uint64_t* b = a.bucket + static_cast<size_t>(t) * a.bucket_cap;
  const uint32_t c1 = min(c0 + kLookupChunk, cnt);
  for (uint32_t i = c0 + tid; i < c1; i += kLookupNT) {
    const uint64_t e = b[i];
    a.backend[static_cast<uint32_t>(e >> 32)] = tlut[static_cast<uint32_t>(e)];
  }
}

// ---- small batches: classify + stable grouping in one launch -------------------------------------
// A batch of at most kSmallMax packets (one grouping partition) and at most kMaxGroupBins bins is
// classified and grouped by one 1024-thread block: NetBricks' own bursts are 32 packets
// (receive_batch.rs:26), where two launches and their gaps were the whole cost of a call.  Wave w
// owns packets [256w, 256w + 256) in four 64-packet rounds.  Per packet: the chunks 0..2 of its
// 64-B window are loaded as three 16-B vectors when the frame allows (aligned, >= 48 B), and it
// takes the fast path (IHL 5) or the byte-wise path.  The loads are coalesced: in a round, load k
// of lane l fetches chunk (64k + l) % 3 of packet (64k + l) / 3, so three neighbouring lanes read one
// packet's 48 contiguous bytes in one instruction (one request per line, where a lane per packet
// touched every line three times, once per instruction: the host path's direct batches read their
// windows over PCIe, uncached); an LDS pass hands each lane its packet's three chunks.  Then each round ranks its lanes among the
// same bin (readlane match) into per-wave counters, one block scan over (bin, wave) in bin-major
// order gives every wave's start per bin, and perm is scattered: per-group FIFO order as the
// reference's producer (group_by.rs:46-51).
constexpr uint32_t kSmallNT = 1024, kSmallW = kSmallNT / 64;
constexpr uint32_t kSmallMax = 4 * kSmallNT;

// W32 (the host path's 32-B staging, a.win32): window p holds frame bytes 8..39 (the host swapped the
// MACs and staged no bytes below 8), so c[0] is frame bytes 8..23 and c[1] bytes 24..39, and the frame
// starts 8 B before its window; every byte the parse reads for IHL <= 5 lies in it (the host stages a
// batch with a longer IP header in whole 48/64/80-B windows instead).
template <int LUTM, bool F4, bool W32 = false>
__device__ __forceinline__ uint32_t small_classify(const ClassifyArgs& a, uint32_t p, uint32_t off, uint32_t len,
                                                   const uint4* c) {
  if constexpr (W32) {
    uint8_t* w = a.pkts + off;
    if ((reinterpret_cast<uintptr_t>(w) & 15u) == 0 && len >= 40u && ((c[0].y >> 16) & 0xfu) == 5u) {
      // frame bytes: IHL 14, protocol 23, src 26..29, dst 30..33, ports 34..37
      const uint32_t src = (c[1].x >> 16) | (c[1].y << 16);
      const uint32_t dst = (c[1].y >> 16) | (c[1].z << 16);
      const uint32_t ports = (c[1].z >> 16) | (c[1].w << 16);
      uint32_t lo, hi;
      fnv_flow(lo, hi, src, dst, ports, c[0].w >> 24);
      return lookup<LUTM, F4>(a, nullptr, lo, hi);
    }
    uint32_t gate;  // reads frame bytes 14 .. min(len, 40) - 1 only (no swap on this path)
    return classify_slow<LUTM, F4, false>(a, nullptr, w - 8, len, p, gate);
  }
  uint8_t* pk = a.pkts + off;
  const bool vec = (reinterpret_cast<uintptr_t>(pk) & 15u) == 0 && len >= 48u;
  if (vec && ((c[0].w >> 16) & 0xfu) == 5u) {
    const uint32_t src = (c[1].z >> 16) | (c[1].w << 16);
    const uint32_t dst = (c[1].w >> 16) | (c[2].x << 16);
    const uint32_t ports = (c[2].x >> 16) | (c[2].y << 16);
    uint32_t lo, hi;
    fnv_flow(lo, hi, src, dst, ports, c[1].y >> 24);
    const uint32_t bin = lookup<LUTM, F4>(a, nullptr, lo, hi);
    if (a.swap) {
      const uint32_t w0 = (c[0].y >> 16) | (c[0].z << 16), w1 = (c[0].z >> 16) | (c[0].x << 16),
                     w2 = (c[0].x >> 16) | (c[0].y << 16);
      if (a.mac_out) {
        uint32_t* mo = reinterpret_cast<uint32_t*>(a.mac_out + static_cast<size_t>(p) * 12u);
        mo[0] = w0;
        mo[1] = w1;
        mo[2] = w2;
      } else {
        *reinterpret_cast<uint4*>(pk) = make_uint4(w0, w1, w2, c[0].w);
      }
    }
    return bin;
  }
  uint32_t gate;
  return classify_slow<LUTM, F4, false>(a, nullptr, pk, len, p, gate);
}

template <int LUTM, bool F4, int BITS, bool W32 = false>
__device__ __forceinline__ void small_body(const ClassifyArgs& a, const GroupArgs& g) {
  extern __shared__ __align__(16) uint32_t sm[];
  const uint32_t nbins = a.nb + 1, nbp = (nbins + 3) & ~3u;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t nw = blockDim.x >> 6;  // waves launched: ceil(n / 256)
  uint32_t* cnt = sm;                                            // [nw][nbp]: per-wave counts
  uint16_t* rank16 = reinterpret_cast<uint16_t*>(cnt + kSmallW * nbp);  // [kSmallMax]
  uint16_t* bin16 = rank16 + kSmallMax;                          // [kSmallMax]
  __shared__ uint32_t s_wave[kSmallW];
  const bool group = g.perm || g.counts;
  if (group)
    for (uint32_t i = tid; i < nw * nbp; i += blockDim.x) cnt[i] = 0;
  // this wave's rounds that hold packets (wave-uniform)
  const uint32_t rounds = min(4u, (a.n_pkts - min(a.n_pkts, wave * 256u) + 63u) / 64u);
  // loads of every round first (unconditional, clamped), then every round's classification (its
  // LUT gathers in flight together), then the ranking
  uint32_t off[4], len[4], bin[4];
  uint4 v[4][3];
#pragma unroll
  for (uint32_t r = 0; r < 4; ++r) {
    const uint32_t p = min(wave * 256u + r * 64u + lane, a.n_pkts - 1u);
    off[r] = a.off ? a.off[p] : p * a.stride;
    len[r] = a.len ? a.len[p] : a.fixed_len;
  }
  // owned windows (slots of >= 64 B, mbuf data rooms, the host path's staging): the 48 B at every
  // packet start are readable whatever its length, so the window loads do not wait for len[] (over
  // PCIe, for the host path's direct batches, one round trip less per batch)
  const bool owned = a.win_owned != 0;
  constexpr uint32_t kCh = W32 ? 2u : 3u;  // 16-B chunks per window
#pragma unroll
  for (uint32_t r = 0; r < 4; ++r) {
    if constexpr (W32) {
      // 32-B windows: lane pair (2i, 2i + 1) reads window i of the round's first 32, then of the last
#pragma unroll
      for (uint32_t k = 0; k < 2; ++k) {
        const uint32_t q = 64u * k + lane, pi = q >> 1, part = q & 1u;
        const uint8_t* w = a.pkts + __shfl(off[r], static_cast<int>(pi));
        const bool vec = (reinterpret_cast<uintptr_t>(w) & 15u) == 0;
        v[r][k] = *reinterpret_cast<const uint4*>((vec ? w : a.pkts) + 16u * part);
      }
      continue;
    }
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) {
      const uint32_t q = 64u * k + lane, pi = q / 3u, part = q - 3u * pi;
      const uint8_t* pk = a.pkts + __shfl(off[r], static_cast<int>(pi));
      bool vec = (reinterpret_cast<uintptr_t>(pk) & 15u) == 0;
      if (!owned) {
        // every lane shuffles (not under `vec &&`: a bpermute from a lane the short-circuit
        // disabled reads 0, and the packet would then take the batch base's window)
        const uint32_t l = __shfl(len[r], static_cast<int>(pi));
        vec = vec && l >= 48u;
      }
      // the batch base is 16-B aligned by the host check; its 48 B are read for packets off the path
      v[r][k] = *reinterpret_cast<const uint4*>((vec ? pk : a.pkts) + 16u * part);
    }
  }
  uint4* tp = reinterpret_cast<uint4*>(bin16 + kSmallMax) + wave * 192u;  // [192] chunks of one round
#pragma unroll
  for (uint32_t r = 0; r < 4; ++r) {
#pragma unroll
    for (uint32_t k = 0; k < kCh; ++k) tp[64u * k + lane] = v[r][k];
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();  // one wave: its LDS operations run in issue order
    uint4 c[3];
#pragma unroll
    for (uint32_t k = 0; k < kCh; ++k) c[k] = tp[kCh * lane + k];
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();  // the next round's writes after these reads
    const uint32_t p = wave * 256u + r * 64u + lane;
    bin[r] = 0xffffffffu;
    if (r < rounds && p < a.n_pkts) bin[r] = small_classify<LUTM, F4, W32>(a, p, off[r], len[r], c);
  }
  // backend[] after every round's gathers: vmcnt counts stores too and retires in order, so a store
  // issued between two rounds' LUT gathers made the second gather's wait also wait for the store (a
  // PCIe round trip for the host path's direct batches)
#pragma unroll
  for (uint32_t r = 0; r < 4; ++r) {
    const uint32_t p = wave * 256u + r * 64u + lane;
    if (r < rounds && p < a.n_pkts) a.backend[p] = static_cast<uint16_t>(bin[r] == a.nb ? kSentinel : bin[r]);
  }
  if (!group) return;
  lds_sync();  // counters zeroed
  uint32_t* wc = cnt + wave * nbp;
  for (uint32_t r = 0; r < rounds; ++r) {
    const uint32_t p = wave * 256u + r * 64u + lane;
    const bool valid = p < a.n_pkts;
    const uint32_t b = valid ? bin[r] : 0u;
    uint32_t rank, count;
    wave_match_rank<BITS>(b, valid, lane, rank, count);
    // every lane of a bin reads the same count and stores the same new one (one wave: its LDS
    // operations execute in issue order)
    const uint32_t before = wc[b];
    __builtin_amdgcn_wave_barrier();
    if (valid) {
      rank16[p] = static_cast<uint16_t>(before + rank);
      bin16[p] = static_cast<uint16_t>(b);
      wc[b] = before + count;
    }
    __builtin_amdgcn_wave_barrier();
  }
  lds_sync();
  // exclusive scan over the counters in (bin, wave) order; each thread owns `per` consecutive
  // entries; the waves' partial sums are combined through s_wave
  const uint32_t ne = nbins * nw, per = (ne + blockDim.x - 1) / blockDim.x;
  uint32_t sum = 0;
  for (uint32_t k = 0; k < per; ++k) {
    const uint32_t e = tid * per + k;
    sum += e < ne ? cnt[(e % nw) * nbp + e / nw] : 0u;
  }
  const uint32_t xs = wave_incl_scan(sum);
  if (lane == 63u) s_wave[wave] = xs;
  // counts: a bin's packets = the sum of its wave counters (read before they are replaced)
  if (g.counts)
    for (uint32_t b = tid; b < nbins; b += blockDim.x) {
      uint32_t t = 0;
      for (uint32_t w = 0; w < nw; ++w) t += cnt[w * nbp + b];
      g.counts[b] = t;
    }
  lds_sync();
  uint32_t x = xs - sum;
  for (uint32_t w = 0; w < wave; ++w) x += s_wave[w];
  for (uint32_t k = 0; k < per; ++k) {
    const uint32_t e = tid * per + k;
    if (e < ne) {
      const uint32_t v = cnt[(e % nw) * nbp + e / nw];
      cnt[(e % nw) * nbp + e / nw] = x;
      x += v;
    }
  }
  lds_sync();
  if (g.perm) {
    // perm is scattered in LDS (the load-transpose area, free now: 3 KB per wave >= 4 B per packet)
    // and stored in order, 16 B per lane: scattered 4-B stores were a partial line each, and over
    // PCIe (the host path's direct batches) a write of its own for the block's system fence to wait
    // for (host-batch server at 16 pipelines: 41.5 us body + 27.4 us fence per 992-packet batch)
    uint32_t* pl = reinterpret_cast<uint32_t*>(bin16 + kSmallMax);
    for (uint32_t p = tid; p < a.n_pkts; p += blockDim.x) pl[cnt[(p >> 8) * nbp + bin16[p]] + rank16[p]] = p;
    lds_sync();
    if ((reinterpret_cast<uintptr_t>(g.perm) & 15u) == 0) {
      for (uint32_t i = 4u * tid; i < a.n_pkts; i += 4u * blockDim.x) {
        if (i + 4u <= a.n_pkts) {
          *reinterpret_cast<uint4*>(g.perm + i) = *reinterpret_cast<const uint4*>(pl + i);
        } else {
          for (uint32_t j = i; j < a.n_pkts; ++j) g.perm[j] = pl[j];
        }
      }
    } else {
      for (uint32_t i = tid; i < a.n_pkts; i += blockDim.x) g.perm[i] = pl[i];
    }
  }
}

// done (nullable): a completion word in pinned host memory (nbg_maglev_host_submit's direct path), set
// to done_val once every output of the batch is visible to the host: each thread's stores are
// released at system scope, then, behind the block barrier, one vector store of the word.  The host
// polls it with plain loads instead of querying an event through the runtime.
template <int LUTM, bool F4, int BITS, bool W32>
__global__ __launch_bounds__(kSmallNT) void small_kernel(ClassifyArgs a, GroupArgs g, uint32_t* done, uint32_t done_val) {
  small_body<LUTM, F4, BITS, W32>(a, g);
  if (done) {
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(done, done_val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ---- host-batch server (nbg_host_ring_*) ---------------------------------------------------------
// One launch per GPU serves every producer thread's small host batches (nbg_maglev_host_submit's
// direct path) without a kernel launch per batch: the GPU's dispatch rate, ~200k launches/s per GPU
// measured with 16 producer threads, capped the drop-in path at ~200 Mpps at the
// reference's 992-packet batches.  Each 1024-thread block: claim the next ticket (device atomic), wait
// for its descriptor in pinned host memory (thread 0 polls seq with s_sleep; exits on the host's stop,
// or after idle_ticks without any post), copy it to LDS, acknowledge it, run the small kernel's body
// on it, set the batch's completion word.  Every posted ticket is claimed by some block before any
// block can exit on a stop (tickets are claimed in order and a block exits only at an unposted one).
__global__ __launch_bounds__(kSmallNT) void host_ring_kernel(HostRingArgs r) {
  __shared__ __align__(16) uint32_t s_desc[kHostRingDescBytes / 4];
  __shared__ uint32_t s_ticket, s_go;
  const uint32_t tid = threadIdx.x;
  for (;;) {
    if (tid == 0) {
      const uint32_t t = __hip_atomic_fetch_add(r.claim, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t* seq = reinterpret_cast<const uint32_t*>(r.desc + static_cast<size_t>(t & (r.slots - 1u)) *
                                                                           kHostRingDescBytes);
      uint64_t t_act = wall_clock64();
      uint32_t seen = __hip_atomic_load(&r.ctl->posted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      uint32_t go = 0;
      for (uint32_t nap = 1;; nap = min(2u * nap, 8u)) {
        if (__hip_atomic_load(seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) == t + 1u) {
          go = 1;
          break;
        }
        if (__hip_atomic_load(&r.ctl->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) break;
        const uint32_t p = __hip_atomic_load(&r.ctl->posted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (p != seen) {
          seen = p;
          t_act = wall_clock64();
        } else if (static_cast<uint64_t>(wall_clock64()) - t_act > r.idle_ticks) {
          __hip_atomic_store(&r.ctl->ended, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
        for (uint32_t i = 0; i < nap; ++i) __builtin_amdgcn_s_sleep(4);
      }
      s_ticket = t;
      s_go = go;
    }
    __syncthreads();
    if (!s_go) break;
    const uint32_t t = s_ticket;
    uint32_t* d = reinterpret_cast<uint32_t*>(r.desc + static_cast<size_t>(t & (r.slots - 1u)) * kHostRingDescBytes);
    if (tid < sizeof(HostRingDesc) / 4)
      s_desc[tid] = __hip_atomic_load(d + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __syncthreads();
    if (tid == 0) __hip_atomic_store(d + 1, t + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // ack: reusable
    const HostRingDesc& hd = *reinterpret_cast<const HostRingDesc*>(s_desc);
    const ClassifyArgs a = hd.a;
    const GroupArgs g = hd.g;
    switch (hd.variant & 15u) {
      case 0: small_body<kGlobalU8, false, 7>(a, g); break;
      case 1: small_body<kGlobalU16, false, 7>(a, g); break;
      case 2: small_body<kGlobalU8, true, 7>(a, g); break;
      case 3: small_body<kGlobalU16, true, 7>(a, g); break;
      case 4: small_body<kGlobalU8, false, 10>(a, g); break;
      case 5: small_body<kGlobalU16, false, 10>(a, g); break;
      case 6: small_body<kGlobalU8, true, 10>(a, g); break;
      case 7: small_body<kGlobalU16, true, 10>(a, g); break;
      case 8: small_body<kGlobalU8, false, 7, true>(a, g); break;
      case 9: small_body<kGlobalU16, false, 7, true>(a, g); break;
      case 10: small_body<kGlobalU8, true, 7, true>(a, g); break;
      case 11: small_body<kGlobalU16, true, 7, true>(a, g); break;
      case 12: small_body<kGlobalU8, false, 10, true>(a, g); break;
      case 13: small_body<kGlobalU16, false, 10, true>(a, g); break;
      case 14: small_body<kGlobalU8, true, 10, true>(a, g); break;
      default: small_body<kGlobalU16, true, 10, true>(a, g); break;
    }
    __threadfence_system();  // this thread's outputs are visible to the host
    __syncthreads();
    if (tid == 0) __hip_atomic_store(hd.done, hd.done_val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    __syncthreads();  // s_desc and the small body's LDS are reused by the next batch
  }
}

// ---- many backends (more than kMaxGroupBins - 1, up to 32767) ------------------------------------
// The multisplit group kernel keeps a counter row per wave and bin in LDS, which does not scale to
// 32768 bins.  Past 1023 backends the per-partition histograms (hist_kernel) and their prefix over
// partitions (scan_kernel) feed two small kernels: bin_base_kernel scans the bin totals into group
// bases (and writes counts), and group_wide_kernel walks each partition in packet order, one wave
// per partition, with one LDS counter per bin: a lane's position is its bin's base + the bin's
// prefix over earlier partitions + the bin's count so far in this partition + its rank among the
// lanes of its 64-packet step with the same bin (a readlane match over the step), so perm keeps the
// per-group FIFO order of group_by.rs:46-51 for any bin count.
__global__ __launch_bounds__(kGBlock) void bin_base_kernel(GroupArgs a) {
  __shared__ uint32_t s_wave[kGBlock / 64];
  const uint32_t nbins = a.nb + 1, tid = threadIdx.x;
  const uint32_t per = (nbins + kGBlock - 1) / kGBlock;  // consecutive bins per thread
  uint32_t s = 0;
  for (uint32_t k = 0; k < per; ++k) {
    const uint32_t b = tid * per + k;
    s += b < nbins ? a.totals[b] : 0u;
  }
  uint32_t all;
  uint32_t base = block_excl_scan_n<kGBlock>(s, s_wave, all);
  for (uint32_t k = 0; k < per; ++k) {
    const uint32_t b = tid * per + k;
    if (b < nbins) {
      const uint32_t t = a.totals[b];
      a.bin_base[b] = base;
      if (a.counts) a.counts[b] = t;
      base += t;
    }
  }
}

__global__ __launch_bounds__(64) void group_wide_kernel(GroupArgs a) {
  extern __shared__ __align__(16) uint32_t cnt[];  // [nbins]: packets of each bin seen so far
  const uint32_t nbins = a.nb + 1, lane = threadIdx.x, c = blockIdx.x;
  for (uint32_t b = lane; b < nbins; b += 64) cnt[b] = 0;
  const uint32_t pbeg = c * a.part_pkts, pend = min(pbeg + a.part_pkts, a.n_pkts);
  const uint32_t* prefix = a.part_prefix + static_cast<size_t>(c) * nbins;
  for (uint32_t i0 = pbeg; i0 < pend; i0 += 64u) {
    const uint32_t i = i0 + lane;
    const bool valid = i < pend;
    const uint32_t raw = ld_u16(a.backend, min(i, a.n_pkts - 1u) * 2u);
    const uint32_t bin = !valid ? 0xffffffffu : (raw == NBG_SENTINEL ? a.nb : raw);
    // rank among earlier lanes of this step with the same bin, and the bin's lanes in the step
    uint32_t rank, count;
    wave_match_rank<15>(valid ? bin : 0u, valid, lane, rank, count);
    // every lane reads its bin's count before any lane of the step writes one (one wave: its LDS
    // operations execute in issue order; the wave barriers keep the compiler from moving them)
    const uint32_t slot = valid ? bin : 0u;
    const uint32_t before = cnt[slot];
    __builtin_amdgcn_wave_barrier();
    if (valid && a.perm) a.perm[a.bin_base[bin] + prefix[bin] + before + rank] = i;
    if (valid) cnt[bin] = before + count;  // every lane of a bin stores the same new count
    __builtin_amdgcn_wave_barrier();
  }
}

// One 512-thread block per partition (part_pkts packets, processed in 4096-packet chunks): the
// stable per-group FIFO order of group_by.rs:46-51.  Wave w owns rounds [8w, 8w + 8) of 64 packets of
// every chunk (packet = chunk base + 512 w + 64 r + lane).
//   Entry: every global load of the block is issued at once: the first chunk's backends, then the
//     prologue's (kScanDirect: this partition's share of the L2-resident partition rows; kScanKernel:
//     scan_kernel's prefix row and the bin totals).  The first chunk is ranked while the prologue's
//     loads are in flight (a wave ballot multisplit per 64-packet round, one ballot per bin bit; the
//     wave's 16-bit LDS counter row carries its earlier rounds).
//   Then four barrier-separated phases per chunk: (1) the prologue's sums and the first half of the
//     chunk's bin-major exclusive scan over the (bin, wave) counters; (2) the group bases (exclusive
//     scan of the totals over bins) and the scan's write-back; (3) per bin, the perm position of the
//     chunk's first packet of the bin, and the local counting sort into LDS; (4) coalesced perm
//     stores (consecutive sorted slots of one bin are consecutive perm entries).
// The round-4 form ranked only after the prologue and took 8 barriers per chunk; its phase timeline
// (tools/gprobe.py, profiles/r05_gprobe_v1.txt) had the row prologue (1.84 us) and the ranks (1.55 us,
// VALU-bound) one after the other on each block's critical path.  The ranks take 4 VALU operations per
// bin bit (mismatch_all), the backends and the rows are raw buffer loads (no clamps, one 32-bit offset
// per lane): 11,324 instead of 14,954 cycles per C2 block (profiles/r05_gprobe_final.txt).  Up to 128
// bins a lane's peers come from a per-wave LDS table of lane masks instead (one OR, one read, one clear
// per round; 1,069 instead of 1,565 VALU instructions in the kernel): 11,026 cycles
// (profiles/r05_gprobe_peer.txt), the ranks now wait on the backends' HBM latency.
// 4 waves per SIMD (two resident blocks per CU, <= 128 VGPRs).
constexpr int kGroupWaves = 4;
// BITS: bin bits the multisplit compares (7 for up to 128 bins, else 10); unused high bits are 0
template <int SCAN, int BITS>
// Blocks [j * gm.per, j * gm.per + g[j].n_parts) group batch j (a single batch: j = 0, c = blockIdx.x).
__global__ __launch_bounds__(kGBlock, kGroupWaves) void group_kernel(GroupMulti gm) {
  extern __shared__ __align__(16) uint32_t gs[];
  __shared__ uint32_t s_wave[2][kGBlock / 64];
  constexpr uint32_t kW = kGBlock / 64;  // waves
  constexpr uint32_t kMaxBins = 1u << BITS;
  const uint32_t bj = blockIdx.x / gm.per;
  const GroupArgs a = gm.g[bj];
  const uint32_t nbins = a.nb + 1;
  const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u;
  // partition of batch bj, XCD-aware: the dispatcher deals blocks round-robin over the 8 XCDs, and
  // neighbouring partitions write adjacent pieces of every bin's perm run (~4 packets per bin and chunk
  // at 1001 bins), so XCD x takes partitions [x n / 8, (x + 1) n / 8) and the pieces of one line meet
  // in one L2: C3 hist + scan + group 20.5 -> 19.5 us, 8 per launch 6.8 -> 6.2 us per batch, C2 9.3 ->
  // 9.1 us (profiles/r05_group_xcd_ab.txt)
  const uint32_t c_lin = blockIdx.x - bj * gm.per;
  const uint32_t c = (a.n_parts % 8u == 0u && c_lin < a.n_parts) ? (c_lin % 8u) * (a.n_parts / 8u) + c_lin / 8u : c_lin;
  // The next call accumulates into the other histogram buffer: every block of the grid zeroes a
  // slice of it, last, after its perm stores.  Stores issued earlier would sit in vmcnt, and the
  // first wait for a backend load would also wait for them (the counter retires in issue order).
  auto zero_next = [&] {
    for (uint32_t i = blockIdx.x * kGBlock + tid; i < a.next_words; i += gridDim.x * kGBlock) a.part_hist_next[i] = 0;
  };
  if (c >= a.n_parts) {  // a smaller batch of a multi-batch launch
    zero_next();
    return;
  }
  const uint32_t nbp = (nbins + 3) & ~3u;
  uint32_t* base = gs;                 // [nbins] next perm position of this partition, per bin
  uint32_t* tot = base + nbp;          // [nbins] bin totals (prologue), then the chunk's perm bases
  // 16-bit per-wave counters (a wave counts <= 512 packets of a chunk; chunk slots < kChunk) and one
  // word per sorted slot (bin << 12 | packet within the chunk): 40 KB of LDS at 1001 bins
  static_assert(kChunk <= 4096 && kChunk == kGBlock * kGRounds, "sorted slots hold a 12-bit packet index");
  const uint32_t cst = (nbins + 8) & ~7u;  // cnt row stride: a scratch slot for lanes past the end; 16-B rows
  uint16_t* cnt = reinterpret_cast<uint16_t*>(tot + nbp);  // [kW][cst]
  uint32_t* sslot = reinterpret_cast<uint32_t*>(cnt + kW * cst);  // [kChunk]
  uint16_t* mycnt = cnt + wave * cst;
  // <= 128 bins: the lanes that share a lane's bin come from a per-wave table of 64-bit lane masks
  // [kW][nbins + 1] (slot nbins: lanes past the end), else from the ballot multisplit
  constexpr bool kPeer = BITS <= 7;
  unsigned long long* peer = reinterpret_cast<unsigned long long*>(sslot + kChunk) + wave * (nbins + 1);
  const bool perm = a.perm != nullptr;

  // ---- entry: the first chunk's backends, then the prologue's loads, all in flight together
  const uint32_t pbeg = c * a.part_pkts;
  const uint32_t pend = min(pbeg + a.part_pkts, a.n_pkts);
  const __amdgpu_buffer_rsrc_t rbe = raw_rsrc(a.backend, a.n_pkts * 2u);  // packets past the batch read 0
  uint32_t pre_bin[kGRounds];
  {
    const uint32_t wb = pbeg + wave * (64u * kGRounds);
#pragma unroll
    for (int r = 0; r < kGRounds; ++r) pre_bin[r] = __builtin_amdgcn_raw_buffer_load_b16(rbe, (wb + r * 64u + lane) * 2u, 0, 0);
  }
  // the scheduler keeps the backend loads ahead of the prologue's (vmcnt retires in issue order: the
  // ranks then wait for the backends only)
  __builtin_amdgcn_sched_barrier(0);
  // kScanDirect: thread (w, j) = (tid % hw, tid / hw) sums rows j, j + L, ... of row word w (L threads
  // per word; consecutive threads read consecutive words of one row); the first kU of its rows are
  // loaded here.  kScanKernel: this thread's consecutive bins of the prefix row and the totals.
  constexpr uint32_t kU = 18;  // 65 backends, 16-bit rows: 33 words, L = 15, 18 rows per thread
  constexpr uint32_t kCb = kMaxBins > kGBlock ? kMaxBins / kGBlock : 1u;  // consecutive bins per thread
  const uint32_t hw = a.hist16 ? (nbins + 1) >> 1 : nbins;  // row words
  const uint32_t L = hw >= kGBlock ? 1u : kGBlock / hw;
  const uint32_t rw0 = tid % hw, rj0 = tid / hw;  // this thread's first (word, row) pair
  uint32_t h[kU];
  uint32_t pk[kCb], tk[kCb];
  if constexpr (SCAN == kScanDirect) {
    // every thread loads its first (word, row) pair's first kU rows (a thread past hw * L ignores
    // them): a load inside a branch makes the compiler wait for all of them at the join, before the
    // ranks
    const __amdgpu_buffer_rsrc_t rrows = raw_rsrc(a.part_hist, a.n_parts * hw * 4u);  // rows past the last read 0
#pragma unroll
    for (uint32_t k = 0; k < kU; ++k) h[k] = __builtin_amdgcn_raw_buffer_load_b32(rrows, ((rj0 + k * L) * hw + rw0) * 4u, 0, 0);
  } else {
#pragma unroll
    for (uint32_t k = 0; k < kCb; ++k) {
      const uint32_t b = min(tid * kCb + k, nbins - 1u);
      pk[k] = ld_u32(a.part_prefix, (c * nbins + b) * 4u);
      tk[k] = ld_u32(a.totals, b * 4u);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  for (uint32_t b = tid; b < nbp; b += kGBlock) {
    base[b] = 0;
    tot[b] = 0;
  }
  // each wave clears its own peer table (its LDS operations execute in order: no barrier)
  if constexpr (kPeer)
    for (uint32_t b = lane; b <= nbins; b += 64) peer[b] = 0;

  const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const uint32_t lt_lo = static_cast<uint32_t>(lt), lt_hi = static_cast<uint32_t>(lt >> 32);
  uint32_t br[kGRounds];  // rank << 16 | bin (bins < kMaxGroupBins, ranks < kChunk), or ~0 past the end
  // one chunk's ranks (its backends in pre_bin); afterwards the next chunk's backends are loaded
  auto rank_chunk = [&](uint32_t cbase) {
    // each wave zeroes its own counter row: every reader of the previous chunk's counters has passed
    // a barrier since, and one wave's LDS operations execute in order
#pragma unroll
    for (uint32_t k = 0; k < (kMaxBins + 8 + 511) / 512; ++k)
      if ((lane + k * 64) * 8 < cst) reinterpret_cast<uint4*>(mycnt)[lane + k * 64] = make_uint4(0, 0, 0, 0);
    const uint32_t wbase = cbase + wave * (64u * kGRounds);
#pragma unroll
    for (int r = 0; r < kGRounds; ++r) {
      const uint32_t i = wbase + r * 64u + lane;
      const bool valid = i < pend;
      const uint32_t bin = min(pre_bin[r], a.nb);  // the sentinel (and any value > nb, as in hist_kernel)
      const uint32_t slot = valid ? bin : nbins;   // lanes past the end use the scratch slot
      uint32_t elo, ehi;                           // the lanes with my bin (and my validity)
      if constexpr (kPeer) {
        // every lane ORs its bit into its slot's mask, reads the mask back and clears it: three LDS
        // instructions of one wave, executed in order (the compiler barriers keep them in order)
        unsigned long long* pw = peer + slot;
        __hip_atomic_fetch_or(pw, 1ull << lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __asm__ volatile("" ::: "memory");
        const unsigned long long pm = *pw;
        __asm__ volatile("" ::: "memory");
        *pw = 0;
        elo = static_cast<uint32_t>(pm);
        ehi = static_cast<uint32_t>(pm >> 32);
      } else {
        // accumulate, per bin bit, the lanes whose ballot bit differs from mine; the rest match
        const uint32_t mv = valid ? ~0u : 0u;
        const unsigned long long bv = __builtin_amdgcn_ballot_w64(valid);
        uint32_t mlo = static_cast<uint32_t>(bv) ^ mv, mhi = static_cast<uint32_t>(bv >> 32) ^ mv;
        mismatch_all<BITS>(bin, mlo, mhi);
        elo = ~mlo;
        ehi = ~mhi;
      }
      // every lane of a bin stores the same new count (no branch)
      const uint32_t prior = mycnt[slot];
      mycnt[slot] = static_cast<uint16_t>(prior + __popc(elo) + __popc(ehi));
      const uint32_t rank = prior + __popc(elo & lt_lo) + __popc(ehi & lt_hi);
      br[r] = valid ? (rank << 16) | bin : 0xffffffffu;
    }
    // the next chunk's backends (partitions of more than one chunk): loaded now, behind this
    // chunk's scans and stores
    if (cbase + kChunk < pend) {
#pragma unroll
      for (int r = 0; r < kGRounds; ++r)
        pre_bin[r] = __builtin_amdgcn_raw_buffer_load_b16(rbe, (wbase + kChunk + r * 64u + lane) * 2u, 0, 0);
    }
  };
  if (perm) rank_chunk(pbeg);

  // bin-major exclusive scan over the chunk's (bin, wave) counters: the chunk-local slot where wave
  // w's packets of bin b start (each thread owns kPer consecutive elements: whole bins' wave counters
  // when kPer >= kW); first half: the wave-level scan
  constexpr uint32_t kPer = (kMaxBins * kW + kGBlock - 1) / kGBlock;
  const uint32_t ne = nbins * kW;
  uint32_t ev[kPer], esum = 0, ex = 0;
  // kPer == 2 * kW (10 bits): a thread's elements are bins 2t and 2t + 1 of every wave's row, one
  // 32-bit LDS word per wave (the rows are 16-B aligned, cst even)
  constexpr bool kPair = kPer == 2 * kW;
  auto chunk_scan_begin = [&] {
    esum = 0;
    if constexpr (kPair) {
#pragma unroll
      for (uint32_t w = 0; w < kW; ++w) {
        const uint32_t v = 2 * tid < nbins ? reinterpret_cast<const uint32_t*>(cnt + w * cst)[tid] : 0u;
        ev[w] = v & 0xffffu;
        ev[kW + w] = 2 * tid + 1 < nbins ? v >> 16 : 0u;
      }
#pragma unroll
      for (uint32_t k = 0; k < kPer; ++k) esum += ev[k];
      ex = wave_incl_scan(esum);
      if (lane == 63u) s_wave[0][wave] = ex;
      return;
    }
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {
      const uint32_t e = tid * kPer + k;
      ev[k] = e < ne ? cnt[(e % kW) * cst + e / kW] : 0u;
      esum += ev[k];
    }
    ex = wave_incl_scan(esum);
    if (lane == 63u) s_wave[0][wave] = ex;
  };
  // second half (after a barrier): the wave's offset, the write-back; returns the chunk's packets
  auto chunk_scan_end = [&]() -> uint32_t {
    uint32_t wpre = 0, ctotal = 0;
#pragma unroll
    for (uint32_t w = 0; w < kW; ++w) {
      const uint32_t t = s_wave[0][w];
      wpre += w < wave ? t : 0u;
      ctotal += t;
    }
    uint32_t x = wpre + ex - esum;
    if constexpr (kPair) {
      uint32_t lo[kW];
#pragma unroll
      for (uint32_t w = 0; w < kW; ++w) {  // bin 2t over the waves, then bin 2t + 1
        lo[w] = x;
        x += ev[w];
      }
#pragma unroll
      for (uint32_t w = 0; w < kW; ++w) {
        if (2 * tid < nbins) reinterpret_cast<uint32_t*>(cnt + w * cst)[tid] = lo[w] | (x << 16);
        x += ev[kW + w];
      }
      return ctotal;
    }
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {
      const uint32_t e = tid * kPer + k;
      if (e < ne) cnt[(e % kW) * cst + e / kW] = static_cast<uint16_t>(x);
      x += ev[k];
    }
    return ctotal;
  };

  lds_sync();  // (B1) base / tot zeroed, every wave's counts of the first chunk in LDS

  // ---- (1) prologue sums, the chunk scan's first half
  uint32_t gs_incl = 0, gs_own = 0;  // kScanKernel: this thread's bins' totals, scanned over the wave
  if constexpr (SCAN == kScanDirect) {
    // (word, row) pair (rw, rj): rows rj, rj + L, ...; the first kU of the first pair's rows are in
    // h[] (static indices only, so that h stays in registers), any further rows are loaded one by one
    // (more than kU rows per thread, or more than kGBlock row words: many bins, rare)
    auto add_row = [&](uint32_t q, uint32_t v, uint32_t (&acc)[4]) {
      const uint32_t lo = q < a.n_parts ? (a.hist16 ? v & 0xffffu : v) : 0u;
      const uint32_t hi = q < a.n_parts && a.hist16 ? v >> 16 : 0u;
      acc[0] += q < c ? lo : 0u;
      acc[1] += q < c ? hi : 0u;
      acc[2] += lo;
      acc[3] += hi;
    };
    auto publish = [&](uint32_t rw, const uint32_t (&acc)[4]) {
      const uint32_t b0 = a.hist16 ? 2 * rw : rw;
      atomicAdd(&base[b0], acc[0]);
      atomicAdd(&tot[b0], acc[2]);
      if (a.hist16 && b0 + 1 < nbins) {
        atomicAdd(&base[b0 + 1], acc[1]);
        atomicAdd(&tot[b0 + 1], acc[3]);
      }
    };
    if (tid < hw * L) {
      uint32_t acc[4] = {0u, 0u, 0u, 0u};
      if (a.hist16 && a.part_pkts * 15u < 65536u) {
        // packed: the two 16-bit bins of a row word are summed by one 32-bit add, at most 15 rows per
        // partial sum (15 partitions' counts of one bin fit 16 bits); rows past the last read 0
        uint32_t pall = 0, ppre = 0;
#pragma unroll
        for (uint32_t k = 0; k < kU; ++k) {
          pall += h[k];
          ppre += rj0 + k * L < c ? h[k] : 0u;
          if (k % 15u == 14u || k == kU - 1u) {
            acc[0] += ppre & 0xffffu;
            acc[1] += ppre >> 16;
            acc[2] += pall & 0xffffu;
            acc[3] += pall >> 16;
            pall = ppre = 0;
          }
        }
      } else {
#pragma unroll
        for (uint32_t k = 0; k < kU; ++k) add_row(rj0 + k * L, h[k], acc);
      }
      for (uint32_t q = rj0 + kU * L; q < a.n_parts; q += L) add_row(q, ld_u32(a.part_hist, (q * hw + rw0) * 4u), acc);
      publish(rw0, acc);
    }
    for (uint32_t t = tid + kGBlock; t < hw * L; t += kGBlock) {
      uint32_t acc[4] = {0u, 0u, 0u, 0u};
      const uint32_t rw = t % hw;
      for (uint32_t q = t / hw; q < a.n_parts; q += L) add_row(q, ld_u32(a.part_hist, (q * hw + rw) * 4u), acc);
      publish(rw, acc);
    }
  } else {
#pragma unroll
    for (uint32_t k = 0; k < kCb; ++k) gs_own += tid * kCb + k < nbins ? tk[k] : 0u;
    gs_incl = wave_incl_scan(gs_own);
    if (lane == 63u) s_wave[1][wave] = gs_incl;
  }
  if (perm) chunk_scan_begin();
  lds_sync();  // (B2)

  // ---- (2) group bases (exclusive scan of the totals over bins), the chunk scan's write-back
  if constexpr (SCAN == kScanDirect && kMaxBins <= 128) {  // one wave, <= 2 bins per lane
    if (wave == 0) {
      uint32_t t2[2], s = 0;
#pragma unroll
      for (uint32_t k = 0; k < 2; ++k) {
        const uint32_t b = lane * 2 + k;
        t2[k] = b < nbins ? tot[b] : 0u;
        s += t2[k];
      }
      uint32_t gb = wave_incl_scan(s) - s;
#pragma unroll
      for (uint32_t k = 0; k < 2; ++k) {
        const uint32_t b = lane * 2 + k;
        if (b < nbins) {
          if (c == 0 && a.counts) a.counts[b] = t2[k];
          base[b] += gb;  // group base + prefix over earlier partitions
        }
        gb += t2[k];
      }
    }
  } else if constexpr (SCAN == kScanDirect) {  // many bins summed here: a block-wide scan of tot[]
    uint32_t tb[kCb], s = 0;
#pragma unroll
    for (uint32_t k = 0; k < kCb; ++k) {
      const uint32_t b = tid * kCb + k;
      tb[k] = b < nbins ? tot[b] : 0u;
      s += tb[k];
    }
    uint32_t all;
    uint32_t gb = block_excl_scan_n<kGBlock>(s, s_wave[1], all);
#pragma unroll
    for (uint32_t k = 0; k < kCb; ++k) {
      const uint32_t b = tid * kCb + k;
      if (b < nbins) {
        if (c == 0 && a.counts) a.counts[b] = tb[k];
        base[b] += gb;
      }
      gb += tb[k];
    }
  } else {  // the wave-level scan of (1) completed across waves
    uint32_t gb = gs_incl - gs_own;
#pragma unroll
    for (uint32_t w = 0; w < kW; ++w) gb += w < wave ? s_wave[1][w] : 0u;
#pragma unroll
    for (uint32_t k = 0; k < kCb; ++k) {
      const uint32_t b = tid * kCb + k;
      if (b < nbins) {
        if (c == 0 && a.counts) a.counts[b] = tk[k];
        base[b] = pk[k] + gb;
      }
      gb += tk[k];
    }
  }
  if (!perm) {
    zero_next();
    return;
  }
  uint32_t ctotal = chunk_scan_end();
  for (uint32_t cbase = pbeg;;) {
    lds_sync();  // (B3)
    // ---- (3) per bin: perm position of chunk slot j of bin b = tot[b] + j; advance past the bin.
    // Local counting sort of the chunk's packets into LDS.
    for (uint32_t b = tid; b < nbins; b += kGBlock) {
      const uint32_t st = cnt[b];                                // wave 0's start = the bin's start
      const uint32_t en = b + 1 < nbins ? cnt[b + 1] : ctotal;
      tot[b] = base[b] - st;
      base[b] += en - st;
    }
    const uint32_t wbase = cbase + wave * (64u * kGRounds);
#pragma unroll
    for (int r = 0; r < kGRounds; ++r) {
      if (br[r] != 0xffffffffu) {
        const uint32_t bin = br[r] & 0xffffu;
        const uint32_t j = mycnt[bin] + (br[r] >> 16);
        sslot[j] = (bin << 12) | (wbase - cbase + r * 64u + lane);
      }
    }
    lds_sync();  // (B4)
    // ---- (4) coalesced output, unrolled: the slot reads, then the dependent base reads, issue back
    // to back (a loop paid two LDS round trips per iteration)
    {
      uint32_t sv[kGRounds], pb[kGRounds];
#pragma unroll
      for (int k = 0; k < kGRounds; ++k) sv[k] = sslot[tid + k * kGBlock];  // < kChunk; slots >= ctotal unused
#pragma unroll
      for (int k = 0; k < kGRounds; ++k) pb[k] = tot[min(sv[k] >> 12, nbins - 1u)];
#pragma unroll
      for (int k = 0; k < kGRounds; ++k) {
        const uint32_t j = tid + k * kGBlock;
        if (j < ctotal) a.perm[pb[k] + j] = cbase + (sv[k] & 0xfffu);
      }
    }
    cbase += kChunk;
    if (cbase >= pend) break;
    // the next chunk (its backends are loaded): ranks, then the scan's two halves
    rank_chunk(cbase);
    lds_sync();
    chunk_scan_begin();
    lds_sync();
    ctotal = chunk_scan_end();
  }
  zero_next();
}

// group_direct_kernel: the compact form of group_kernel, for many bins beside an in-place
// persistent ring (whose blocks leave ~30 KB of a CU's LDS; group_kernel takes 40 KB at 1001 bins
// and would wait for the ring to end).  Same grid, arguments and outputs.  One 512-thread block per
// partition (part_pkts packets, processed in 4096-packet chunks): the stable per-group FIFO order
// of group_by.rs:46-51.  Wave w owns the contiguous 512-packet segment [512w, 512w + 512) of every
// chunk, 8 rounds of 64 packets.
//   Ranks: per round a ballot multisplit (one ballot per bin bit) gives every lane its rank among
//     the round's lanes of its bin; the wave's LDS counter row (16 bit per bin) carries the counts
//     of its earlier rounds.  The first chunk is ranked while the prologue's loads are in flight.
//   Prologue: this partition's prefix over earlier partitions and the bin totals, summed from the
//     L2-resident partition rows (few bins) or read from scan_kernel's output; group bases (an
//     exclusive scan of the totals over bins) give run[b], the perm position of the partition's
//     first packet of bin b.
//   Per chunk, one pass over the bins turns each bin's 8 wave counts into exclusive prefixes (and
//     advances run[] past the chunk), then every lane stores perm[run[b] + prefix[w][b] + rank] =
//     its packet directly, without the local sort (measured 1-2 us per 1M batch slower than
//     group_kernel's coalesced stores: profiles/r05_group_ab.txt).
// LDS: run[2][nbins] + tot[nbins] u32, cnt[8][nbins] u16: 28 KB at 1001 bins.
template <int SCAN, int BITS>
__global__ __launch_bounds__(kGBlock, kGroupWaves) void group_direct_kernel(GroupMulti gm) {
  extern __shared__ __align__(16) uint32_t gs[];
  __shared__ uint32_t s_wave[kGBlock / 64];
  constexpr uint32_t kW = kGBlock / 64;  // waves
  static_assert(kChunk == kGBlock * kGRounds && kChunk / kW <= 65535, "16-bit per-wave counters");
  const uint32_t bj = blockIdx.x / gm.per;
  const GroupArgs a = gm.g[bj];
  const uint32_t nbins = a.nb + 1;
  const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u;
  // partition of batch bj, XCD-aware as in group_kernel (neighbouring partitions on one XCD)
  const uint32_t c_lin = blockIdx.x - bj * gm.per;
  const uint32_t c = (a.n_parts % 8u == 0u && c_lin < a.n_parts) ? (c_lin % 8u) * (a.n_parts / 8u) + c_lin / 8u : c_lin;
  // The next call accumulates into the other histogram buffer: every block of the grid zeroes a
  // slice of it, last, after its perm stores.  Stores issued earlier would sit in vmcnt, and the
  // first wait for a backend load would also wait for them (the counter retires in issue order).
  auto zero_next = [&] {
    for (uint32_t i = blockIdx.x * kGBlock + tid; i < a.next_words; i += gridDim.x * kGBlock) a.part_hist_next[i] = 0;
  };
  if (c >= a.n_parts) {  // a smaller batch of a multi-batch launch
    zero_next();
    return;
  }
  const uint32_t nbp = (nbins + 3) & ~3u;
  const uint32_t cst = (nbins + 8) & ~7u;  // cnt row stride: a scratch slot for lanes past the end; 16-B rows
  uint32_t* run = gs;                      // [2][nbp] by chunk parity
  uint32_t* tot = run + 2 * nbp;           // [nbp] bin totals (prologue)
  uint16_t* cnt = reinterpret_cast<uint16_t*>(tot + nbp);  // [kW][cst]
  uint16_t* mycnt = cnt + wave * cst;
  constexpr uint32_t kMaxBins = 1u << BITS;

  // ---- the first chunk's backends, then the prologue's loads: all in flight together
  const uint32_t pbeg = c * a.part_pkts;
  const uint32_t pend = min(pbeg + a.part_pkts, a.n_pkts);
  uint32_t pre_bin[kGRounds];
  {
    const uint32_t wb = pbeg + wave * (64u * kGRounds);
#pragma unroll
    for (int r = 0; r < kGRounds; ++r) pre_bin[r] = ld_u16(a.backend, min(wb + r * 64u + lane, a.n_pkts - 1u) * 2u);
  }
  // kScanDirect: L threads per row word, each summing a strided subset of the partition rows (its
  // first kU rows loaded here); kScanKernel: this partition's prefix row and the totals
  constexpr uint32_t kU = 24;
  const uint32_t hw = a.hist16 ? (nbins + 1) >> 1 : nbins;  // row words
  const uint32_t L = hw >= kGBlock ? 1u : kGBlock / hw;
  uint32_t h[kU];
  constexpr uint32_t kCh = (kMaxBins + kGBlock - 1) / kGBlock;
  uint32_t pk[kCh], tk[kCh];
  auto load_rows = [&](uint32_t t, uint32_t q0) {
#pragma unroll
    for (uint32_t k = 0; k < kU; ++k) h[k] = ld_u32(a.part_hist, (min(q0 + k * L, a.n_parts - 1u) * hw + t % hw) * 4u);
  };
  if constexpr (SCAN == kScanDirect) {
    if (tid < hw * L) load_rows(tid, tid / hw);
  } else {
#pragma unroll
    for (uint32_t k = 0; k < kCh; ++k) {
      const uint32_t b = min(tid + k * kGBlock, nbins - 1u);
      pk[k] = a.part_prefix[static_cast<size_t>(c) * nbins + b];
      tk[k] = a.totals[b];
    }
  }

  const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const uint32_t lt_lo = static_cast<uint32_t>(lt), lt_hi = static_cast<uint32_t>(lt >> 32);
  uint32_t br[kGRounds];  // rank << 16 | bin, or ~0 past the end
  // one chunk's ranks (its backends in pre_bin); afterwards the next chunk's backends are loaded
  auto rank_chunk = [&](uint32_t cbase) {
#pragma unroll
    for (uint32_t k = 0; k < (kMaxBins + 8 + 511) / 512; ++k)
      if ((lane + k * 64) * 8 < cst) reinterpret_cast<uint4*>(mycnt)[lane + k * 64] = make_uint4(0, 0, 0, 0);
    const uint32_t wbase = cbase + wave * (64u * kGRounds);
#pragma unroll
    for (int r = 0; r < kGRounds; ++r) {
      const uint32_t i = wbase + r * 64u + lane;
      const bool valid = i < pend;
      const uint32_t bin = min(pre_bin[r], a.nb);  // the sentinel (and any value > nb, as in hist_kernel)
      // lanes with my bin (and my validity): accumulate, per bit, the lanes whose ballot bit differs
      // from mine; the rest match
      const uint32_t mv = valid ? ~0u : 0u;
      const unsigned long long bv = __builtin_amdgcn_ballot_w64(valid);
      uint32_t mlo = static_cast<uint32_t>(bv) ^ mv, mhi = static_cast<uint32_t>(bv >> 32) ^ mv;
      mismatch_all<BITS>(bin, mlo, mhi);
      const uint32_t elo = ~mlo, ehi = ~mhi;
      // every lane of a bin stores the same new count (no branch); lanes past the end use the
      // scratch slot
      const uint32_t slot = valid ? bin : nbins;
      const uint32_t prior = mycnt[slot];
      mycnt[slot] = static_cast<uint16_t>(prior + __popc(elo) + __popc(ehi));
      const uint32_t rank = prior + __popc(elo & lt_lo) + __popc(ehi & lt_hi);
      br[r] = valid ? (rank << 16) | bin : 0xffffffffu;
    }
    if (cbase + kChunk < pend) {
#pragma unroll
      for (int r = 0; r < kGRounds; ++r)
        pre_bin[r] = ld_u16(a.backend, min(wbase + kChunk + r * 64u + lane, a.n_pkts - 1u) * 2u);
    }
  };
  if (a.perm) rank_chunk(pbeg);

  // ---- prologue: per-bin prefix over earlier partitions (run[0]) and totals
  if constexpr (SCAN == kScanDirect) {
    for (uint32_t b = tid; b < nbp; b += kGBlock) {
      run[b] = 0;
      tot[b] = 0;
    }
    lds_sync();
    // the first (thread, word) pair's rows are loaded already; more than kGBlock row words (many bins,
    // 16-bit rows off) take further pairs
    for (uint32_t t = tid; t < hw * L; t += kGBlock) {
      const uint32_t w = t % hw, j = t / hw;
      if (t != tid) load_rows(t, j);
      uint32_t pre_lo = 0, pre_hi = 0, all_lo = 0, all_hi = 0;
      for (uint32_t q0 = j;;) {
#pragma unroll
        for (uint32_t k = 0; k < kU; ++k) {
          const uint32_t q = q0 + k * L;
          const uint32_t lo = q < a.n_parts ? (a.hist16 ? h[k] & 0xffffu : h[k]) : 0u;
          const uint32_t hi = q < a.n_parts && a.hist16 ? h[k] >> 16 : 0u;
          all_lo += lo;
          all_hi += hi;
          pre_lo += q < c ? lo : 0u;
          pre_hi += q < c ? hi : 0u;
        }
        q0 += kU * L;
        if (q0 >= a.n_parts) break;
        load_rows(t, q0);
      }
      const uint32_t b0 = a.hist16 ? 2 * w : w;
      if (pre_lo) atomicAdd(&run[b0], pre_lo);
      if (all_lo) atomicAdd(&tot[b0], all_lo);
      if (a.hist16 && b0 + 1 < nbins) {
        if (pre_hi) atomicAdd(&run[b0 + 1], pre_hi);
        if (all_hi) atomicAdd(&tot[b0 + 1], all_hi);
      }
    }
    lds_sync();
  }
  // group bases: an exclusive scan of the totals over bins.  Loops have compile-time trip counts
  // (bins < 2^BITS) so that their LDS reads issue back to back.
  if constexpr (SCAN == kScanDirect && kMaxBins <= 128) {  // one wave, <= 2 bins per lane
    if (wave == 0) {
      uint32_t t2[2], s = 0;
#pragma unroll
      for (uint32_t k = 0; k < 2; ++k) {
        const uint32_t b = lane * 2 + k;
        t2[k] = b < nbins ? tot[b] : 0u;
        s += t2[k];
      }
      uint32_t gb = wave_incl_scan(s) - s;
#pragma unroll
      for (uint32_t k = 0; k < 2; ++k) {
        const uint32_t b = lane * 2 + k;
        if (b < nbins) {
          if (c == 0 && a.counts) a.counts[b] = t2[k];
          run[b] += gb;  // group base + prefix over earlier partitions
        }
        gb += t2[k];
      }
    }
  } else {  // the whole block; bin b = tid + k * kGBlock... scanned in thread-major order below
    constexpr uint32_t kCb = (kMaxBins + kGBlock - 1) / kGBlock;  // consecutive bins per thread
    uint32_t tb[kCb], pb[kCb], s = 0;
    if constexpr (SCAN == kScanDirect) {
#pragma unroll
      for (uint32_t k = 0; k < kCb; ++k) {
        const uint32_t b = tid * kCb + k;
        tb[k] = b < nbins ? tot[b] : 0u;
        pb[k] = b < nbins ? run[b] : 0u;
      }
    } else {  // this thread's loaded bins (tid + k * kGBlock) to consecutive ones through LDS
#pragma unroll
      for (uint32_t k = 0; k < kCh; ++k) {
        const uint32_t b = tid + k * kGBlock;
        if (b < nbins) {
          run[b] = pk[k];
          tot[b] = tk[k];
        }
      }
      lds_sync();
#pragma unroll
      for (uint32_t k = 0; k < kCb; ++k) {
        const uint32_t b = tid * kCb + k;
        tb[k] = b < nbins ? tot[b] : 0u;
        pb[k] = b < nbins ? run[b] : 0u;
      }
    }
#pragma unroll
    for (uint32_t k = 0; k < kCb; ++k) s += tb[k];
    uint32_t all;
    uint32_t gb = block_excl_scan_n<kGBlock>(s, s_wave, all);
#pragma unroll
    for (uint32_t k = 0; k < kCb; ++k) {
      const uint32_t b = tid * kCb + k;
      if (b < nbins) {
        if (c == 0 && a.counts) a.counts[b] = tb[k];
        run[b] = pb[k] + gb;
      }
      gb += tb[k];
    }
  }
  if (!a.perm) {
    zero_next();
    return;
  }

  // ---- per chunk: wave prefixes per bin, then the stores (the first chunk is ranked already)
  uint32_t par = 0;
  for (uint32_t cbase = pbeg;;) {
    lds_sync();  // every wave's counts of the chunk (and, the first time, run[]) are in LDS
    for (uint32_t b = tid; b < nbins; b += kGBlock) {
      uint32_t s = 0;
#pragma unroll
      for (uint32_t w = 0; w < kW; ++w) {
        const uint32_t t = cnt[w * cst + b];
        cnt[w * cst + b] = static_cast<uint16_t>(s);
        s += t;
      }
      run[(par ^ 1u) * nbp + b] = run[par * nbp + b] + s;
    }
    lds_sync();
    const uint32_t* rb = run + par * nbp;
    const uint32_t wbase = cbase + wave * (64u * kGRounds);
#pragma unroll
    for (int r = 0; r < kGRounds; ++r) {
      if (br[r] != 0xffffffffu) {
        const uint32_t bin = br[r] & 0xffffu;
        a.perm[rb[bin] + mycnt[bin] + (br[r] >> 16)] = wbase + r * 64u + lane;
      }
    }
    cbase += kChunk;
    if (cbase >= pend) break;
    par ^= 1u;
    rank_chunk(cbase);  // its own counter row only: the other waves' prefixes are read by now
  }
  zero_next();
}

template <int LUTM, bool F4, bool HIST, bool CHAIN>
int launch_one(const ClassifyArgs& a, int grid, size_t lds, hipStream_t s) {
  constexpr int NT = (LUTM == kLdsU8 || LUTM == kLdsU16) ? kLdsBlock : kBlock;
  auto fn = a.off ? classify_kernel<LUTM, F4, HIST, CHAIN, kDesc, NT>
                  : (a.lean ? classify_kernel<LUTM, F4, HIST, CHAIN, kLean, NT>
                            : classify_kernel<LUTM, F4, HIST, CHAIN, kFixed, NT>);

  hipLaunchKernelGGL(fn, dim3(grid), dim3(NT), lds, s, a);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(NBG_EIO, "classify launch: %s", hipGetErrorString(e));
  return NBG_OK;
}

template <int LUTM, bool F4, bool HIST>
int launch_v(const ClassifyArgs& a, int grid, size_t lds, hipStream_t s) {
  if (a.tbl24) return launch_one<LUTM, F4, HIST, true>(a, grid, lds, s);
  return launch_one<LUTM, F4, HIST, false>(a, grid, lds, s);
}

template <int LUTM>
int launch_mode(const ClassifyArgs& a, bool hist, int grid, size_t lds, hipStream_t s) {
  if (a.m == 65537u)
    return hist ? launch_v<LUTM, true, true>(a, grid, lds, s) : launch_v<LUTM, true, false>(a, grid, lds, s);
  return hist ? launch_v<LUTM, false, true>(a, grid, lds, s) : launch_v<LUTM, false, false>(a, grid, lds, s);
}

template <bool F4, bool HIST, int GB>
int launch_stream_mode(const ClassifyArgs& a, const StreamBatches& sb, const LagGroup& lg, int mode, int grid,
                       size_t lds, hipStream_t s) {
  auto fn = mode == 1 ? classify_stream_kernel<F4, HIST, 1, GB>
                      : (mode == 2 ? classify_stream_kernel<F4, HIST, 2, GB> : classify_stream_kernel<F4, HIST, 0, GB>);
  static bool attr_set[2][2][3] = {};
  if (!attr_set[F4][HIST][mode]) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024) != hipSuccess)
      return set_error(NBG_EIO, "streaming classify: LDS attribute: %s", hipGetErrorString(hipGetLastError()));
    attr_set[F4][HIST][mode] = true;
  }
  hipLaunchKernelGGL(fn, dim3(grid), dim3(kStreamNT), lds, s, a, sb, lg);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(NBG_EIO, "streaming classify launch: %s", hipGetErrorString(e));
  return NBG_OK;
}

template <int LUTM, bool F4, bool HIST, int MODE, bool CHAIN>
int launch_desc_v(const ClassifyArgs& a, int grid, size_t lds, hipStream_t s) {
  auto fn = classify_stream_desc_kernel<LUTM, F4, HIST, MODE, CHAIN>;
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024) != hipSuccess)
      return set_error(NBG_EIO, "streaming classify (descriptors): LDS attribute: %s",
                       hipGetErrorString(hipGetLastError()));
    attr_set = true;
  }
  hipLaunchKernelGGL(fn, dim3(grid), dim3(kStreamNT), lds, s, a);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(NBG_EIO, "streaming classify (descriptors) launch: %s", hipGetErrorString(e));
  return NBG_OK;
}

template <int LUTM, bool F4, bool HIST>
int launch_desc_mode(const ClassifyArgs& a, int mode, int grid, size_t lds, hipStream_t s) {
  if (a.tbl24) {
    if constexpr (LUTM == kLdsU8Tail) return launch_desc_v<LUTM, F4, HIST, 0, true>(a, grid, lds, s);
    return set_error(NBG_EINVAL, "streaming classify (descriptors): chain needs the u8 LUT");
  }
  if (mode == 2) return launch_desc_v<LUTM, F4, HIST, 2, false>(a, grid, lds, s);
  if (mode == 1) {
    if constexpr (LUTM == kGlobalU16) return launch_desc_v<LUTM, F4, HIST, 1, false>(a, grid, lds, s);
    return set_error(NBG_EINVAL, "streaming classify (descriptors): in place needs the u16 LUT");
  }
  return launch_desc_v<LUTM, F4, HIST, 0, false>(a, grid, lds, s);
}

template <int LUTM>
int launch_desc_lut(const ClassifyArgs& a, int mode, int grid, size_t lds, hipStream_t s) {
  const bool hist = a.part_hist != nullptr;
  if (a.m == 65537u)
    return hist ? launch_desc_mode<LUTM, true, true>(a, mode, grid, lds, s)
                : launch_desc_mode<LUTM, true, false>(a, mode, grid, lds, s);
  return hist ? launch_desc_mode<LUTM, false, true>(a, mode, grid, lds, s)
              : launch_desc_mode<LUTM, false, false>(a, mode, grid, lds, s);
}

// The block histogram is allocated only when the kernel keeps one (HIST): C3's 1001 bins would
// otherwise cost every 256-thread block 4 KB of the LDS a co-resident group block needs.
size_t classify_lds(uint32_t nb, uint32_t lut_lds_bytes, bool hist = true) {
  const uint32_t waves = (lut_lds_bytes ? kLdsBlock : kBlock) / 64;
  return static_cast<size_t>(lut_lds_bytes) + waves * 64u * kXStride + (hist ? static_cast<size_t>(nb + 1) * 4 : 0u);
}

}  // namespace

size_t stream_lds(uint32_t nb, int mode, bool lag) {
  const uint32_t hstride = ((nb + 1) + 3) & ~3u;
  const size_t tile = 64u * (mode == 1 ? stream_row_of<1>() : stream_row_of<0>());
  // past the histograms: the lag state, or the waves' backend words (64 x 2 B each)
  const size_t words = 2 * hstride + (lag ? lag_lds_words(hstride) : kStreamW * 32u);
  return kLutLds + static_cast<size_t>(kStreamW) * kRing * tile + words * 4u;
}

int stream_waves_per_block() { return kStreamW; }

size_t stream_desc_lds(uint32_t nb, int mode, bool wide_lut) {
  const size_t hwords = 2 * (((nb + 1) + 3) & ~3u);
  const size_t wave = mode == 1 ? desc_wave_lds<1>() : (mode == 2 ? desc_wave_lds<2>() : desc_wave_lds<0>());
  return (wide_lut ? 0u : kLutLds) + static_cast<size_t>(kStreamW) * wave + hwords * 4u;
}

int launch_classify_stream_desc(const ClassifyArgs& a, bool wide_lut, int grid, void* stream) {
  const int mode = a.tbl24 || !a.swap ? 0 : (a.mac_out ? 2 : 1);
  const size_t lds = stream_desc_lds(a.nb, mode, wide_lut);
  if (lds > 160u * 1024u) return set_error(NBG_EINVAL, "streaming classify (descriptors): %zu B of LDS", lds);
  hipStream_t s = static_cast<hipStream_t>(stream);
  return wide_lut ? launch_desc_lut<kGlobalU16>(a, mode, grid, lds, s) : launch_desc_lut<kLdsU8Tail>(a, mode, grid, lds, s);
}

int launch_classify_stream_multi(const ClassifyArgs& a, const StreamBatches& sb, int grid, void* stream) {
  const bool hist = a.part_hist != nullptr;
  const int mode = !a.swap ? 0 : (a.mac_out ? 2 : 1);
  const size_t lds = stream_lds(a.nb, mode, false);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const LagGroup none{};
  if (a.m == 65537u)
    return hist ? launch_stream_mode<true, true, 0>(a, sb, none, mode, grid, lds, s)
                : launch_stream_mode<true, false, 0>(a, sb, none, mode, grid, lds, s);
  return hist ? launch_stream_mode<false, true, 0>(a, sb, none, mode, grid, lds, s)
              : launch_stream_mode<false, false, 0>(a, sb, none, mode, grid, lds, s);
}

int launch_classify_stream_lag(const ClassifyArgs& a, const LagGroup& lg, int grid, void* stream) {
  const uint32_t nbins = a.nb + 1;
  if (!a.part_hist || nbins > 512 || lg.n_parts > static_cast<uint32_t>(grid))
    return set_error(NBG_EINVAL, "streaming classify (lagged group): %u bins, %u partitions on %d blocks", nbins,
                     lg.n_parts, grid);
  StreamBatches sb{};
  sb.pkts[0] = a.pkts;
  sb.backend[0] = a.backend;
  sb.mac_out[0] = a.mac_out;
  sb.part_hist[0] = a.part_hist;
  sb.n_pkts[0] = a.n_pkts;
  sb.unit_base[0] = 0;
  sb.unit_base[1] = (((a.n_pkts + 63u) >> 6) + kStreamW - 1) / kStreamW;
  sb.n = 1;
  const int mode = !a.swap ? 0 : (a.mac_out ? 2 : 1);
  const size_t lds = stream_lds(a.nb, mode, true);
  if (lds > 160u * 1024u) return set_error(NBG_EINVAL, "streaming classify (lagged group): %zu B of LDS", lds);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool b7 = nbins <= 128;
  if (a.m == 65537u)
    return b7 ? launch_stream_mode<true, true, 7>(a, sb, lg, mode, grid, lds, s)
              : launch_stream_mode<true, true, 9>(a, sb, lg, mode, grid, lds, s);
  return b7 ? launch_stream_mode<false, true, 7>(a, sb, lg, mode, grid, lds, s)
            : launch_stream_mode<false, true, 9>(a, sb, lg, mode, grid, lds, s);
}

size_t ring_lds(int mode) {
  const size_t tile = 64u * (mode == 1 ? stream_row_of<1>() : stream_row_of<0>());
  return kLutLds + static_cast<size_t>(kStreamW) * kRing * tile + kRingCtlWords * 4u;
}

int launch_classify_ring(const ClassifyArgs& a, const RingArgs& r, int mode, int grid, void* stream) {
  const bool f4 = a.m == 65537u;
  auto fn = mode == 1 ? (f4 ? classify_ring_kernel<true, 1> : classify_ring_kernel<false, 1>)
                      : (f4 ? classify_ring_kernel<true, 0> : classify_ring_kernel<false, 0>);
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=
      hipSuccess)
    return set_error(NBG_EIO, "ring classify: LDS attribute: %s", hipGetErrorString(hipGetLastError()));
  hipLaunchKernelGGL(fn, dim3(grid), dim3(kRingNT), ring_lds(mode), static_cast<hipStream_t>(stream), a, r);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(NBG_EIO, "ring classify launch: %s", hipGetErrorString(e));
  return NBG_OK;
}

int launch_ring_gate(const uint32_t* dcomp, const uint32_t* dexit, uint32_t target, uint32_t grid, void* stream) {
  hipLaunchKernelGGL(ring_gate_kernel, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream), dcomp, dexit, target,
                     grid);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(NBG_EIO, "ring gate launch: %s", hipGetErrorString(e));
  return NBG_OK;
}

int launch_classify_stream(const ClassifyArgs& a, int grid, void* stream) {
  StreamBatches sb{};
  sb.pkts[0] = a.pkts;
  sb.backend[0] = a.backend;
  sb.mac_out[0] = a.mac_out;
  sb.part_hist[0] = a.part_hist;
  sb.n_pkts[0] = a.n_pkts;
  sb.unit_base[0] = 0;
  sb.unit_base[1] = (((a.n_pkts + 63u) >> 6) + kStreamW - 1) / kStreamW;
  sb.n = 1;
  return launch_classify_stream_multi(a, sb, grid, stream);
}

int launch_classify(const ClassifyArgs& a, bool wide_lut, bool lds_lut, int grid, void* stream) {
  const bool hist = a.part_hist != nullptr;
  const size_t lds = classify_lds(a.nb, lds_lut ? a.lut_lds_bytes : 0, hist);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (lds_lut)
    return wide_lut ? launch_mode<kLdsU16>(a, hist, grid, lds, s) : launch_mode<kLdsU8>(a, hist, grid, lds, s);
  return wide_lut ? launch_mode<kGlobalU16>(a, hist, grid, lds, s) : launch_mode<kGlobalU8>(a, hist, grid, lds, s);
}

__global__ __launch_bounds__(kBlock) void lpm_lookup_kernel(const uint16_t* __restrict__ tbl24,
                                                            const uint16_t* __restrict__ tbl_long,
                                                            const uint32_t* __restrict__ ips, uint32_t n,
                                                            uint16_t* __restrict__ gate) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i < n) gate[i] = static_cast<uint16_t>(lpm_lookup(tbl24, tbl_long, ips[i]));
}

int launch_lpm_lookup(const uint16_t* tbl24, const uint16_t* tbl_long, const uint32_t* ips, uint64_t n,
                      uint16_t* gate, void* stream) {
  const uint32_t grid = static_cast<uint32_t>((n + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(lpm_lookup_kernel, dim3(grid), dim3(kBlock), 0, static_cast<hipStream_t>(stream), tbl24,
                     tbl_long, ips, static_cast<uint32_t>(n), gate);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(NBG_EIO, "lpm lookup launch: %s", hipGetErrorString(e));
  return NBG_OK;
}

int launch_hist(const HistArgs& a, void* stream) {
  const size_t lds = static_cast<size_t>(a.nb + 1) * 4;
  if (lds > 64 * 1024) {  // many backends: up to 32768 bins (128 KiB)
    static bool attr = false;
    if (!attr) {
      if (hipFuncSetAttribute(reinterpret_cast<const void*>(hist_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024) != hipSuccess)
        return set_error(NBG_EIO, "hist: LDS attribute: %s", hipGetErrorString(hipGetLastError()));
      attr = true;
    }
  }
  HistMulti hm{};
  hm.h[0] = a;
  hm.per = a.n_parts;
  hipLaunchKernelGGL(hist_kernel, dim3(a.n_parts), dim3(kGBlock), lds, static_cast<hipStream_t>(stream), hm);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(NBG_EIO, "hist launch: %s", hipGetErrorString(e));
  return NBG_OK;
}

int launch_hist_multi(const HistMulti& hm, uint32_t n, void* stream) {
  if (n == 0 || n > kMaxMulti) return set_error(NBG_EINVAL, "hist (multi): %u batches", n);
  if ((hm.h[0].nb + 1) * 4 > 64 * 1024) return set_error(NBG_EINVAL, "hist (multi): at most 16383 bins");
  hipLaunchKernelGGL(hist_kernel, dim3(hm.per * n), dim3(kGBlock), (hm.h[0].nb + 1) * 4,
                     static_cast<hipStream_t>(stream), hm);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(NBG_EIO, "hist launch (multi): %s", hipGetErrorString(e));
  return NBG_OK;
}

__global__ __launch_bounds__(kBlock) void zero_kernel(uint32_t* p, uint32_t words) {
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < words; i += gridDim.x * kBlock) p[i] = 0;
}

int launch_zero(uint32_t* p, size_t words, void* stream) {
  if (words == 0) return NBG_OK;
  const uint32_t grid = static_cast<uint32_t>(std::min<size_t>((words + kBlock - 1) / kBlock, 1024));
  hipLaunchKernelGGL(zero_kernel, dim3(grid), dim3(kBlock), 0, static_cast<hipStream_t>(stream), p,
                     static_cast<uint32_t>(words));
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(NBG_EIO, "zero launch: %s", hipGetErrorString(e));
  return NBG_OK;
}

int launch_scan_multi(const ScanMulti& sm, uint32_t n, void* stream) {
  if (n == 0 || n > kMaxMulti) return set_error(NBG_EINVAL, "scan (multi): %u batches", n);
  hipLaunchKernelGGL(scan_kernel, dim3((sm.s[0].nbins + kScanBins - 1) / kScanBins, n), dim3(kScanWaves * 64), 0,
                     static_cast<hipStream_t>(stream), sm);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(NBG_EIO, "scan launch: %s", hipGetErrorString(e));
  return NBG_OK;
}

int launch_scan(const ScanArgs& a, void* stream) {
  ScanMulti sm{};
  sm.s[0] = a;
  return launch_scan_multi(sm, 1, stream);
}

uint32_t classify_block_pkts() { return kBlock; }  // per tile per wave (64 packets x 4 waves)

template <int LUTM, bool F4, bool HIST>
int launch_desc_multi_v(const ClassifyArgs& a, const DescBatches& db, size_t lds, hipStream_t s) {
  auto fn = a.tbl24 ? classify_desc_multi_kernel<LUTM, F4, HIST, true> : classify_desc_multi_kernel<LUTM, F4, HIST, false>;
  hipLaunchKernelGGL(fn, dim3(db.blk_base[db.n]), dim3(kBlock), lds, s, a, db);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(NBG_EIO, "classify launch (descriptor multi): %s", hipGetErrorString(e));
  return NBG_OK;
}

int launch_classify_desc_multi(const ClassifyArgs& a, const DescBatches& db, bool wide_lut, void* stream) {
  if (db.n == 0 || db.n > kMaxMulti || (a.tiles_per_wave != 1u && a.tiles_per_wave != 2u && a.tiles_per_wave != 4u))
    return set_error(NBG_EINVAL, "classify (descriptor multi): %u batches, %u tiles per wave", db.n, a.tiles_per_wave);
  if (db.blk_base[db.n] == 0) return NBG_OK;
  const bool hist = db.part_hist[0] != nullptr;
  const size_t lds = classify_lds(a.nb, 0, hist);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (wide_lut) {
    if (a.m == 65537u)
      return hist ? launch_desc_multi_v<kGlobalU16, true, true>(a, db, lds, s) : launch_desc_multi_v<kGlobalU16, true, false>(a, db, lds, s);
    return hist ? launch_desc_multi_v<kGlobalU16, false, true>(a, db, lds, s) : launch_desc_multi_v<kGlobalU16, false, false>(a, db, lds, s);
  }
  if (a.m == 65537u)
    return hist ? launch_desc_multi_v<kGlobalU8, true, true>(a, db, lds, s) : launch_desc_multi_v<kGlobalU8, true, false>(a, db, lds, s);
  return hist ? launch_desc_multi_v<kGlobalU8, false, true>(a, db, lds, s) : launch_desc_multi_v<kGlobalU8, false, false>(a, db, lds, s);
}

int launch_classify_idx(const ClassifyArgs& a, int grid, void* stream) {
  const size_t lds = classify_lds(a.nb, 0);
  hipStream_t s = static_cast<hipStream_t>(stream);
  auto fn = a.off ? classify_kernel<kIdx, false, false, false, kDesc>
                  : (a.lean ? classify_kernel<kIdx, false, false, false, kLean>
                            : classify_kernel<kIdx, false, false, false, kFixed>);
  hipLaunchKernelGGL(fn, dim3(grid), dim3(kBlock), lds, s, a);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(NBG_EIO, "classify (index) launch: %s", hipGetErrorString(e));
  return NBG_OK;
}

int launch_tiled_lookup(const TileArgs& a, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(tile_bucket_kernel, dim3((a.n_pkts + kBucketPkts - 1) / kBucketPkts), dim3(kBucketNT),
                     a.n_tiles * 4, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(NBG_EIO, "tile bucket launch: %s", hipGetErrorString(e));
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(tile_lookup_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            kTileEntries * 2) != hipSuccess)
      return set_error(NBG_EIO, "tile lookup: LDS attribute: %s", hipGetErrorString(hipGetLastError()));
    attr = true;
  }
  hipLaunchKernelGGL(tile_lookup_kernel, dim3((a.n_pkts + kLookupChunk - 1) / kLookupChunk, a.n_tiles),
                     dim3(kLookupNT), kTileEntries * 2, s, a);
  e = hipGetLastError();
  if (e != hipSuccess) return set_error(NBG_EIO, "tile lookup launch: %s", hipGetErrorString(e));
  return NBG_OK;
}

uint32_t lut_tiles(uint64_t m) { return static_cast<uint32_t>((m + kTileEntries - 1) / kTileEntries); }

// counters [kSmallW][nbp], rank16 / bin16 [kSmallMax], then a 3-KB load transpose area per wave
size_t small_lds(uint32_t nb, uint32_t waves) {
  return (kSmallW * (((nb + 1) + 3) & ~3u)) * 4u + kSmallMax * 4u + waves * 192u * 16u;
}

int launch_small(const ClassifyArgs& a, const GroupArgs& g, bool wide_lut, void* stream, uint32_t* done,
                 uint32_t done_val) {
  using Fn = void (*)(ClassifyArgs, GroupArgs, uint32_t*, uint32_t);
  static const Fn kFns[16] = {
      small_kernel<kGlobalU8, false, 7, false>,  small_kernel<kGlobalU16, false, 7, false>,
      small_kernel<kGlobalU8, true, 7, false>,   small_kernel<kGlobalU16, true, 7, false>,
      small_kernel<kGlobalU8, false, 10, false>, small_kernel<kGlobalU16, false, 10, false>,
      small_kernel<kGlobalU8, true, 10, false>,  small_kernel<kGlobalU16, true, 10, false>,
      small_kernel<kGlobalU8, false, 7, true>,   small_kernel<kGlobalU16, false, 7, true>,
      small_kernel<kGlobalU8, true, 7, true>,    small_kernel<kGlobalU16, true, 7, true>,
      small_kernel<kGlobalU8, false, 10, true>,  small_kernel<kGlobalU16, false, 10, true>,
      small_kernel<kGlobalU8, true, 10, true>,   small_kernel<kGlobalU16, true, 10, true>};
  const Fn fn = kFns[small_variant(wide_lut, a.m, a.nb, a.win32 != 0)];
  const uint32_t waves = (a.n_pkts + 255u) / 256u;  // 1..16: a wave per 256 packets
  const size_t lds = small_lds(a.nb, waves);
  if (lds > 64 * 1024 &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                          static_cast<int>(lds)) != hipSuccess)
    return set_error(NBG_EIO, "small: LDS attribute: %s", hipGetErrorString(hipGetLastError()));
  hipLaunchKernelGGL(fn, dim3(1), dim3(64 * waves), lds, static_cast<hipStream_t>(stream), a, g, done, done_val);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(NBG_EIO, "small launch: %s", hipGetErrorString(e));
  return NBG_OK;
}

uint32_t small_max() { return kSmallMax; }

// host_ring_kernel's dispatch over the small kernel's instantiations (as launch_small picks them)
uint32_t small_variant(bool wide_lut, uint32_t m, uint32_t nb, bool win32) {
  return (wide_lut ? 1u : 0u) | (m == 65537u ? 2u : 0u) | (nb + 1 > 128 ? 4u : 0u) | (win32 ? 8u : 0u);
}

int launch_host_ring(const HostRingArgs& r, uint32_t blocks, void* stream) {
  const size_t lds = small_lds(kMaxGroupBins - 1, kSmallW);  // any handle's batch: up to 1023 backends
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(host_ring_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                          static_cast<int>(lds)) != hipSuccess)
    return set_error(NBG_EIO, "host ring: LDS attribute: %s", hipGetErrorString(hipGetLastError()));
  hipLaunchKernelGGL(host_ring_kernel, dim3(blocks), dim3(kSmallNT), lds, static_cast<hipStream_t>(stream), r);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(NBG_EIO, "host ring launch: %s", hipGetErrorString(e));
  return NBG_OK;
}

int launch_group_wide(const GroupArgs& a, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(bin_base_kernel, dim3(1), dim3(kGBlock), 0, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(NBG_EIO, "bin_base launch: %s", hipGetErrorString(e));
  const size_t lds = static_cast<size_t>(a.nb + 1) * 4;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(group_wide_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
      return set_error(NBG_EIO, "group_wide: LDS attribute: %s", hipGetErrorString(hipGetLastError()));
    attr = true;
  }
  hipLaunchKernelGGL(group_wide_kernel, dim3(a.n_parts), dim3(64), lds, s, a);
  e = hipGetLastError();
  if (e != hipSuccess) return set_error(NBG_EIO, "group_wide launch: %s", hipGetErrorString(e));
  return NBG_OK;
}

// group_kernel: base[nbp] + tot[nbp] u32, cnt[waves][cst] u16, sslot[kChunk] u32 (40 KB at 1001 bins),
// and <= 128 bins peer[waves][nbins + 1] u64 (22 KB at 66 bins);
// compact (group_direct_kernel): run[2][nbp] + tot[nbp] u32, cnt[waves][cst] u16 (28 KB at 1001 bins)
size_t group_lds(uint32_t nbins, bool compact) {
  const size_t nbp = (nbins + 3) & ~3u, cst = (nbins + 8) & ~7u;
  if (compact) return (nbp * 3 + cst * (kGBlock / 64) / 2) * 4;
  const size_t peer = nbins <= 128 ? (kGBlock / 64) * (nbins + 1) * 8 : 0;
  return (nbp * 2 + kChunk + cst * (kGBlock / 64) / 2) * 4 + peer;
}

// What an in-place persistent ring leaves of a CU's LDS for one co-resident group block: 160 KiB less
// the ring block's LDS, rounded up to the allocation granule (one ring block per CU; the grouping's
// hist and group kernels run in stream order, so one group block is what must fit beside it).
constexpr size_t kLdsGranule = 512u;
size_t group_lds_beside_ring() {
  const size_t ring = (ring_lds(1) + kLdsGranule - 1) / kLdsGranule * kLdsGranule;
  return 160u * 1024u - ring;
}

// The grouping beside a running ring takes the compact kernel when the default one's block would not
// fit in what the ring leaves.  The compact block fits for every bin count the group kernels take
// (<= 1024 bins: group_lds(1024, true) = 28,800 B, checked by tests/test_cpu_wrapper.py through
// nbg_debug_group_lds); a block that did not would simply wait for the ring to end (stop or idle
// exit), never deadlock: the ring completes its batches without the grouping.
// g_group_compact: -1 = that rule, 0 / 1 = forced (tests and measurements: nbg_debug_set_group_compact,
// or NBG_GROUP_COMPACT read once at the first grouping).
std::atomic<int> g_group_compact{-2};
bool group_compact(uint32_t nbins, bool ring_running) {
  int f = g_group_compact.load(std::memory_order_relaxed);
  if (f == -2) {
    const char* e = std::getenv("NBG_GROUP_COMPACT");
    int v = e ? (std::atoi(e) != 0) : -1;
    g_group_compact.compare_exchange_strong(f, v);
    f = g_group_compact.load(std::memory_order_relaxed);
  }
  if (f >= 0) return f != 0;
  return ring_running && group_lds(nbins, false) > group_lds_beside_ring();
}

// Default: sum the partition histograms from L2 inside the group kernel while the rows are
// small (every block reads all of them), else a separate scan kernel.  NBG_GSCAN=0/2 forces a mode
// (measurements).
// Partition histograms from the classify kernel's per-block flush for few bins, from hist_kernel
// for many (NBG_HIST_KERNEL_BINS overrides the threshold, for measurements).
bool hist_in_classify(uint32_t nbins) {
  static const uint32_t limit = [] {
    const char* e = std::getenv("NBG_HIST_KERNEL_BINS");
    return e ? static_cast<uint32_t>(std::atoi(e)) : 257u;
  }();
  return nbins < limit;
}

int pick_group_scan(uint32_t nbins, uint32_t n_parts) {
  static const int forced = [] {
    const char* e = std::getenv("NBG_GSCAN");
    return e ? std::atoi(e) : -1;
  }();
  if (forced == kScanKernel || forced == kScanDirect) return forced;
  return static_cast<size_t>(nbins) * n_parts <= 32u * 1024u ? kScanDirect : kScanKernel;
}

auto group_fn(uint32_t bits, int scan, bool compact) {
  if (compact)
    return bits <= 7 ? (scan == kScanDirect ? group_direct_kernel<kScanDirect, 7> : group_direct_kernel<kScanKernel, 7>)
                     : (scan == kScanDirect ? group_direct_kernel<kScanDirect, 10> : group_direct_kernel<kScanKernel, 10>);
  return bits <= 7 ? (scan == kScanDirect ? group_kernel<kScanDirect, 7> : group_kernel<kScanKernel, 7>)
                   : (scan == kScanDirect ? group_kernel<kScanDirect, 10> : group_kernel<kScanKernel, 10>);
}

int launch_group(const GroupArgs& a, int scan, void* stream, bool compact) {
  GroupMulti gm{};
  gm.g[0] = a;
  gm.per = a.n_parts;
  hipLaunchKernelGGL(group_fn(a.bits, scan, compact), dim3(a.n_parts), dim3(kGBlock), group_lds(a.nb + 1, compact),
                     static_cast<hipStream_t>(stream), gm);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(NBG_EIO, "group launch: %s", hipGetErrorString(e));
  return NBG_OK;
}

int launch_group_multi(const GroupMulti& gm, uint32_t n, int scan, void* stream, bool compact) {
  const GroupArgs& a = gm.g[0];
  if (n == 0 || n > kMaxMulti) return set_error(NBG_EINVAL, "group (multi): %u batches", n);
  hipLaunchKernelGGL(group_fn(a.bits, scan, compact), dim3(gm.per * n), dim3(kGBlock), group_lds(a.nb + 1, compact),
                     static_cast<hipStream_t>(stream), gm);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(NBG_EIO, "group launch (multi): %s", hipGetErrorString(e));
  return NBG_OK;
}

// Grid for the classify kernel: resident blocks (CUs x blocks/CU by LDS), so that the
// LDS-staged LUT is loaded once per resident block and amortised over its tiles.
int classify_grid(bool lds_lut, uint32_t lut_bytes, uint32_t nb, int device, int* grid) {
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0)
    return set_error(NBG_ENODEV, "hipDeviceGetAttribute(CU count) failed");
  const size_t lds = classify_lds(nb, lds_lut ? lut_bytes : 0);
  int per_cu = static_cast<int>((160 * 1024) / lds);
  per_cu = per_cu < 1 ? 1 : (per_cu > 8 ? 8 : per_cu);
  *grid = cus * per_cu;
  return NBG_OK;
}

}  // namespace nbg

// Diagnostics (not in include/nbgpu.h; tests only): `blocks` one-wave workgroups that each hold
// `lds_bytes` of a CU's LDS for `us` microseconds (100 MHz wall clock; every wave exits by time) —
// other work occupying CUs when a persistent ring starts (tests/test_gpu_ring.py).
namespace nbg {
__global__ __launch_bounds__(64) void hold_cus_kernel(uint64_t ticks, uint32_t* sink) {
  extern __shared__ uint32_t held[];
  const uint64_t t0 = wall_clock64();
  held[threadIdx.x] = threadIdx.x;
  while (static_cast<uint64_t>(wall_clock64()) - t0 < ticks) __builtin_amdgcn_s_sleep(16);
  if (held[threadIdx.x] == 0xdeadbeefu) sink[0] = 1u;
}
}  // namespace nbg

extern "C" int nbg_debug_hold_cus(uint32_t blocks, uint32_t lds_bytes, uint32_t us, void* stream) {
  if (blocks == 0 || blocks > 4096 || lds_bytes < 256 || lds_bytes > 160u * 1024u || us > 10000000u) return NBG_EINVAL;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(nbg::hold_cus_kernel),
                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
    return NBG_EIO;
  hipLaunchKernelGGL(nbg::hold_cus_kernel, dim3(blocks), dim3(64), lds_bytes, static_cast<hipStream_t>(stream),
                     static_cast<uint64_t>(us) * 100u, static_cast<uint32_t*>(nullptr));
  return hipGetLastError() == hipSuccess ? NBG_OK : NBG_EIO;
}

// Diagnostics (not in include/nbgpu.h; tests only, no GPU needed): force the compact group kernel
// (mode 1), the default one (0) or the library's rule (-1); and the LDS sizes the rule compares.
extern "C" int nbg_debug_set_group_compact(int mode) {
  if (mode < -1 || mode > 1) return NBG_EINVAL;
  nbg::g_group_compact.store(mode);
  return NBG_OK;
}
extern "C" uint64_t nbg_debug_group_lds(uint32_t nbins, int compact) { return nbg::group_lds(nbins, compact != 0); }
extern "C" uint64_t nbg_debug_lds_beside_ring(void) { return nbg::group_lds_beside_ring(); }
