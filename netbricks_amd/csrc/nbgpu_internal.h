// Internal declarations shared by the nbgpu translation units.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

#include "../../include/nbgpu.h"

namespace nbg {

// Thread-local last-error string (nbg_last_error); returns `code` for chaining.
int set_error(int code, const char* fmt, ...);

uint64_t fnv1a64(const uint8_t* p, size_t n);
uint64_t xxh64(const uint8_t* p, size_t n, uint64_t seed);
int build_lut(const char* const* names, const uint32_t* lens, uint32_t n, uint64_t m, std::vector<uint32_t>& entry);
int build_lpm(const uint32_t* prefixes, const uint8_t* lens, const uint16_t* gates, uint64_t n,
              std::vector<uint16_t>& tbl24, std::vector<uint16_t>& tbl_long, uint64_t& long_used);

// Kernel geometry.
constexpr int kBlock = 256;          // classify threads per workgroup (4 waves), L2-gather LUT
constexpr int kLdsBlock = 1024;      // classify threads per workgroup with the LDS-staged LUT (1 per CU)
constexpr int kXStride = 48;         // LDS bytes per packet in the transpose: chunks 0..2 (a 12-dword row
                                     // stride keeps the b128 reads conflict-free; 8 blocks fit per CU)
constexpr int kLoadPrio = 3;         // s_setprio while a classify wave issues its tile loads
constexpr int kGBlock = 512;         // group kernel threads per workgroup (8 waves: overlaps classify better)
constexpr int kChunk = 4096;         // packets per group-kernel chunk
constexpr int kGRounds = kChunk / kGBlock;  // group kernel rounds of 64 packets per wave per chunk
constexpr uint32_t kMaxParts = 256;  // partitions per batch (part_pkts is a multiple of kChunk)
constexpr uint32_t kMaxGroupBins = 1024;  // multisplit group kernel: n_backends + 1 <= 1024
constexpr uint32_t kMaxWideBins = 32768;  // wide grouping path: n_backends <= 32767 (LUT sentinel bound,
                                          // test/maglev/src/nf.rs:46)

struct ClassifyArgs {
  uint8_t* pkts;
  const uint32_t* off;      // nullable
  const uint16_t* len;      // nullable
  uint32_t stride;
  uint32_t fixed_len;
  uint32_t n_pkts;
  uint32_t tiles_per_wave;  // consecutive 64-packet tiles per wave (power of 2, <= 64)
  const void* lut;          // u8 or u16 entries
  uint32_t m;               // table size
  uint32_t lut_lds_bytes;   // bytes of LUT staged in LDS (0 = global gather)
  uint32_t lut_tail;        // streaming kernel: entry 65536 of a 65537-slot u8 LUT (LDS holds 0..65535)
  uint64_t mu;              // floor(2^64 / m) for Barrett
  uint32_t nb;              // backends; bins = nb + 1 (sentinel bin = nb)
  uint32_t swap;
  uint32_t win_owned;       // every packet start owns 64 readable/writable bytes
  uint32_t wb_full;         // write back the whole owned window (full lines) instead of 16 B
  uint32_t lean;            // fixed slots, 16-B aligned, owned windows, no len[], fixed_len >= 48
  uint16_t* backend;
  uint8_t* mac_out;         // nullable: dense 12-B swapped-MAC records instead of in-place swap
  uint32_t* part_hist;      // nullable: [n_parts][nb+1] partition histograms (pre-zeroed)
  uint32_t part_pkts;       // packets per partition
  uint32_t hist16;          // part_hist rows hold two 16-bit bins per word (partitions < 65536 packets)
  // chained test/lpm stage (nbg_chain_lpm_maglev_device); tbl24 == nullptr: Maglev alone
  const uint16_t* tbl24;
  const uint16_t* tbl_long;
  uint32_t lpm_groups;
  uint16_t* gate;
  uint32_t* idx_out;        // NBG_LUT_TILED: per-packet LUT index (0xffffffff = would panic)
  uint8_t* sink;            // descriptor streaming kernel: 1 KiB scratch for stores of lanes with none
  uint32_t win32;           // small kernel: window i (pkts + i * stride) holds frame bytes 8..39 (the host
                            // path's 32-B staging; no MAC swap on the GPU)
};

// Several batches in one streaming-classify launch (nbg_maglev_classify_device_multi): what differs
// per batch.  A single-batch launch passes n = 1.  Units (512 packets) never straddle batches.
constexpr uint32_t kMaxMulti = 16;
struct StreamBatches {
  uint8_t* pkts[kMaxMulti];
  uint16_t* backend[kMaxMulti];
  uint8_t* mac_out[kMaxMulti];
  uint32_t* part_hist[kMaxMulti];
  uint32_t n_pkts[kMaxMulti];
  uint32_t unit_base[kMaxMulti + 1];  // first unit of batch j; unit_base[n] = all units
  uint32_t n;
};

// NBG_GROUP_LAG: the handle's pending batch (classified by the previous launch) whose grouping rides
// on this streaming-classify launch.  Block c groups partition c (n_parts <= grid), in 512-packet
// pieces between its classify units.  n_parts == 0: nothing pending (the launch only zeroes).
struct LagGroup {
  const uint16_t* backend;    // the pending batch's backend[]
  uint32_t* perm;             // nullable: counts only
  uint32_t* counts;
  const uint32_t* part_hist;  // its partition rows (written by the previous launch)
  uint32_t* zero;             // nullable: the lag histogram buffer the launch after next accumulates into
  uint32_t zero_words;
  uint32_t n_pkts;
  uint32_t part_pkts;
  uint32_t n_parts;
  uint32_t hist16;            // rows of two 16-bit bins per word
};

// Persistent RX-ring classify (nbg_ring_*).  One batch per ring slot (64 B, one line), written by
// nbg_ring_post into pinned host memory.  No classify CU ever touches host memory: a one-wave relay
// (the ring kernel's last block, on a CU of its own: ring_relay) copies each posted descriptor into a device ring in
// uncached HBM (`reps` replicas, block b reads replica b % reps), forwards the host's stop, and
// reports the minimum of the blocks' per-block completion counts (also uncached HBM) to the host.
// Measured before the relay: with every classify block reading host memory, the per-batch time
// varied from 12 to 190 us from run to run and box to box (a PCIe read in a CU's vector memory path
// holds that CU's tile loads behind it).
struct RingDesc {
  uint64_t pkts;
  uint64_t backend;
  uint64_t ulo, uhi;  // the batch's units [ulo, uhi) in the ring's unit sequence (512 packets each)
  uint32_t n_pkts;
  uint32_t seq;       // batch index + 1 (mod 2^32)
  uint32_t pad[4];
  uint64_t check;     // ring_check(): a read that overlaps a rewrite of the slot fails it
};
static_assert(sizeof(RingDesc) == 64, "one descriptor per 64-B line");
struct RingCtl {      // pinned host memory, the first line
  uint32_t stop;      // host: exit once everything posted is classified
  uint32_t error;     // device: 1 = idle timeout (the kernels exited by themselves)
  uint32_t completed; // relay: batches complete on every block (mod 2^32)
  uint32_t pad[13];
};
struct RingArgs {
  RingCtl* ctl;           // host
  const RingDesc* hdesc;  // host [slots]: read by the relay only
  RingDesc* desc;         // device, uncached [reps][slots]: the classify blocks' descriptors
  uint32_t* dstop;        // device, uncached: relay -> blocks, every posted batch is relayed and stop was asked
  uint32_t* dcomp;        // device, uncached: relay, batches complete on every block (the gate kernels poll it)
  uint32_t* dexit;        // device, uncached: classify blocks that have exited (their stores retired)
  uint32_t* prog;         // device, uncached [grid]: per block, batches all of whose units of it are complete
  uint32_t slots;         // power of two
  uint32_t reps;          // power of two: replicas of the device ring
  uint32_t grid;          // classify blocks (block `grid` is the relay)
  uint64_t idle_ticks;    // exit after this long (100 MHz wall clock) without a new batch
};
#ifdef __HIPCC__
#define NBG_HD __host__ __device__
#else
#define NBG_HD
#endif
constexpr uint32_t kRingReps = 8;  // device-ring replicas, one per XCD (NBG_RING_REPS overrides: measurement)
NBG_HD inline uint64_t ring_check(uint64_t pkts, uint64_t backend, uint64_t ulo, uint64_t uhi, uint32_t n_pkts,
                                  uint32_t seq) {
  uint64_t h = 0x6a09e667f3bcc909ull ^ (static_cast<uint64_t>(seq) << 32 | n_pkts);
  const uint64_t w[4] = {pkts, backend, ulo, uhi};
  for (int i = 0; i < 4; ++i) {
    h ^= w[i] + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 33;
  }
  return h;
}

// NBG_LUT_TILED: bucket packets by 64-KiB LUT tile, then look them up per tile in LDS.
struct TileArgs {
  const uint32_t* idx;      // [n_pkts] from the classify kernel (kIdx)
  uint32_t n_pkts;
  uint32_t n_tiles;
  uint32_t m;               // LUT entries
  const void* lut;          // u16 entries (padded to whole 16-B vectors)
  uint32_t* cursor;         // [n_tiles] bucket fill counts (zeroed before the bucket kernel)
  uint64_t* bucket;         // [n_tiles][bucket_cap] (packet << 32 | index in tile)
  uint32_t bucket_cap;
  uint16_t* backend;
};

struct HistArgs {
  const uint16_t* backend;
  uint32_t n_pkts;
  uint32_t nb;
  uint32_t part_pkts;
  uint32_t n_parts;
  uint32_t* part_hist;      // [n_parts][nb+1] (hist16: [n_parts][(nb+2)/2]), every entry stored
  uint32_t hist16;          // rows of two 16-bit bins per word (partitions < 65536 packets; for the
                            // group kernel's direct prefix, not for scan_kernel)
};

// hist_kernel over several batches: blocks [j * per, j * per + h[j].n_parts) count batch j.
struct HistMulti {
  HistArgs h[kMaxMulti];
  uint32_t per;
};

struct ScanArgs {
  const uint32_t* part_hist;  // [n_parts][nbins]
  uint32_t* part_prefix;      // [n_parts][nbins] exclusive prefix over earlier partitions
  uint32_t* totals;           // [nbins]
  uint32_t n_parts;
  uint32_t nbins;
};

// scan_kernel over several batches: blockIdx.y = batch
struct ScanMulti {
  ScanArgs s[kMaxMulti];
};

// Several descriptor-layout batches (IMIX: u32 offset + u16 length per packet) in one launch of the
// tile-per-wave classify kernel (nbg_maglev_classify_desc_multi / nbg_chain_lpm_maglev_multi): what
// differs per batch.  Blocks [blk_base[j], blk_base[j + 1]) classify batch j (tiles never straddle).
struct DescBatches {
  uint8_t* pkts[kMaxMulti];
  const uint32_t* off[kMaxMulti];
  const uint16_t* len[kMaxMulti];
  uint16_t* backend[kMaxMulti];
  uint16_t* gate[kMaxMulti];        // chain only
  uint32_t* part_hist[kMaxMulti];   // nullable: partition rows written by the classify kernel
  uint32_t n_pkts[kMaxMulti];
  uint32_t blk_base[kMaxMulti + 1];
  uint32_t n;
};

struct GroupArgs {
  const uint16_t* backend;
  uint32_t n_pkts;
  uint32_t nb;
  uint32_t bits;              // ceil(log2(nb+1))
  uint32_t n_parts;
  uint32_t part_pkts;
  const uint32_t* part_hist;  // [n_parts][nb+1]      (kScanDirect)
  const uint32_t* part_prefix;// [n_parts][nb+1]      (scan_kernel path)
  const uint32_t* totals;     // [nb+1]               (scan_kernel path)
  uint32_t hist16;            // kScanDirect: rows of two 16-bit bins per word ((nbins + 1) / 2 words)
  uint32_t* part_hist_next;   // zeroed for the next call
  uint32_t next_words;
  uint32_t* counts;           // nullable
  uint32_t* perm;             // nullable (counts only)
  uint32_t* bin_base;         // [nb+1] wide path: first perm slot of every group
};

// The group kernel over several batches: blocks [j * per, j * per + g[j].n_parts) group batch j.
// Every g[j] names the same part_hist_next / next_words (zeroed by the whole grid).
struct GroupMulti {
  GroupArgs g[kMaxMulti];
  uint32_t per;
};

// How the group kernel gets each partition's per-bin prefix: from scan_kernel's output, or by
// summing the partition histograms straight from L2.
enum GroupScan { kScanKernel = 0, kScanDirect = 2 };

// The host-batch server (nbg_host_ring_*): a persistent kernel whose blocks each take the next posted
// small host batch (the direct path of nbg_maglev_host_submit) from a descriptor ring in pinned host
// memory, so a batch costs no kernel launch.  Descriptors are written by producer threads: the
// arguments the small kernel would have been launched with, then seq = ticket + 1 (release); a block
// copies them, stores ack = ticket + 1 (the slot may be reused), classifies + groups, and sets the
// batch's completion word.
struct HostRingDesc {
  uint32_t seq;       // ticket + 1 once posted
  uint32_t ack;       // ticket + 1 once a block has copied the descriptor
  uint32_t variant;   // small-kernel instantiation: bit 0 u16 LUT, bit 1 M = 65537, bit 2 more than 128 bins
  uint32_t done_val;  // stored into *done when the batch's outputs are visible
  uint32_t* done;     // the batch's completion word (pinned host memory)
  uint64_t pad0;
  ClassifyArgs a;
  GroupArgs g;
};
constexpr uint32_t kHostRingDescBytes = 512;  // one slot (a whole number of lines)
static_assert(sizeof(HostRingDesc) <= kHostRingDescBytes, "host ring slot");
struct HostRingCtl {   // pinned host memory, the first line
  uint32_t stop;       // host: exit once every posted batch is done
  uint32_t ended;      // device: 1 = exited after idle_ticks without a post
  uint32_t posted;     // host: batches posted (mod 2^32), so idle blocks see activity
  uint32_t pad[13];
};
struct HostRingArgs {
  HostRingCtl* ctl;         // host (device address)
  uint8_t* desc;            // host [slots] x kHostRingDescBytes (device address)
  uint32_t* claim;          // device: next ticket to claim
  uint32_t slots;           // power of two
  uint64_t idle_ticks;      // 100 MHz wall clock
};
int launch_host_ring(const HostRingArgs& r, uint32_t blocks, void* stream);
uint32_t small_variant(bool wide_lut, uint32_t m, uint32_t nb, bool win32);


// Launchers (maglev_kernels.hip).  `wide_lut` = u16 entries; `lds_lut` = stage in LDS.
int launch_classify(const ClassifyArgs& a, bool wide_lut, bool lds_lut, int grid, void* stream);
// Streaming classify (lean fixed slots, u8 LUT of <= 65537 entries staged in LDS): one block per
// CU; a.tiles_per_wave = the contiguous 64-packet tiles of each of the grid's waves.
int launch_classify_stream(const ClassifyArgs& a, int grid, void* stream);
// The same over several batches (sb.n >= 1; a carries what they share)
int launch_classify_stream_multi(const ClassifyArgs& a, const StreamBatches& sb, int grid, void* stream);
// One batch (a.part_hist set) plus the grouping of the pending batch lg (NBG_GROUP_LAG); needs
// lg.n_parts <= grid and (nb + 1) * lg.n_parts within the direct-scan limit (pick_group_scan)
int launch_classify_stream_lag(const ClassifyArgs& a, const LagGroup& lg, int grid, void* stream);
size_t stream_lds(uint32_t nb, int mode, bool lag);
// The persistent ring kernel (nbg_ring_start): a.pkts / n_pkts / backend come from the ring; mode 0
// read only, 1 MAC swap in place.  Returns after the launch; the kernel runs until stop or idle.
int launch_classify_ring(const ClassifyArgs& a, const RingArgs& r, int mode, int grid, void* stream);
size_t ring_lds(int mode);
// One wave on `stream` that returns once the ring has completed `target` batches (dcomp, mod 2^32) or
// every one of its `grid` classify blocks has exited (dexit): the stream's later launches (a ring
// batch's grouping) run after the batch is in HBM, with no host round trip.
int launch_ring_gate(const uint32_t* dcomp, const uint32_t* dexit, uint32_t target, uint32_t grid, void* stream);
int stream_waves_per_block();
// Streaming classify for descriptor layouts with owned windows (u8 LUT in LDS, or the u16 LUT
// gathered from L2); stream_desc_lds: its dynamic LDS bytes (mode 0 read only, 1 in place, 2 records).
int launch_classify_stream_desc(const ClassifyArgs& a, bool wide_lut, int grid, void* stream);
size_t stream_desc_lds(uint32_t nb, int mode, bool wide_lut);
int launch_scan(const ScanArgs& a, void* stream);
int launch_scan_multi(const ScanMulti& sm, uint32_t n, void* stream);
// the tile-per-wave classify kernel (256 threads, one 64-packet tile per wave) over db.n descriptor
// batches; a carries what they share (LUT, flags, lpm tables), db what differs
int launch_classify_desc_multi(const ClassifyArgs& a, const DescBatches& db, bool wide_lut, void* stream);
uint32_t classify_block_pkts();  // packets per block and tile per wave of launch_classify_desc_multi
int launch_zero(uint32_t* p, size_t words, void* stream);  // p[0, words) = 0 (one kernel)
int launch_hist(const HistArgs& a, void* stream);
int launch_hist_multi(const HistMulti& hm, uint32_t n, void* stream);  // nb + 1 <= 16384
bool hist_in_classify(uint32_t nbins);
int launch_lpm_lookup(const uint16_t* tbl24, const uint16_t* tbl_long, const uint32_t* ips, uint64_t n,
                      uint16_t* gate, void* stream);
// compact: the LDS-light group kernel (group_compact(): many bins while a persistent ring runs)
int launch_group(const GroupArgs& a, int scan, void* stream, bool compact);
// one launch grouping gm.g[0 .. n): blocks per batch gm.per (the largest n_parts)
int launch_group_multi(const GroupMulti& gm, uint32_t n, int scan, void* stream, bool compact);
bool group_compact(uint32_t nbins, bool ring_running);
int launch_group_wide(const GroupArgs& a, void* stream);  // nb + 1 > kMaxGroupBins
// One launch for a batch of at most small_max() packets and at most kMaxGroupBins bins: classify
// and (when g.perm / g.counts) group.  The batch base must be 16-B aligned.
// done (nullable): completion word the kernel sets to done_val once its outputs are visible to the host
int launch_small(const ClassifyArgs& a, const GroupArgs& g, bool wide_lut, void* stream, uint32_t* done = nullptr,
                 uint32_t done_val = 0);
uint32_t small_max();
int launch_classify_idx(const ClassifyArgs& a, int grid, void* stream);  // kIdx classify (tile per wave)
int launch_tiled_lookup(const TileArgs& a, void* stream);
uint32_t lut_tiles(uint64_t m);
size_t group_lds(uint32_t nbins, bool compact);
int pick_group_scan(uint32_t nbins, uint32_t n_parts);
int classify_grid(bool lds_lut, uint32_t lut_bytes, uint32_t nb, int device, int* grid);

}  // namespace nbg
