// C-ABI of the Maglev flow-steering path (include/nbgpu.h).
//
// Handle lifecycle mirrors the reference's one-time pipeline construction
// (test/maglev/src/nf.rs:84-111: Maglev::new + operator chain) and the per-batch
// producer task (framework/src/operators/group_by.rs:43-55).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <cctype>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "nbgpu_internal.h"

namespace nbg {

namespace {
thread_local char g_err[512] = "";
}

int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

}  // namespace nbg

using namespace nbg;

#define NBG_HIP(call)                                                                      \
  do {                                                                                     \
    hipError_t e_ = (call);                                                                \
    if (e_ != hipSuccess) return set_error(NBG_EIO, "%s: %s", #call, hipGetErrorString(e_)); \
  } while (0)

struct nbg_lpm {
  int device = 0;
  uint16_t* d_tbl24 = nullptr;     // NBG_LPM_TBL24_SIZE entries
  uint16_t* d_tbl_long = nullptr;  // the used 256-entry blocks (at least one entry)
  uint64_t long_used = 0;
};

struct nbg_maglev {
  int device = 0;
  uint32_t nb = 0;
  uint64_t m = 0;
  std::vector<uint16_t> lut_host;
  void* d_lut = nullptr;      // u8 (nb <= 256) or u16 entries, padded to 16 B
  bool wide = false;
  uint32_t lut_bytes = 0;     // LUT bytes (padded to 16 B)
  uint32_t lut_alloc = 0;     // device LUT allocation: lut_bytes rounded up to 1 KiB (LDS-DMA pieces)
  int cus = 0;                // compute units (streaming classify: one block per CU)
  // grouping scratch (independent of the batch size: at most kMaxParts partitions)
  uint32_t* d_part_hist = nullptr;    // [2][kMaxParts][nb+1] ping-pong partition histograms
  uint32_t* d_part_graph = nullptr;   // [kMaxParts][nb+1] histograms of calls captured in a hipGraph
  uint32_t* d_part_prefix = nullptr;  // [kMaxParts][nb+1] (scan-kernel fallback)
  uint32_t* d_totals = nullptr;       // [nb+1]            (scan-kernel fallback)
  uint32_t* d_bin_base = nullptr;     // [nb+1]            (wide grouping path)
  uint8_t* d_sink = nullptr;          // [1 KiB] stores of idle lanes (descriptor streaming kernel)
  uint32_t* d_part_multi = nullptr;   // [2][kMaxMulti][kMaxParts][nb+1] (nbg_maglev_classify_device_multi, on first use)
  uint32_t mparity = 0;
  uint32_t parity = 0;
  uint32_t* d_counts = nullptr;       // used when the caller passes no counts buffer
  // deferred grouping (NBG_DEFER_GROUP): the group kernel's arguments, launched by finish_group
  bool pending = false;
  int pending_scan_mode = 0;
  bool pending_hist = false;
  bool pending_wide = false;
  HistArgs pending_hist_args{};
  GroupArgs pending_args{};
  ScanArgs pending_scan{};
  uint32_t pending_multi = 0;         // > 0: the deferred group is a multi-batch group launch
  GroupMulti pending_gm{};
  bool pending_hist_multi = false;    // ... preceded by a multi-batch hist launch (many backends)
  HistMulti pending_hm{};
  ScanMulti pending_sm{};             // ... and a multi-batch scan launch (pending_scan_mode == kScanKernel)
  uint32_t* d_prefix_multi = nullptr; // [kMaxMulti][kMaxParts][nb+1] prefixes + [kMaxMulti][nb+1] totals (descriptor multi, scan kernel)
  // lagged grouping (NBG_GROUP_LAG): three rotating partition-histogram sets; a lagged classify
  // accumulates into set lag_idx, groups the pending batch from the previous set and zeroes the third
  bool pending_lag = false;           // the pending group is a lagged one (pending_args / pending_lg)
  LagGroup pending_lg{};
  uint32_t* d_part_lag = nullptr;     // [3][kMaxParts][nb+1] (on first use)
  uint32_t lag_idx = 0;
  uint32_t lag_dirty = 0;             // bit k: set k may hold counts (zeroed before it is accumulated into)
  nbg_ring* ring = nullptr;           // the running persistent ring (nbg_ring_start), if any
  nbg_ring* ring_spare = nullptr;     // a stopped ring's buffers and stream, kept for the next start
  std::vector<nbg_ring*> ring_dead;   // rings whose stream failed: kept (callers may hold them) until destroy
  bool ring_leaked = false;           // a ring's kernel did not end at stop: never free what it may touch
  float ring_kernel_ms = -1.f;        // the last ring kernel's duration (HIP events), after its stop
  hipStream_t last_stream = nullptr;  // the stream of the handle's last launch
  bool issued = false;                // a launch has been issued on last_stream
  hipEvent_t order_ev = nullptr;      // cross-stream ordering of consecutive calls (order_after_last)
  int grid_lds = 0, grid_global = 0;
  uint32_t tiles_per_wave = 1;        // L2-LUT classify: 64-packet tiles per wave (NBG_TPW)
  // NBG_LUT_TILED scratch (grown on demand, outside graph capture): per-packet LUT indices, bucket
  // fill counts, and one bucket of (packet, index in tile) per 64-KiB LUT tile
  uint32_t* d_idx = nullptr;
  uint32_t* d_cursor = nullptr;
  uint64_t* d_bucket = nullptr;
  uint64_t tiled_cap = 0;
  // descriptor mode without lengths: a fixed_len-filled u16[] (the kernel reads off[] and len[])
  uint16_t* d_fixed_len = nullptr;
  uint64_t fixed_len_cap = 0;
  uint16_t fixed_len_val = 0;
  // host path (PCIe): NBG_HOST_SLOTS staging slots, one batch in flight per slot
  struct HostSlot {
    uint64_t cap = 0;          // packets the buffers hold
    uint8_t* h_win = nullptr;  // pinned: windows (cap * 80 B + 64 B of slack for the last chunk load)
    uint16_t* h_len = nullptr;
    uint16_t* h_backend = nullptr;
    uint32_t* h_perm = nullptr;
    uint32_t* h_counts = nullptr;
    uint8_t* d_win = nullptr;
    uint16_t* d_len = nullptr;
    uint16_t* d_backend = nullptr;
    uint32_t* d_perm = nullptr;
    uint32_t* d_counts = nullptr;
    // device addresses of the pinned buffers above (mapped, fine-grained): a small batch is classified
    // straight out of h_win / h_len with its results stored straight into h_backend / h_perm /
    // h_counts — one launch, no copy (host_submit's direct path)
    uint8_t* dh_win = nullptr;
    uint16_t* dh_len = nullptr;
    uint16_t* dh_backend = nullptr;
    uint32_t* dh_perm = nullptr;
    uint32_t* dh_counts = nullptr;
    // the direct path's completion word (pinned, fine-grained, its own line): the small kernel stores
    // the batch's ticket there once its outputs are visible; polled with plain loads
    uint32_t* h_flag = nullptr;
    uint32_t* dh_flag = nullptr;
    bool direct = false;        // the slot's batch took the direct path (completion = h_flag)
    uint32_t win = 0;           // the stride its windows were staged at (32: frame bytes 8..39; 0: zero-copy)
    hipStream_t watch = nullptr;  // the direct batch's kernel runs on it (its end without the flag is a failure)
    bool on_ring = false;         // posted to the host-batch server: ra / rg relaunch it if the server ended first
    ClassifyArgs ra{};
    GroupArgs rg{};
    hipEvent_t done = nullptr;  // after the slot's D2H copies (on the handle's host stream)
    bool busy = false;
    uint64_t ticket = 0;
    // the submitted batch's outputs (the caller keeps them valid until its wait)
    uint64_t n = 0;
    uint16_t* backend_out = nullptr;
    uint32_t* perm_out = nullptr;
    uint32_t* counts_out = nullptr;
  };
  HostSlot slots[NBG_HOST_SLOTS];
  hipStream_t host_compute = nullptr;  // the classify and group kernels of every slot, in submit order
  uint64_t next_ticket = 1;
  nbg_host_ring* hring = nullptr;      // direct batches go to this host-batch server instead of a launch
};

// The host-batch server of one device (nbg_host_ring_start): a persistent kernel fed descriptors.
struct nbg_host_ring {
  int device = 0;
  uint32_t blocks = 0, slots = 0, idle_ms = 0;
  hipStream_t stream = nullptr;     // private, highest priority (a hardware queue no ordinary stream shares)
  uint8_t* host = nullptr;          // pinned, mapped, fine-grained: HostRingCtl | slots x kHostRingDescBytes
  HostRingCtl* ctl = nullptr;
  uint8_t* desc = nullptr;
  uint32_t* claim = nullptr;        // device
  std::atomic<uint64_t> next{0};    // tickets handed out (producer threads post concurrently)
  std::atomic<uint32_t> attached{0};
  std::atomic<bool> stopping{false};
  bool leaked = false;
};

namespace {

// Host regions registered with nbg_host_register: host_submit batches whose frames all lie in one
// of them take the zero-copy path (the GPU reads and rewrites the frames over PCIe).
struct HostRegionRec {
  uintptr_t base;
  uint64_t bytes;
  uint8_t* dev;
  int device;
};
std::mutex g_regions_mu;
std::vector<HostRegionRec> g_regions;

bool find_region(const void* p, int device, HostRegionRec* out) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  std::lock_guard<std::mutex> g(g_regions_mu);
  for (const auto& r : g_regions)
    if (r.device == device && a >= r.base && a - r.base < r.bytes) {
      *out = r;
      return true;
    }
  return false;
}

// NBG_OK, or NBG_ENODEV with the reason (no device: the path has no CPU fallback).
int check_device(int device) {
  int ndev = 0;
  const hipError_t ce = hipGetDeviceCount(&ndev);
  if (ce != hipSuccess || ndev <= 0)
    return set_error(NBG_ENODEV, "no HIP device available (no CPU fallback): %s, %d devices", hipGetErrorString(ce),
                     ndev);
  if (device < 0 || device >= ndev) return set_error(NBG_ENODEV, "device %d out of range (%d devices)", device, ndev);
  return NBG_OK;
}

// The running persistent ring of each device (one per GPU: its kernel holds every CU's LDS).
std::mutex g_dev_ring_mu;
std::vector<nbg_ring*> g_dev_ring;
std::vector<nbg_host_ring*> g_dev_hring;  // host-batch servers (nbg_host_ring_start), under g_dev_ring_mu
// a stopped server's private stream, kept for the device's next server: a batch's completion wait may
// still query it after the stop (never a destroyed stream)
std::vector<hipStream_t> g_hring_stream;

bool device_ring_running(int device) {
  std::lock_guard<std::mutex> g(g_dev_ring_mu);
  return device >= 0 && static_cast<size_t>(device) < g_dev_ring.size() && g_dev_ring[device] != nullptr;
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// Setup copies and zeroing (handle creation, buffer growth) on a private non-blocking stream that
// is synchronised before the call returns.  Never the legacy null stream: hipMemset there returns
// before it runs and is not ordered with non-blocking streams (tools/memset_probe.py: 6 of 6 trials
// with a busy null stream zeroed data a later copy on a non-blocking stream had written), which is
// what let round-1 host-path kernels read zeroed staging windows.
struct SetupStream {
  hipStream_t s = nullptr;
  hipError_t err = hipSuccess;
  SetupStream() { err = hipStreamCreateWithFlags(&s, hipStreamNonBlocking); }
  ~SetupStream() {
    if (s) (void)hipStreamDestroy(s);
  }
  hipError_t zero(void* p, size_t bytes) { return err ? err : (err = hipMemsetAsync(p, 0, bytes, s)); }
  hipError_t h2d(void* d, const void* hsrc, size_t bytes) {
    return err ? err : (err = hipMemcpyAsync(d, hsrc, bytes, hipMemcpyHostToDevice, s));
  }
  hipError_t finish() { return err ? err : (err = hipStreamSynchronize(s)); }
};

// A handle's kernels share its scratch (the ping-pong partition histograms), so consecutive calls
// must run in call order even when they name different streams (NBG_DEFER_GROUP's finish_group on
// another stream, a host submit after device calls, or a caller that moves the handle between
// streams): when the stream changes, the new stream waits for everything issued so far on the
// previous one.  Calls that stay on one stream pay nothing.
// Blocks of a streaming-classify launch: one per CU, or NBG_STREAM_GRID (measurement: 1..CUs).
int stream_grid(const nbg_maglev* h) {
  static const int forced = [] {
    const char* e = std::getenv("NBG_STREAM_GRID");
    return e ? std::atoi(e) : 0;
  }();
  return forced > 0 && forced <= h->cus ? forced : h->cus;
}

int order_after_last(nbg_maglev* h, hipStream_t s) {
  if (!h->issued || h->last_stream == s) return NBG_OK;
  if (!h->order_ev) NBG_HIP(hipEventCreateWithFlags(&h->order_ev, hipEventDisableTiming));
  NBG_HIP(hipEventRecord(h->order_ev, h->last_stream));
  NBG_HIP(hipStreamWaitEvent(s, h->order_ev, 0));
  return NBG_OK;
}

void ring_free(nbg_ring* r);  // the persistent ring's resources (below)

void free_scratch(nbg_maglev* h) {
  (void)hipFree(h->d_idx);
  (void)hipFree(h->d_cursor);
  (void)hipFree(h->d_bucket);
  h->d_idx = h->d_cursor = nullptr;
  h->d_bucket = nullptr;
  h->tiled_cap = 0;
  (void)hipFree(h->d_fixed_len);
  h->d_fixed_len = nullptr;
  h->fixed_len_cap = 0;
  (void)hipFree(h->d_part_hist);
  (void)hipFree(h->d_part_graph);
  (void)hipFree(h->d_part_prefix);
  (void)hipFree(h->d_totals);
  (void)hipFree(h->d_bin_base);
  (void)hipFree(h->d_sink);
  (void)hipFree(h->d_part_multi);
  (void)hipFree(h->d_prefix_multi);
  h->d_prefix_multi = nullptr;
  (void)hipFree(h->d_part_lag);
  (void)hipFree(h->d_counts);
  h->d_part_lag = nullptr;
  h->d_part_hist = nullptr;
  h->d_part_graph = nullptr;
  h->d_part_prefix = nullptr;
  h->d_totals = nullptr;
  h->d_bin_base = nullptr;
  h->d_sink = nullptr;
  h->d_part_multi = nullptr;
  h->d_counts = nullptr;
}

void free_slot_buffers(nbg_maglev::HostSlot& t) {
  (void)hipHostFree(t.h_win);
  (void)hipHostFree(t.h_len);
  (void)hipHostFree(t.h_backend);
  (void)hipHostFree(t.h_perm);
  (void)hipHostFree(t.h_counts);
  (void)hipFree(t.d_win);
  (void)hipFree(t.d_len);
  (void)hipFree(t.d_backend);
  (void)hipFree(t.d_perm);
  (void)hipFree(t.d_counts);
  t.h_win = t.d_win = nullptr;
  t.h_len = t.d_len = t.h_backend = t.d_backend = nullptr;
  t.h_perm = t.h_counts = t.d_perm = t.d_counts = nullptr;
  t.dh_win = nullptr;
  t.dh_len = t.dh_backend = nullptr;
  t.dh_perm = t.dh_counts = nullptr;
  t.cap = 0;
}

bool flag_set(const nbg_maglev::HostSlot& t);
int wait_flag(nbg_maglev* h, nbg_maglev::HostSlot& t);

void free_host_path(nbg_maglev* h) {
  if (h->host_compute) (void)hipStreamSynchronize(h->host_compute);  // direct launches record no event
  for (auto& t : h->slots)
    if (t.busy && t.direct) (void)wait_flag(h, t);  // a host-ring batch reads the LUT and writes the slot
  if (h->hring) {
    h->hring->attached.fetch_sub(1);
    h->hring = nullptr;
  }
  for (auto& t : h->slots) {
    if (t.h_flag) (void)hipHostFree(t.h_flag);
    t.h_flag = t.dh_flag = nullptr;
    if (t.busy && t.done) (void)hipEventSynchronize(t.done);
    t.busy = false;
    free_slot_buffers(t);
    if (t.done) (void)hipEventDestroy(t.done);
    t.done = nullptr;
  }
  if (h->host_compute) (void)hipStreamDestroy(h->host_compute);
  h->host_compute = nullptr;
}

int upload(nbg_maglev* h) {
  DeviceGuard g(h->device);
  h->wide = h->nb > 256;
  const size_t esz = h->wide ? 2 : 1;
  h->lut_bytes = static_cast<uint32_t>((h->m * esz + 15) & ~uint64_t(15));
  h->lut_alloc = (h->lut_bytes + 1023u) & ~1023u;
  std::vector<uint8_t> buf(h->lut_alloc, 0);
  if (h->wide) {
    std::memcpy(buf.data(), h->lut_host.data(), h->m * 2);
  } else {
    for (uint64_t j = 0; j < h->m; ++j) buf[j] = static_cast<uint8_t>(h->lut_host[j]);
  }
  NBG_HIP(hipMalloc(&h->d_lut, h->lut_alloc));
  const size_t nbins = h->nb + 1;
  NBG_HIP(hipMalloc(&h->d_part_hist, 2 * kMaxParts * nbins * sizeof(uint32_t)));
  NBG_HIP(hipMalloc(&h->d_part_graph, kMaxParts * nbins * sizeof(uint32_t)));
  NBG_HIP(hipMalloc(&h->d_part_prefix, kMaxParts * nbins * sizeof(uint32_t)));
  NBG_HIP(hipMalloc(&h->d_totals, nbins * sizeof(uint32_t)));
  NBG_HIP(hipMalloc(&h->d_bin_base, nbins * sizeof(uint32_t)));
  NBG_HIP(hipMalloc(&h->d_sink, 1024));
  NBG_HIP(hipMalloc(&h->d_counts, nbins * sizeof(uint32_t)));
  SetupStream st;  // complete before the handle is returned: any caller stream may use it next
  (void)st.h2d(h->d_lut, buf.data(), h->lut_alloc);
  (void)st.zero(h->d_part_hist, 2 * kMaxParts * nbins * sizeof(uint32_t));
  NBG_HIP(st.finish());  // reports the first failure of the sequence
  if (const char* e = std::getenv("NBG_TPW")) {
    const int v = std::atoi(e);
    h->tiles_per_wave = 1;
    while (static_cast<int>(h->tiles_per_wave) < v && h->tiles_per_wave < 64) h->tiles_per_wave <<= 1;
  }
  if (hipDeviceGetAttribute(&h->cus, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess || h->cus <= 0)
    return set_error(NBG_ENODEV, "hipDeviceGetAttribute(CU count) failed");
  int rc = classify_grid(true, h->lut_bytes, h->nb, h->device, &h->grid_lds);
  if (rc) return rc;
  return classify_grid(false, 0, h->nb, h->device, &h->grid_global);
}

// The LUT is gathered from L2 by default (measured faster: the LDS-staged copy costs
// occupancy); NBG_LUT_LDS stages it in LDS when it fits.
// While a persistent ring runs on the device, kernels that need a whole CU's LDS (the streaming
// kernels, the LDS-staged LUT) would wait for it to end: batches of other handles then take the
// tile-per-wave kernel, which co-runs in the LDS the ring leaves free.
// Many bins while a persistent ring runs on the device: the LDS-light group kernel, which co-runs
// beside the ring instead of waiting for its end.
bool compact_group(const nbg_maglev* h) { return group_compact(h->nb + 1, device_ring_running(h->device)); }

bool use_lds_lut(const nbg_maglev* h, uint32_t flags) {
  return (flags & NBG_LUT_LDS) && h->lut_bytes <= 72 * 1024 && !device_ring_running(h->device);
}

// The streaming classify kernel serves fixed 64-B-aligned slots with a u8 LUT of at most 65537
// entries (config C2); NBG_STREAM=0 selects the tile-per-wave kernel instead (A/B measurements).
// Below ~2 units per block the per-block LUT staging (64 KiB from L2 for every CU) is not
// amortised: smaller batches take the tile-per-wave kernel.
bool use_stream(const nbg_maglev* h, uint64_t n_pkts) {
  static const bool on = [] {
    const char* e = std::getenv("NBG_STREAM");
    return !e || std::atoi(e) != 0;
  }();
  return on && !h->wide && h->m <= 65537 && n_pkts >= 262144 && !device_ring_running(h->device);
}

// NBG_STREAM_DESC: descriptor layouts (IMIX offsets + lengths) with owned windows take the
// streaming kernel too: the u8 LUT staged in LDS (read only, records, or the lpm chain), or the u16
// LUT gathered from L2 (any mode, no chain).  The in-place mode with the u8 LUT does not fit LDS.
// Opt-in: one stream, it classifies C5 in 27.1 us against 28.7 for the tile-per-wave kernel, but it
// holds all LDS of every CU, so with three streams the tile-per-wave kernels co-running beat it
// (profiles/r02_stream_desc_ab.txt).
bool use_stream_desc(const nbg_maglev* h, uint64_t n_pkts, uint32_t flags, bool chain, int mode) {
  if (!(flags & NBG_STREAM_DESC) || n_pkts < 262144 || device_ring_running(h->device)) return false;
  if (h->wide) return !chain;
  return h->m <= 65537 && mode != 1;
}

// Batches of at most 2048 packets take the single-launch small kernel (one block: 3.5 us per call
// back to back at 32 packets and 6.9 us at 1024, against 9.5 and 10.6 us for classify + group; at
// 4096 packets one CU is too little: 14.1 against 11.0 us, profiles/r02_small_batches.json).
// NBG_SMALL=0 disables it (A/B measurements).
bool use_small(uint64_t n_pkts, uint32_t nbins, uint32_t flags, const uint8_t* d_pkts) {
  static const bool on = [] {
    const char* e = std::getenv("NBG_SMALL");
    return !e || std::atoi(e) != 0;
  }();
  return on && n_pkts <= std::min<uint32_t>(small_max(), 2048) && nbins <= kMaxGroupBins &&
         !(flags & (NBG_DEFER_GROUP | NBG_LUT_LDS | NBG_LUT_TILED)) &&
         (reinterpret_cast<uintptr_t>(d_pkts) & 15u) == 0;
}

// Persistent host worker pool for the host path's gather and MAC swap (bound by host
// memory latency over scattered mbufs, not bandwidth): up to 16 threads (the GPU box's CPU share), started on first use and
// kept for the life of the process (no thread start per batch).  One job at a time.
class HostPool {
 public:
  static HostPool& get() {
    static HostPool* pool = new HostPool();  // never destroyed: its workers live as long as the process
    return *pool;
  }
  // fn(begin, end) over [0, n) split into one contiguous part per thread (the caller runs one)
  void run(uint64_t n, const std::function<void(uint64_t, uint64_t)>& fn) {
    if (n < 32768 || workers_ == 0) {
      fn(0, n);
      return;
    }
    std::lock_guard<std::mutex> job_lock(job_mutex_);
    const unsigned parts = workers_ + 1;
    const uint64_t per = (n + parts - 1) / parts;
    {
      std::lock_guard<std::mutex> g(m_);
      job_ = [&](unsigned k) {
        const uint64_t b = std::min(n, k * per), e = std::min(n, b + per);
        if (b < e) fn(b, e);
      };
      pending_ = workers_;
      ++gen_;
    }
    cv_.notify_all();
    job_(0);
    std::unique_lock<std::mutex> lk(m_);
    done_cv_.wait(lk, [&] { return pending_ == 0; });
  }

 private:
  HostPool() {
    const unsigned hw = std::thread::hardware_concurrency();
    workers_ = (hw ? std::min(hw, 16u) : 1u) - 1;
    for (unsigned k = 1; k <= workers_; ++k) std::thread([this, k] { loop(k); }).detach();
  }
  void loop(unsigned k) {
    uint64_t seen = 0;
    for (;;) {
      std::function<void(unsigned)> job;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        job = job_;
      }
      job(k);
      std::lock_guard<std::mutex> g(m_);
      if (--pending_ == 0) done_cv_.notify_one();
    }
  }
  unsigned workers_ = 0;
  std::mutex job_mutex_, m_;
  std::condition_variable cv_, done_cv_;
  std::function<void(unsigned)> job_;
  unsigned pending_ = 0;
  uint64_t gen_ = 0;
};

template <typename F>
void parallel_for(uint64_t n, F fn) {
  HostPool::get().run(n, std::function<void(uint64_t, uint64_t)>(fn));
}

int finish_create(nbg_maglev* h, int device, nbg_maglev** out) {
  int ndev = 0;
  const hipError_t ce = hipGetDeviceCount(&ndev);
  if (ce != hipSuccess || ndev <= 0) {
    delete h;
    return set_error(NBG_ENODEV, "no HIP device available (the Maglev path has no CPU fallback): %s, %d devices",
                     hipGetErrorString(ce), ndev);
  }
  if (device < 0 || device >= ndev) {
    delete h;
    return set_error(NBG_ENODEV, "device %d out of range (%d devices)", device, ndev);
  }
  h->device = device;
  int rc = upload(h);
  if (rc) {
    nbg_maglev_destroy(h);
    return rc;
  }
  *out = h;
  return NBG_OK;
}

}  // namespace

extern "C" {

const char* nbg_last_error(void) { return g_err; }

int nbg_maglev_create(const char* const* names, const uint32_t* name_lens, uint32_t n_backends, uint64_t table_size,
                      int device, nbg_maglev** out) {
  if (!out || !names || !name_lens) return set_error(NBG_EINVAL, "nbg_maglev_create: null argument");
  *out = nullptr;
  if (n_backends < 1 || n_backends > 65534) return set_error(NBG_EINVAL, "n_backends must be in [1, 65534]");
  if (table_size < 2 || table_size > (1ull << 31)) return set_error(NBG_EINVAL, "table_size must be in [2, 2^31]");
  std::vector<uint32_t> e;
  int rc = build_lut(names, name_lens, n_backends, table_size, e);
  if (rc) return rc;
  nbg_maglev* h = new (std::nothrow) nbg_maglev();
  if (!h) return set_error(NBG_ENOMEM, "out of host memory");
  h->nb = n_backends;
  h->m = table_size;
  h->lut_host.resize(table_size);
  for (uint64_t j = 0; j < table_size; ++j) h->lut_host[j] = static_cast<uint16_t>(e[j]);
  return finish_create(h, device, out);
}

int nbg_maglev_create_from_lut(const uint16_t* lut, uint64_t table_size, uint32_t n_backends, int device,
                               nbg_maglev** out) {
  if (!out || !lut) return set_error(NBG_EINVAL, "nbg_maglev_create_from_lut: null argument");
  *out = nullptr;
  if (n_backends < 1 || n_backends > 65534) return set_error(NBG_EINVAL, "n_backends must be in [1, 65534]");
  if (table_size < 2 || table_size > (1ull << 31)) return set_error(NBG_EINVAL, "table_size must be in [2, 2^31]");
  for (uint64_t j = 0; j < table_size; ++j)
    if (lut[j] >= n_backends) return set_error(NBG_EINVAL, "lut[%llu]=%u >= n_backends", (unsigned long long)j, lut[j]);
  nbg_maglev* h = new (std::nothrow) nbg_maglev();
  if (!h) return set_error(NBG_ENOMEM, "out of host memory");
  h->nb = n_backends;
  h->m = table_size;
  h->lut_host.assign(lut, lut + table_size);
  return finish_create(h, device, out);
}

void nbg_maglev_destroy(nbg_maglev* h) {
  if (!h) return;
  if (h->ring) (void)nbg_ring_stop(h->ring);
  if (h->ring_leaked) {
    // a ring kernel that did not end at its stop may still read the LUT and the ring's buffers: leak
    // the handle's device memory rather than free it under the kernel (the host struct goes)
    delete h;
    return;
  }
  if (h->ring_spare) {
    DeviceGuard g(h->device);
    ring_free(h->ring_spare);
    h->ring_spare = nullptr;
  }
  for (nbg_ring* r : h->ring_dead) {
    DeviceGuard g(h->device);
    ring_free(r);
  }
  h->ring_dead.clear();
  {
    DeviceGuard g(h->device);
    free_scratch(h);
    free_host_path(h);
    (void)hipFree(h->d_lut);
    if (h->order_ev) (void)hipEventDestroy(h->order_ev);
  }
  delete h;
}

uint32_t nbg_maglev_backends(const nbg_maglev* h) { return h ? h->nb : 0; }
uint64_t nbg_maglev_table_size(const nbg_maglev* h) { return h ? h->m : 0; }

int nbg_maglev_lut(const nbg_maglev* h, uint16_t* out, uint64_t n) {
  if (!h || !out) return set_error(NBG_EINVAL, "nbg_maglev_lut: null argument");
  if (n < h->m) return set_error(NBG_EINVAL, "nbg_maglev_lut: buffer of %llu < table size %llu",
                                 (unsigned long long)n, (unsigned long long)h->m);
  std::memcpy(out, h->lut_host.data(), h->m * sizeof(uint16_t));
  return NBG_OK;
}

int nbg_maglev_reserve(nbg_maglev* h, uint64_t max_pkts) {
  if (!h) return set_error(NBG_EINVAL, "nbg_maglev_reserve: null handle");
  (void)max_pkts;  // scratch is sized per handle (at most kMaxParts partitions), never per call
  return NBG_OK;
}

int nbg_maglev_classify_device(nbg_maglev* h, uint8_t* d_pkts, const uint32_t* d_off, const uint16_t* d_len,
                               uint32_t stride, uint16_t fixed_len, uint64_t n_pkts, uint32_t flags,
                               uint16_t* d_backend, uint32_t* d_perm, uint32_t* d_counts, void* stream) {
  return nbg_maglev_classify_device_ex(h, d_pkts, d_off, d_len, stride, fixed_len, n_pkts, flags, d_backend, d_perm,
                                       d_counts, nullptr, stream);
}

}  // extern "C"

namespace {

// The partition rows of a captured call are zeroed inside the graph, by a kernel node.  A memset node
// faults on its second replay when the graph is launched on the legacy null stream under PyTorch's
// bundled HIP 7.0 runtime, as torch.cuda.graph replays do by default; the image's HIP 7.2 replays it
// clean, and so does HIP 7.0 on a created stream (profiles/DESIGN_r01-r03_history.md, r03_graph_*.txt).
int zero_captured(uint32_t* p, size_t words, void* stream) { return launch_zero(p, words, stream); }

// The pending lagged group (NBG_GROUP_LAG) as a group launch of its own on `s` (already ordered
// after the handle's last launch).  Its rows live in the lag set it was classified into; the
// standalone group kernel zeroes nothing there (the next lagged classify zeroes the sets).
int flush_lag(nbg_maglev* h, hipStream_t s) {
  h->pending = h->pending_lag = false;
  return launch_group(h->pending_args, kScanDirect, s, compact_group(h));
}

// A lagged classify (NBG_GROUP_LAG): the streaming kernel accumulates this batch's partition rows
// into lag set k, groups the pending batch (fuse) from set k - 1, and zeroes set k + 1 (mod 3) for
// the call after next; this batch becomes the pending one.
int classify_lag(nbg_maglev* h, ClassifyArgs& a, bool fuse, uint32_t n_parts, uint32_t part_pkts, uint32_t* d_perm,
                 uint32_t* d_counts, hipStream_t s) {
  const uint32_t nbins = h->nb + 1;
  const size_t set_words = static_cast<size_t>(kMaxParts) * nbins;
  if (!h->d_part_lag) {
    NBG_HIP(hipMalloc(&h->d_part_lag, 3 * set_words * sizeof(uint32_t)));
    NBG_HIP(hipMemsetAsync(h->d_part_lag, 0, 3 * set_words * sizeof(uint32_t), s));
    h->lag_dirty = 0;
    h->lag_idx = 0;
  }
  const uint32_t k = h->lag_idx, z = (k + 1) % 3;
  uint32_t* setk = h->d_part_lag + k * set_words;
  if (h->lag_dirty & (1u << k)) {  // only after an unusual call sequence: the rotation zeroes ahead
    NBG_HIP(hipMemsetAsync(setk, 0, set_words * sizeof(uint32_t), s));
    h->lag_dirty &= ~(1u << k);
  }
  a.part_hist = setk;
  LagGroup lg = fuse ? h->pending_lg : LagGroup{};
  lg.zero = h->d_part_lag + z * set_words;
  lg.zero_words = static_cast<uint32_t>(set_words);
  const int rc = launch_classify_stream_lag(a, lg, h->cus, s);
  if (rc) return rc;  // the pending group (if any) stays pending: finish_group or the next call launches it
  h->pending = h->pending_lag = false;
  h->lag_dirty = (h->lag_dirty | (1u << k)) & ~(1u << z);
  h->lag_idx = z;
  LagGroup& p = h->pending_lg;
  p = LagGroup{};
  p.backend = a.backend;
  p.perm = d_perm;
  p.counts = d_counts ? d_counts : h->d_counts;
  p.part_hist = setk;
  p.n_pkts = a.n_pkts;
  p.part_pkts = part_pkts;
  p.n_parts = n_parts;
  p.hist16 = a.hist16;
  GroupArgs& ga = h->pending_args;
  ga = GroupArgs{};
  ga.backend = a.backend;
  ga.n_pkts = a.n_pkts;
  ga.nb = h->nb;
  uint32_t bits = 0;
  while ((1u << bits) < nbins) ++bits;
  ga.bits = bits;
  ga.n_parts = n_parts;
  ga.part_pkts = part_pkts;
  ga.part_hist = setk;
  ga.hist16 = a.hist16;
  ga.counts = p.counts;
  ga.perm = d_perm;
  ga.bin_base = h->d_bin_base;
  h->pending = h->pending_lag = true;
  return NBG_OK;
}

// One classify (+ grouping) launch; `lpm` non-null runs the chained test/lpm stage first.
// small_done (the host path's direct batches): the small kernel's completion word and value; the call
// fails unless the batch takes the small kernel
int classify_common(nbg_maglev* h, uint8_t* d_pkts, const uint32_t* d_off, const uint16_t* d_len, uint32_t stride,
                    uint16_t fixed_len, uint64_t n_pkts, uint32_t flags, uint16_t* d_backend, uint32_t* d_perm,
                    uint32_t* d_counts, uint8_t* d_mac_out, const nbg_lpm* lpm, uint32_t lpm_groups,
                    uint16_t* d_gate, void* stream, uint32_t* small_done = nullptr, uint32_t small_done_val = 0,
                    bool win32 = false) {
  if (!h) return set_error(NBG_EINVAL, "classify: null handle");
  if (h->ring) return set_error(NBG_EBUSY, "classify: the handle's persistent ring is running (nbg_ring_stop first)");
  if (h->pending && !h->pending_lag)
    return set_error(NBG_EINVAL, "classify: a deferred group is pending (nbg_maglev_finish_group)");
  if ((flags & NBG_GROUP_LAG) && (flags & NBG_DEFER_GROUP))
    return set_error(NBG_EINVAL, "classify: NBG_GROUP_LAG with NBG_DEFER_GROUP");
  if (n_pkts >= (1ull << 30)) return set_error(NBG_EINVAL, "classify: n_pkts must be < 2^30");
  if (n_pkts == 0) {
    return d_counts ? zero_captured(d_counts, h->nb + 1, stream) : NBG_OK;  // a kernel: capturable
  }
  if (!d_pkts || !d_backend) return set_error(NBG_EINVAL, "classify: null packet or backend buffer");
  if (lpm && (!d_gate || lpm->device != h->device))
    return set_error(NBG_EINVAL, "chain: null gate buffer, or lpm and maglev handles on different devices");
  if (!d_off && stride == 0) return set_error(NBG_EINVAL, "classify: stride 0 without offsets");
  if (!d_off && stride >= (1u << 24)) return set_error(NBG_EINVAL, "classify: stride must be < 2^24 (use offsets)");
  if (!d_off && static_cast<unsigned __int128>(n_pkts) * stride > (1ull << 40))
    return set_error(NBG_EINVAL, "classify: batch too large");
  DeviceGuard g(h->device);
  const bool group = d_perm || d_counts;
  const uint32_t nbins = h->nb + 1;
  if (group && nbins > kMaxWideBins)
    return set_error(NBG_EINVAL, "classify: group output supports at most %u backends", kMaxWideBins - 1);
  const bool wide = group && nbins > kMaxGroupBins;  // wide grouping path (hist + scan + group_wide)
  // A call captured into a hipGraph is replayed with the same arguments, so it must not rely on the
  // ping-pong histograms (a replay would find them unzeroed): it zeroes and uses its own buffer,
  // and leaves the handle's parity alone.  Cross-stream ordering cannot be recorded during capture:
  // the caller orders the capture after the handle's earlier work.
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  NBG_HIP(hipStreamIsCapturing(static_cast<hipStream_t>(stream), &cap));
  const bool capturing = cap != hipStreamCaptureStatusNone;
  if (capturing && (flags & (NBG_DEFER_GROUP | NBG_GROUP_LAG)))
    return set_error(NBG_EINVAL, "classify: NBG_DEFER_GROUP / NBG_GROUP_LAG cannot be captured in a graph");
  if (capturing && h->pending)
    return set_error(NBG_EINVAL, "classify: a lagged group is pending (nbg_maglev_finish_group before capturing)");
  // A graph keeps the pointers it was captured with, so a captured call must not use scratch that a
  // later eager call may reallocate: the NBG_LUT_TILED buckets and the fixed_len array that
  // descriptor batches without lengths get (grown on demand).  Everything else it touches is
  // allocated with the handle.
  if (capturing && (flags & NBG_LUT_TILED))
    return set_error(NBG_EINVAL, "classify: NBG_LUT_TILED cannot be captured in a graph (its scratch grows)");
  if (capturing && d_off && !d_len && !(!lpm && use_small(n_pkts, nbins, flags, d_pkts)))
    return set_error(NBG_EINVAL, "classify: pass d_len to capture a descriptor batch of more than %u packets",
                     small_max());
  int rc = capturing ? NBG_OK : order_after_last(h, static_cast<hipStream_t>(stream));
  if (rc) return rc;
  const bool lds = use_lds_lut(h, flags);
  // each wave walks tpw consecutive 64-packet tiles (software-pipelined); the LDS-LUT variant
  // runs a resident grid of 1024-thread blocks so that the LUT staging is amortised
  const uint32_t waves_per_block = (lds ? kLdsBlock : kBlock) / 64;
  const uint64_t n_tiles64 = (n_pkts + 63) / 64;
  // a block's packets (64 * waves * tpw, a power of two <= kChunk) must not straddle a partition
  const uint32_t tpw_max = kChunk / (64u * waves_per_block);
  uint32_t tpw = std::min(h->tiles_per_wave, tpw_max);
  if (lds) {
    const uint64_t want = (n_tiles64 + uint64_t(h->grid_lds) * waves_per_block - 1) / (uint64_t(h->grid_lds) * waves_per_block);
    tpw = 1;
    while (tpw < want && tpw < tpw_max) tpw <<= 1;
  }
  const int grid = static_cast<int>((n_tiles64 + uint64_t(tpw) * waves_per_block - 1) / (uint64_t(tpw) * waves_per_block));
  const uint64_t per = (n_pkts + kChunk * kMaxParts - 1) / (kChunk * kMaxParts);
  const uint32_t part_pkts = static_cast<uint32_t>(per * kChunk);
  const uint32_t n_parts = static_cast<uint32_t>((n_pkts + part_pkts - 1) / part_pkts);
  uint32_t* part_cur = capturing ? h->d_part_graph : h->d_part_hist + static_cast<size_t>(h->parity) * kMaxParts * nbins;
  uint32_t* part_next = capturing ? nullptr : h->d_part_hist + static_cast<size_t>(h->parity ^ 1u) * kMaxParts * nbins;
  const bool small = !lpm && use_small(n_pkts, nbins, flags, d_pkts);

  // Descriptor kernels read off[] and len[] both: offsets without lengths get a fixed_len-filled
  // array.  The small kernel reads fixed_len itself, so a captured call (always the small path)
  // never records this fill nor depends on the cached value (a captured fill, or a
  // capture relying on the cache, went stale when an eager call changed fixed_len).
  if (d_off && !d_len && !small) {
    if (h->fixed_len_cap < n_pkts) {
      (void)hipFree(h->d_fixed_len);
      h->d_fixed_len = nullptr;
      h->fixed_len_cap = 0;
      NBG_HIP(hipMalloc(&h->d_fixed_len, n_pkts * sizeof(uint16_t)));
      h->fixed_len_cap = n_pkts;
      h->fixed_len_val = static_cast<uint16_t>(~fixed_len);  // force the fill below
    }
    if (h->fixed_len_val != fixed_len) {
      NBG_HIP(hipMemsetD16Async(reinterpret_cast<hipDeviceptr_t>(h->d_fixed_len), fixed_len, h->fixed_len_cap,
                                static_cast<hipStream_t>(stream)));
      h->fixed_len_val = fixed_len;
    }
    d_len = h->d_fixed_len;
  }
  ClassifyArgs a{};
  a.pkts = d_pkts;
  a.off = d_off;
  a.len = d_len;
  a.stride = stride;
  a.fixed_len = fixed_len;
  a.n_pkts = static_cast<uint32_t>(n_pkts);
  a.tiles_per_wave = tpw;
  a.lut = h->d_lut;
  a.m = static_cast<uint32_t>(h->m);
  a.lut_lds_bytes = lds ? h->lut_bytes : 0;
  a.mu = ~0ull / h->m + ((~0ull % h->m) + 1 == h->m ? 1 : 0);  // floor(2^64 / m)
  a.nb = h->nb;
  a.swap = (flags & NBG_SWAP_MACS) && !lpm ? 1u : 0u;  // chain: lpm's and maglev's swaps cancel
  // a 64-B window per packet start is owned: fixed slots of >= 64 B, or the caller says so
  a.win_owned = (!d_off && stride >= 64) || (flags & NBG_OWNED_WINDOWS) ? 1u : 0u;
  a.wb_full = (flags & NBG_WB_PARTIAL) ? 0u : 1u;
  a.lean = (!d_off && !d_len && a.win_owned && stride % 16 == 0 && (reinterpret_cast<uintptr_t>(d_pkts) & 15u) == 0 &&
            fixed_len >= 48)
               ? 1u
               : 0u;
  a.backend = d_backend;
  a.mac_out = d_mac_out;
  const bool hist_k = group && !hist_in_classify(nbins);  // histograms by hist_kernel instead
  a.part_hist = group && !hist_k ? part_cur : nullptr;
  a.part_pkts = part_pkts;
  const int scan = group && !wide ? pick_group_scan(nbins, n_parts) : kScanKernel;
  // packed 16-bit partition rows where the classify kernel writes them and the group kernel sums
  // them itself (partition counts stay below 65536)
  a.hist16 = group && !hist_k && scan == kScanDirect && part_pkts < 65536 ? 1u : 0u;
  if (lpm) {
    a.tbl24 = lpm->d_tbl24;
    a.tbl_long = lpm->d_tbl_long;
    a.lpm_groups = lpm_groups;
    a.gate = d_gate;
    a.mac_out = nullptr;
  }
  if (!capturing) {
    h->last_stream = static_cast<hipStream_t>(stream);
    h->issued = true;
  }
  // NBG_GROUP_LAG: this batch's grouping is left pending (carried by the next call's launch) when
  // it takes the streaming kernel with in-kernel histograms and the direct scan; a pending lagged
  // group rides on this launch when both fit, else it is launched alone first
  const bool lag = (flags & NBG_GROUP_LAG) && !capturing && group && !lpm && !wide && !hist_k &&
                   scan == kScanDirect && a.lean && !lds && !(flags & NBG_LUT_TILED) && !small &&
                   use_stream(h, n_pkts) && n_parts <= static_cast<uint32_t>(h->cus) &&
                   stream_lds(h->nb, !a.swap ? 0 : (a.mac_out ? 2 : 1), true) <= 160u * 1024u;
  const bool fuse = lag && h->pending_lag && h->pending_lg.n_parts <= static_cast<uint32_t>(h->cus);
  if (h->pending_lag && !fuse && (rc = flush_lag(h, static_cast<hipStream_t>(stream)))) return rc;
  if (small_done && !small) return set_error(NBG_EINVAL, "classify: a completion word needs the small kernel");
  if (win32 && (!small || a.swap)) return set_error(NBG_EINVAL, "classify: 32-B windows need the small kernel, no swap");
  a.win32 = win32 ? 1u : 0u;
  if (small) {
    GroupArgs g{};
    g.perm = d_perm;
    g.counts = d_counts ? d_counts : (d_perm ? h->d_counts : nullptr);
    return launch_small(a, g, h->wide, stream, small_done, small_done_val);
  }
  const bool tiled = (flags & NBG_LUT_TILED) && h->wide && !lpm;
  if (tiled) {
    const uint32_t n_tiles = lut_tiles(h->m);
    if (h->tiled_cap < n_pkts) {
      if (capturing) return set_error(NBG_EINVAL, "classify: NBG_LUT_TILED scratch cannot grow in a graph");
      (void)hipFree(h->d_idx);
      (void)hipFree(h->d_cursor);
      (void)hipFree(h->d_bucket);
      h->d_idx = h->d_cursor = nullptr;
      h->d_bucket = nullptr;
      h->tiled_cap = 0;
      NBG_HIP(hipMalloc(&h->d_idx, n_pkts * 4));
      NBG_HIP(hipMalloc(&h->d_cursor, n_tiles * 4));
      NBG_HIP(hipMalloc(&h->d_bucket, static_cast<size_t>(n_tiles) * n_pkts * 8));
      h->tiled_cap = n_pkts;
    }
    a.idx_out = h->d_idx;
    if ((rc = launch_classify_idx(a, grid, stream))) return rc;
    NBG_HIP(hipMemsetAsync(h->d_cursor, 0, n_tiles * 4, static_cast<hipStream_t>(stream)));
    TileArgs ta{};
    ta.idx = h->d_idx;
    ta.n_pkts = static_cast<uint32_t>(n_pkts);
    ta.n_tiles = n_tiles;
    ta.m = static_cast<uint32_t>(h->m);
    ta.lut = h->d_lut;
    ta.cursor = h->d_cursor;
    ta.bucket = h->d_bucket;
    ta.bucket_cap = static_cast<uint32_t>(h->tiled_cap);
    ta.backend = d_backend;
    rc = launch_tiled_lookup(ta, stream);
  } else if (a.lean && !lds && !lpm && use_stream(h, n_pkts)) {
    const uint64_t waves = static_cast<uint64_t>(h->cus) * stream_waves_per_block();
    a.tiles_per_wave = static_cast<uint32_t>((n_tiles64 + waves - 1) / waves);
    a.lut_lds_bytes = std::min<uint32_t>(h->lut_alloc, 65536u);
    a.lut_tail = h->m > 65536 ? h->lut_host[65536] : 0u;
    if (capturing && a.part_hist)
      if ((rc = zero_captured(a.part_hist, static_cast<size_t>(n_parts) * nbins, stream))) return rc;
    if (lag) return classify_lag(h, a, fuse, n_parts, part_pkts, d_perm, d_counts, static_cast<hipStream_t>(stream));
    rc = launch_classify_stream(a, stream_grid(h), stream);
  } else if (d_off && d_len && a.win_owned && !lds && (reinterpret_cast<uintptr_t>(d_pkts) & 15u) == 0 &&
             use_stream_desc(h, n_pkts, flags, lpm != nullptr, lpm || !a.swap ? 0 : (a.mac_out ? 2 : 1))) {
    if (!h->wide) {
      a.lut_lds_bytes = std::min<uint32_t>(h->lut_alloc, 65536u);
      a.lut_tail = h->m > 65536 ? h->lut_host[65536] : 0u;
    }
    if (capturing && a.part_hist)
      if ((rc = zero_captured(a.part_hist, static_cast<size_t>(n_parts) * nbins, stream))) return rc;
    a.sink = h->d_sink;
    rc = launch_classify_stream_desc(a, h->wide, h->cus, stream);
  } else {
    if (capturing && a.part_hist)
      if ((rc = zero_captured(a.part_hist, static_cast<size_t>(n_parts) * nbins, stream))) return rc;
    rc = launch_classify(a, h->wide, lds, grid, stream);
  }
  if (rc) return rc;
  if (group) {
    ScanArgs sa{};
    sa.part_hist = part_cur;
    sa.part_prefix = h->d_part_prefix;
    sa.totals = h->d_totals;
    sa.n_parts = n_parts;
    sa.nbins = nbins;
    HistArgs ha{};
    ha.backend = d_backend;
    ha.n_pkts = static_cast<uint32_t>(n_pkts);
    ha.nb = h->nb;
    ha.part_pkts = part_pkts;
    ha.n_parts = n_parts;
    ha.part_hist = part_cur;
    GroupArgs ga{};
    ga.backend = d_backend;
    ga.n_pkts = static_cast<uint32_t>(n_pkts);
    ga.nb = h->nb;
    uint32_t bits = 0;
    while ((1u << bits) < nbins) ++bits;
    ga.bits = bits;
    ga.n_parts = n_parts;
    ga.part_pkts = part_pkts;
    ga.part_hist = part_cur;
    ga.part_prefix = h->d_part_prefix;
    ga.totals = h->d_totals;
    ga.hist16 = a.hist16;
    ga.part_hist_next = part_next;
    ga.next_words = part_next ? kMaxParts * nbins : 0u;
    ga.counts = d_counts ? d_counts : h->d_counts;
    ga.perm = d_perm;
    ga.bin_base = h->d_bin_base;
    if (!capturing) h->parity ^= 1u;
    if (flags & NBG_DEFER_GROUP) {
      h->pending = true;
      h->pending_scan_mode = scan;
      h->pending_hist = hist_k;
      h->pending_hist_args = ha;
      h->pending_args = ga;
      h->pending_scan = sa;
      h->pending_wide = wide;
    } else {
      if (hist_k && (rc = launch_hist(ha, stream))) return rc;
      if (scan == kScanKernel && (rc = launch_scan(sa, stream))) return rc;
      if ((rc = wide ? launch_group_wide(ga, stream) : launch_group(ga, scan, stream, compact_group(h)))) return rc;
    }
  }
  return NBG_OK;
}

// Several descriptor batches (IMIX: u32 offset + u16 length per packet; several RX queues' bursts)
// through one tile-per-wave classify launch, then one hist (many backends), one scan (many
// partitions x bins) and one group launch over all of them.  The launch's ramp and tail, ~6.7 us of a
// 1M C5 batch's 26.9 us on one launch (profiles/r04_desc_size_sweep.txt), are paid once per call.
int desc_multi_common(nbg_maglev* h, const nbg_desc_batch* batches, uint32_t n_batches, uint32_t flags,
                      const nbg_lpm* lpm, uint32_t lpm_groups, void* stream) {
  const char* what = lpm ? "chain (multi)" : "classify (descriptor multi)";
  if (!h) return set_error(NBG_EINVAL, "%s: null handle", what);
  if (!batches || n_batches == 0 || n_batches > NBG_MAX_MULTI)
    return set_error(NBG_EINVAL, "%s: 1..%u batches", what, NBG_MAX_MULTI);
  if (flags & ~(NBG_SWAP_MACS | NBG_OWNED_WINDOWS | NBG_DEFER_GROUP | NBG_WB_PARTIAL))
    return set_error(NBG_EINVAL, "%s: flags other than NBG_SWAP_MACS, NBG_OWNED_WINDOWS, NBG_WB_PARTIAL and NBG_DEFER_GROUP",
                     what);
  if (h->ring) return set_error(NBG_EBUSY, "%s: the handle's persistent ring is running", what);
  if (lpm && lpm->device != h->device) return set_error(NBG_EINVAL, "%s: lpm and maglev handles on different devices", what);
  if (h->pending_lag) {  // a pending lagged group is launched alone first
    const int rc = nbg_maglev_finish_group(h, stream);
    if (rc) return rc;
  }
  if (h->pending) return set_error(NBG_EINVAL, "%s: a deferred group is pending (nbg_maglev_finish_group)", what);
  const bool group = batches[0].d_perm || batches[0].d_counts;
  uint64_t max_n = 0;
  for (uint32_t j = 0; j < n_batches; ++j) {
    const nbg_desc_batch& x = batches[j];
    if ((x.d_perm || x.d_counts) != group)
      return set_error(NBG_EINVAL, "%s: batch %u: every batch or none has perm/counts", what, j);
    if (x.n_pkts >= (1ull << 30)) return set_error(NBG_EINVAL, "%s: batch %u: n_pkts must be < 2^30", what, j);
    if (x.n_pkts && (!x.d_pkts || !x.d_off || !x.d_len || !x.d_backend || (lpm && !x.d_gate)))
      return set_error(NBG_EINVAL, "%s: batch %u: null packet, offset, length, backend%s buffer", what, j,
                       lpm ? " or gate" : "");
    max_n = std::max<uint64_t>(max_n, x.n_pkts);
  }
  const uint32_t nbins = h->nb + 1;
  if (group && nbins > kMaxGroupBins) {
    // the wide grouping path has no multi-batch form: one batch after another (same results)
    if (flags & NBG_DEFER_GROUP)
      return set_error(NBG_EINVAL, "%s: NBG_DEFER_GROUP needs at most %u backends", what, kMaxGroupBins - 1);
    for (uint32_t j = 0; j < n_batches; ++j) {
      const nbg_desc_batch& x = batches[j];
      const int rc = classify_common(h, x.d_pkts, x.d_off, x.d_len, 0, 0, x.n_pkts, flags, x.d_backend, x.d_perm,
                                     x.d_counts, nullptr, lpm, lpm_groups, x.d_gate, stream);
      if (rc) return rc;
    }
    return NBG_OK;
  }
  DeviceGuard g(h->device);
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  NBG_HIP(hipStreamIsCapturing(static_cast<hipStream_t>(stream), &cap));
  if (cap != hipStreamCaptureStatusNone) return set_error(NBG_EINVAL, "%s: cannot be captured in a graph", what);
  // one partition size for every batch (as the fixed-slot multi path): the group grid is
  // n_batches x the largest batch's partitions
  const uint64_t per = (max_n + kChunk * kMaxParts - 1) / (kChunk * kMaxParts);
  const uint32_t part_pkts = static_cast<uint32_t>(std::max<uint64_t>(per, 1) * kChunk);
  const uint32_t n_parts_max = static_cast<uint32_t>(std::max<uint64_t>((max_n + part_pkts - 1) / part_pkts, 1));
  const bool hist_k = group && !hist_in_classify(nbins);
  const int scan = group ? pick_group_scan(nbins, n_parts_max) : kScanDirect;
  const size_t set_words = static_cast<size_t>(kMaxMulti) * kMaxParts * nbins;
  if (group && !h->d_part_multi) {
    NBG_HIP(hipMalloc(&h->d_part_multi, 2 * set_words * sizeof(uint32_t)));
    SetupStream st;
    (void)st.zero(h->d_part_multi, 2 * set_words * sizeof(uint32_t));
    NBG_HIP(st.finish());
  }
  if (group && scan == kScanKernel && !h->d_prefix_multi)
    NBG_HIP(hipMalloc(&h->d_prefix_multi, (set_words + static_cast<size_t>(kMaxMulti) * nbins) * sizeof(uint32_t)));
  int rc = order_after_last(h, static_cast<hipStream_t>(stream));
  if (rc) return rc;
  uint32_t* set_cur = group ? h->d_part_multi + static_cast<size_t>(h->mparity) * set_words : nullptr;
  uint32_t* set_next = group ? h->d_part_multi + static_cast<size_t>(h->mparity ^ 1u) * set_words : nullptr;
  ClassifyArgs a{};
  a.tiles_per_wave = std::min<uint32_t>(h->tiles_per_wave, 4u);  // NBG_TPW (measurement): 1, 2 or 4
  a.lut = h->d_lut;
  a.m = static_cast<uint32_t>(h->m);
  a.mu = ~0ull / h->m + ((~0ull % h->m) + 1 == h->m ? 1 : 0);  // floor(2^64 / m)
  a.nb = h->nb;
  a.swap = (flags & NBG_SWAP_MACS) && !lpm ? 1u : 0u;  // chain: lpm's and maglev's swaps cancel
  a.win_owned = (flags & NBG_OWNED_WINDOWS) ? 1u : 0u;
  a.wb_full = (flags & NBG_WB_PARTIAL) ? 0u : 1u;
  a.part_pkts = part_pkts;
  // partition rows from the classify kernel's flush (few backends, rows accumulated: zeroed by the
  // previous call's group launch) or from hist_kernel (many, rows stored whole)
  a.hist16 = group && !hist_k && scan == kScanDirect && part_pkts < 65536 ? 1u : 0u;
  if (lpm) {
    a.tbl24 = lpm->d_tbl24;
    a.tbl_long = lpm->d_tbl_long;
    a.lpm_groups = lpm_groups;
  }
  const uint32_t bp = classify_block_pkts() * a.tiles_per_wave;
  DescBatches db{};
  GroupMulti gm{};
  HistMulti hm{};
  ScanMulti sm{};
  uint32_t bits = 0;
  while ((1u << bits) < nbins) ++bits;
  uint32_t blocks = 0;
  for (uint32_t j = 0; j < n_batches; ++j) {
    const nbg_desc_batch& x = batches[j];
    const uint32_t n = static_cast<uint32_t>(x.n_pkts);
    const uint32_t n_parts = n ? (n + part_pkts - 1) / part_pkts : 0u;
    uint32_t* rows = group ? set_cur + static_cast<size_t>(j) * kMaxParts * nbins : nullptr;
    db.pkts[j] = x.d_pkts;
    db.off[j] = x.d_off;
    db.len[j] = x.d_len;
    db.backend[j] = x.d_backend;
    db.gate[j] = x.d_gate;
    db.part_hist[j] = group && !hist_k ? rows : nullptr;
    db.n_pkts[j] = n;
    db.blk_base[j] = blocks;
    blocks += (n + bp - 1) / bp;
    if (!group) continue;
    HistArgs& ha = hm.h[j];
    ha.backend = x.d_backend;
    ha.n_pkts = n;
    ha.nb = h->nb;
    ha.part_pkts = part_pkts;
    ha.n_parts = n_parts;
    ha.part_hist = rows;
    uint32_t* pre = h->d_prefix_multi ? h->d_prefix_multi + static_cast<size_t>(j) * kMaxParts * nbins : nullptr;
    uint32_t* tot = h->d_prefix_multi ? h->d_prefix_multi + set_words + static_cast<size_t>(j) * nbins : nullptr;
    ScanArgs& sa = sm.s[j];
    sa.part_hist = rows;
    sa.part_prefix = pre;
    sa.totals = tot;
    sa.n_parts = std::max(n_parts, 1u);  // an empty batch scans row 0 (in bounds, unused: no group block)
    sa.nbins = nbins;
    GroupArgs& ga = gm.g[j];
    ga.backend = x.d_backend;
    ga.n_pkts = n;
    ga.nb = h->nb;
    ga.bits = bits;
    ga.n_parts = n_parts;
    ga.part_pkts = part_pkts;
    ga.part_hist = rows;
    ga.part_prefix = pre;
    ga.totals = tot;
    ga.hist16 = a.hist16;
    // the next call's set is zeroed whenever a call on this handle may accumulate rows into it (the
    // classify kernel's flush: few backends), even if this call's rows come from hist_kernel
    ga.part_hist_next = hist_in_classify(nbins) ? set_next : nullptr;
    ga.next_words = hist_in_classify(nbins) ? static_cast<uint32_t>(set_words) : 0u;
    ga.counts = x.d_counts ? x.d_counts : h->d_counts;
    ga.perm = x.d_perm;
  }
  db.blk_base[n_batches] = blocks;
  db.n = n_batches;
  hm.per = n_parts_max;
  gm.per = n_parts_max;
  // what the batches share; per-batch pointers come from db (a's copies only select the layout)
  a.pkts = db.pkts[0];
  a.off = db.off[0];
  a.len = db.len[0];
  h->last_stream = static_cast<hipStream_t>(stream);
  h->issued = true;
  for (uint32_t j = 0; j < n_batches; ++j)  // an empty batch's counts (no group block writes them)
    if (batches[j].n_pkts == 0 && batches[j].d_counts && (rc = zero_captured(batches[j].d_counts, nbins, stream)))
      return rc;
  if ((rc = launch_classify_desc_multi(a, db, h->wide, stream))) return rc;
  if (!group) return NBG_OK;
  h->mparity ^= 1u;
  if (flags & NBG_DEFER_GROUP) {
    h->pending = true;
    h->pending_multi = n_batches;
    h->pending_gm = gm;
    h->pending_hist_multi = hist_k;
    h->pending_hm = hm;
    h->pending_sm = sm;
    h->pending_scan_mode = scan;
    return NBG_OK;
  }
  if (hist_k && (rc = launch_hist_multi(hm, n_batches, stream))) return rc;
  if (scan == kScanKernel && (rc = launch_scan_multi(sm, n_batches, stream))) return rc;
  return launch_group_multi(gm, n_batches, scan, stream, compact_group(h));
}

}  // namespace

extern "C" {

int nbg_maglev_classify_desc_multi(nbg_maglev* h, const nbg_desc_batch* batches, uint32_t n_batches, uint32_t flags,
                                   void* stream) {
  return desc_multi_common(h, batches, n_batches, flags, nullptr, 0, stream);
}

int nbg_chain_lpm_maglev_multi(nbg_maglev* mg, nbg_lpm* lpm, uint32_t lpm_groups, const nbg_desc_batch* batches,
                               uint32_t n_batches, uint32_t flags, void* stream) {
  if (!lpm) return set_error(NBG_EINVAL, "chain (multi): null lpm handle");
  return desc_multi_common(mg, batches, n_batches, flags & ~NBG_SWAP_MACS, lpm, lpm_groups, stream);
}

int nbg_maglev_classify_device_ex(nbg_maglev* h, uint8_t* d_pkts, const uint32_t* d_off, const uint16_t* d_len,
                                  uint32_t stride, uint16_t fixed_len, uint64_t n_pkts, uint32_t flags,
                                  uint16_t* d_backend, uint32_t* d_perm, uint32_t* d_counts, uint8_t* d_mac_out,
                                  void* stream) {
  return classify_common(h, d_pkts, d_off, d_len, stride, fixed_len, n_pkts, flags, d_backend, d_perm, d_counts,
                         d_mac_out, nullptr, 0, nullptr, stream);
}

int nbg_maglev_classify_device_multi(nbg_maglev* h, const nbg_batch* batches, uint32_t n_batches, uint32_t stride,
                                     uint16_t fixed_len, uint32_t flags, void* stream) {
  if (!h) return set_error(NBG_EINVAL, "classify (multi): null handle");
  if (!batches || n_batches == 0 || n_batches > NBG_MAX_MULTI)
    return set_error(NBG_EINVAL, "classify (multi): 1..%u batches", NBG_MAX_MULTI);
  if (flags & ~(NBG_SWAP_MACS | NBG_DEFER_GROUP))
    return set_error(NBG_EINVAL, "classify (multi): flags other than NBG_SWAP_MACS and NBG_DEFER_GROUP");
  if (h->ring) return set_error(NBG_EBUSY, "classify (multi): the handle's persistent ring is running");
  if (h->pending_lag) {  // a pending lagged group is launched alone first
    const int rc = nbg_maglev_finish_group(h, stream);
    if (rc) return rc;
  }
  if (h->pending) return set_error(NBG_EINVAL, "classify (multi): a deferred group is pending (nbg_maglev_finish_group)");
  const bool group = batches[0].d_perm || batches[0].d_counts;
  uint64_t total = 0, max_n = 0;
  bool lean = stride >= 64 && stride % 16 == 0 && fixed_len >= 48 && stride < (1u << 24);
  for (uint32_t j = 0; j < n_batches; ++j) {
    const nbg_batch& x = batches[j];
    if ((x.d_perm || x.d_counts) != group)
      return set_error(NBG_EINVAL, "classify (multi): batch %u: every batch or none has perm/counts", j);
    if (x.n_pkts >= (1ull << 30)) return set_error(NBG_EINVAL, "classify (multi): batch %u: n_pkts must be < 2^30", j);
    if (x.n_pkts && (!x.d_pkts || !x.d_backend))
      return set_error(NBG_EINVAL, "classify (multi): batch %u: null packet or backend buffer", j);
    if ((x.d_mac_out != nullptr) != (batches[0].d_mac_out != nullptr))
      return set_error(NBG_EINVAL, "classify (multi): batch %u: every batch or none has d_mac_out", j);
    if (x.n_pkts == 0 || (reinterpret_cast<uintptr_t>(x.d_pkts) & 15u)) lean = false;
    total += x.n_pkts;
    max_n = std::max<uint64_t>(max_n, x.n_pkts);
  }
  const uint32_t nbins = h->nb + 1;
  const uint64_t per = (max_n + kChunk * kMaxParts - 1) / (kChunk * kMaxParts);
  const uint32_t part_pkts = static_cast<uint32_t>(std::max<uint64_t>(per, 1) * kChunk);
  const uint32_t n_parts_max = static_cast<uint32_t>((max_n + part_pkts - 1) / part_pkts);
  const int scan = group ? pick_group_scan(nbins, n_parts_max) : kScanDirect;
  // NBG_MULTI_HIST_KERNEL=1 (measurement): partition rows from one hist_kernel launch beside the group
  // launch instead of the classify kernel's per-unit flush (whose block barriers the ring kernel,
  // the faster in-place path, does not have)
  static const bool multi_hist_k = [] {
    const char* e = std::getenv("NBG_MULTI_HIST_KERNEL");
    return e && std::atoi(e) == 1;
  }();
  const bool hist_k = group && multi_hist_k;
  const bool fused = lean && !h->wide && h->m <= 65537 && total >= 262144 && nbins <= 256 && use_stream(h, total) &&
                     (!group || ((hist_k || hist_in_classify(nbins)) && scan != kScanKernel));
  if (!fused && (flags & NBG_DEFER_GROUP)) {
    if (device_ring_running(h->device))
      return set_error(NBG_EINVAL, "classify (multi): NBG_DEFER_GROUP needs the streaming kernel, which cannot run while "
                       "a persistent ring runs on device %d (stop it, or call without NBG_DEFER_GROUP)", h->device);
    return set_error(NBG_EINVAL, "classify (multi): NBG_DEFER_GROUP needs the fused path (fixed 64-B slots, >= 262144 "
                     "packets in all, <= 255 backends)");
  }
  if (!fused) {
    // one batch after another on the same stream (same results, one launch sequence each)
    for (uint32_t j = 0; j < n_batches; ++j) {
      const nbg_batch& x = batches[j];
      const int rc = classify_common(h, x.d_pkts, nullptr, nullptr, stride, fixed_len, x.n_pkts, flags, x.d_backend,
                                     x.d_perm, x.d_counts, x.d_mac_out, nullptr, 0, nullptr, stream);
      if (rc) return rc;
    }
    return NBG_OK;
  }
  DeviceGuard g(h->device);
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  NBG_HIP(hipStreamIsCapturing(static_cast<hipStream_t>(stream), &cap));
  if (cap != hipStreamCaptureStatusNone)
    return set_error(NBG_EINVAL, "classify (multi): multi-launch batches cannot be captured in a graph");
  const size_t set_words = static_cast<size_t>(kMaxMulti) * kMaxParts * nbins;
  if (group && !h->d_part_multi) {
    NBG_HIP(hipMalloc(&h->d_part_multi, 2 * set_words * sizeof(uint32_t)));
    SetupStream st;
    (void)st.zero(h->d_part_multi, 2 * set_words * sizeof(uint32_t));
    NBG_HIP(st.finish());
  }
  int rc = order_after_last(h, static_cast<hipStream_t>(stream));
  if (rc) return rc;
  uint32_t* set_cur = group ? h->d_part_multi + static_cast<size_t>(h->mparity) * set_words : nullptr;
  uint32_t* set_next = group ? h->d_part_multi + static_cast<size_t>(h->mparity ^ 1u) * set_words : nullptr;
  ClassifyArgs a{};
  a.stride = stride;
  a.fixed_len = fixed_len;
  a.lut = h->d_lut;
  a.m = static_cast<uint32_t>(h->m);
  a.mu = ~0ull / h->m + ((~0ull % h->m) + 1 == h->m ? 1 : 0);
  a.nb = h->nb;
  a.swap = (flags & NBG_SWAP_MACS) ? 1u : 0u;
  a.win_owned = 1u;
  a.wb_full = 1u;
  a.lean = 1u;
  a.lut_lds_bytes = std::min<uint32_t>(h->lut_alloc, 65536u);
  a.lut_tail = h->m > 65536 ? h->lut_host[65536] : 0u;
  a.part_pkts = part_pkts;
  a.hist16 = group && !hist_k && scan == kScanDirect && part_pkts < 65536 ? 1u : 0u;
  StreamBatches sb{};
  GroupMulti gm{};
  HistMulti hm{};
  uint32_t units = 0;
  for (uint32_t j = 0; j < n_batches; ++j) {
    const nbg_batch& x = batches[j];
    sb.pkts[j] = x.d_pkts;
    sb.backend[j] = x.d_backend;
    sb.mac_out[j] = x.d_mac_out;
    uint32_t* rows = group ? set_cur + static_cast<size_t>(j) * kMaxParts * nbins : nullptr;
    sb.part_hist[j] = hist_k ? nullptr : rows;
    sb.n_pkts[j] = static_cast<uint32_t>(x.n_pkts);
    sb.unit_base[j] = units;
    units += static_cast<uint32_t>((((x.n_pkts + 63) >> 6) + stream_waves_per_block() - 1) / stream_waves_per_block());
    GroupArgs& ga = gm.g[j];
    ga.backend = x.d_backend;
    ga.n_pkts = static_cast<uint32_t>(x.n_pkts);
    ga.nb = h->nb;
    uint32_t bits = 0;
    while ((1u << bits) < nbins) ++bits;
    ga.bits = bits;
    ga.n_parts = static_cast<uint32_t>((x.n_pkts + part_pkts - 1) / part_pkts);
    ga.part_pkts = part_pkts;
    ga.part_hist = rows;
    ga.hist16 = a.hist16;
    // zeroed for the next call even when this call's rows come from hist_kernel (stored whole): the
    // next call may accumulate into them (the classify kernel's flush)
    ga.part_hist_next = hist_in_classify(nbins) ? set_next : nullptr;
    ga.next_words = hist_in_classify(nbins) ? static_cast<uint32_t>(set_words) : 0u;
    ga.counts = x.d_counts ? x.d_counts : h->d_counts;
    ga.perm = x.d_perm;
    HistArgs& ha = hm.h[j];
    ha.backend = x.d_backend;
    ha.n_pkts = ga.n_pkts;
    ha.nb = h->nb;
    ha.part_pkts = part_pkts;
    ha.n_parts = ga.n_parts;
    ha.part_hist = rows;
  }
  hm.per = n_parts_max;
  sb.unit_base[n_batches] = units;
  sb.n = n_batches;
  a.mac_out = sb.mac_out[0];  // selects the records mode; per-batch pointers come from sb
  a.part_hist = sb.part_hist[0];
  a.pkts = sb.pkts[0];
  a.n_pkts = sb.n_pkts[0];
  a.backend = sb.backend[0];
  h->last_stream = static_cast<hipStream_t>(stream);
  h->issued = true;
  if ((rc = launch_classify_stream_multi(a, sb, stream_grid(h), stream))) return rc;
  if (group) {
    h->mparity ^= 1u;
    gm.per = n_parts_max;
    if (flags & NBG_DEFER_GROUP) {
      h->pending = true;
      h->pending_multi = n_batches;
      h->pending_gm = gm;
      h->pending_hist_multi = hist_k;
      h->pending_hm = hm;
      h->pending_scan_mode = scan;
      return NBG_OK;
    }
    if (hist_k && (rc = launch_hist_multi(hm, n_batches, stream))) return rc;
    if ((rc = launch_group_multi(gm, n_batches, scan, stream, compact_group(h)))) return rc;
  }
  return NBG_OK;
}

int nbg_chain_lpm_maglev_device(nbg_maglev* mg, nbg_lpm* lpm, uint32_t lpm_groups, uint8_t* d_pkts,
                                const uint32_t* d_off, const uint16_t* d_len, uint32_t stride, uint16_t fixed_len,
                                uint64_t n_pkts, uint32_t flags, uint16_t* d_gate, uint16_t* d_backend,
                                uint32_t* d_perm, uint32_t* d_counts, void* stream) {
  if (!lpm) return set_error(NBG_EINVAL, "chain: null lpm handle");
  return classify_common(mg, d_pkts, d_off, d_len, stride, fixed_len, n_pkts, flags & ~NBG_SWAP_MACS, d_backend,
                         d_perm, d_counts, nullptr, lpm, lpm_groups, d_gate, stream);
}

int nbg_lpm_create(const uint32_t* prefixes, const uint8_t* lens, const uint16_t* gates, uint64_t n, int device,
                   nbg_lpm** out) {
  if (!out || ((!prefixes || !lens || !gates) && n)) return set_error(NBG_EINVAL, "nbg_lpm_create: null argument");
  *out = nullptr;
  int ndev = 0;
  const hipError_t ce = hipGetDeviceCount(&ndev);
  if (ce != hipSuccess || ndev <= 0)
    return set_error(NBG_ENODEV, "no HIP device available (the LPM path has no CPU fallback): %s, %d devices",
                     hipGetErrorString(ce), ndev);
  if (device < 0 || device >= ndev) return set_error(NBG_ENODEV, "device %d out of range (%d devices)", device, ndev);
  std::vector<uint16_t> t24, tl;
  uint64_t used = 0;
  int rc = build_lpm(prefixes, lens, gates, n, t24, tl, used);
  if (rc) return rc;
  nbg_lpm* t = new (std::nothrow) nbg_lpm();
  if (!t) return set_error(NBG_ENOMEM, "out of host memory");
  t->device = device;
  t->long_used = used;
  DeviceGuard g(device);
  const uint64_t nl = used ? used : 1;
  SetupStream st;
  if (hipMalloc(&t->d_tbl24, t24.size() * 2) != hipSuccess || hipMalloc(&t->d_tbl_long, nl * 2) != hipSuccess ||
      st.h2d(t->d_tbl24, t24.data(), t24.size() * 2) != hipSuccess ||
      st.h2d(t->d_tbl_long, tl.data(), nl * 2) != hipSuccess || st.finish() != hipSuccess) {
    nbg_lpm_destroy(t);
    return set_error(NBG_ENOMEM, "nbg_lpm_create: device allocation/upload failed");
  }
  *out = t;
  return NBG_OK;
}

void nbg_lpm_destroy(nbg_lpm* t) {
  if (!t) return;
  {
    DeviceGuard g(t->device);
    (void)hipFree(t->d_tbl24);
    (void)hipFree(t->d_tbl_long);
  }
  delete t;
}

int nbg_lpm_lookup_device(nbg_lpm* t, const uint32_t* d_ips, uint64_t n, uint16_t* d_gate, void* stream) {
  if (!t) return set_error(NBG_EINVAL, "lpm lookup: null handle");
  if (n == 0) return NBG_OK;
  if (!d_ips || !d_gate) return set_error(NBG_EINVAL, "lpm lookup: null buffer");
  if (n >= (1ull << 32)) return set_error(NBG_EINVAL, "lpm lookup: n must be < 2^32");
  DeviceGuard g(t->device);
  return launch_lpm_lookup(t->d_tbl24, t->d_tbl_long, d_ips, n, d_gate, stream);
}

int nbg_maglev_finish_group(nbg_maglev* h, void* stream) {
  if (!h) return set_error(NBG_EINVAL, "finish_group: null handle");
  if (!h->pending) return NBG_OK;
  DeviceGuard g(h->device);
  int rc = order_after_last(h, static_cast<hipStream_t>(stream));  // after the classify, on any stream
  if (rc) return rc;
  h->last_stream = static_cast<hipStream_t>(stream);
  if (h->pending_lag) return flush_lag(h, static_cast<hipStream_t>(stream));
  h->pending = false;
  if (h->pending_multi) {
    // fixed slots (nbg_maglev_classify_device_multi): partition rows from the classify kernel and the
    // direct scan, one group launch; descriptor batches with many backends
    // (nbg_maglev_classify_desc_multi) also a hist and a scan launch, each over all batches
    const uint32_t n = h->pending_multi;
    h->pending_multi = 0;
    if (h->pending_hist_multi && (rc = launch_hist_multi(h->pending_hm, n, stream))) return rc;
    if (h->pending_scan_mode == kScanKernel && (rc = launch_scan_multi(h->pending_sm, n, stream))) return rc;
    return launch_group_multi(h->pending_gm, n, h->pending_scan_mode, stream, compact_group(h));
  }
  if (h->pending_hist && (rc = launch_hist(h->pending_hist_args, stream))) return rc;
  if (h->pending_scan_mode == kScanKernel && (rc = launch_scan(h->pending_scan, stream))) return rc;
  if ((rc = h->pending_wide ? launch_group_wide(h->pending_args, stream)
                            : launch_group(h->pending_args, h->pending_scan_mode, stream, compact_group(h))))
    return rc;
  return NBG_OK;
}

int nbg_maglev_check(nbg_maglev* h) {
  if (!h) return set_error(NBG_EINVAL, "check: null handle");
  DeviceGuard g(h->device);
  if (!h->issued) return NBG_OK;
  NBG_HIP(hipStreamSynchronize(h->last_stream));
  NBG_HIP(hipGetLastError());
  return NBG_OK;
}

// ---- persistent RX ring (nbg_ring_*) ---------------------------------------------------------------
}  // extern "C"

// An RX queue's view of the device's ring: its own tickets over the ring's shared sequence.
struct nbg_ring_queue {
  nbg_ring* r = nullptr;
  uint64_t posted = 0, done = 0;        // this queue's batches posted / complete
  uint64_t gidx[NBG_RING_SLOTS] = {};   // the ring ticket of this queue's ticket t, at t % NBG_RING_SLOTS
  bool closed = false;                  // closed by nbg_ring_stop: calls fail, nbg_ring_queue_close frees it
};

struct nbg_ring {
  nbg_maglev* h = nullptr;             // the owning handle (never touched once `leaked`)
  int device = 0;                      // copies of the handle's device and backend count
  uint32_t nb = 0;
  std::mutex mu;                       // posts, completion, queues, grouping: several producer threads
  // calls that release and retake `mu` while they wait (post, wait): nbg_ring_stop lets them leave
  // (the ended kernel makes each return) before it closes the queues or frees anything
  uint32_t calls = 0;
  bool leaked = false;                 // the kernel did not end at stop: every call returns NBG_EBUSY
  bool stopping = false;               // nbg_ring_stop has begun: posts are refused
  bool stopped = false;                // nbg_ring_stop has finished: a repeat stop returns stop_rc, touching nothing
  int stop_rc = NBG_OK;
  hipStream_t stream = nullptr;        // the ring kernel's (private, highest priority)
  hipEvent_t ev_start = nullptr, ev_end = nullptr;  // around the kernel on `stream` (its duration)
  size_t hbytes = 0, dbytes = 0;       // the pinned host ring and the uncached device ring
  uint8_t* host = nullptr;             // pinned, mapped: RingCtl | RingDesc[slots]
  uint8_t* dev = nullptr;              // uncached HBM: stop | completion | exits (a line each) | prog[grid] | RingDesc[reps][slots]
  volatile RingCtl* ctl = nullptr;
  RingDesc* desc = nullptr;
  uint32_t slots = NBG_RING_SLOTS;
  uint32_t reps = kRingReps;
  int grid = 0;
  uint32_t idle_ms = 0;
  uint64_t posted = 0, units = 0, completed = 0;
  // per slot, the batch posted there last (nbg_ring_group groups it from its backend[])
  std::vector<std::pair<uint16_t*, uint64_t>> rec;
  // nbg_ring_group's scratch, one set per side stream (up to kGroupSets streams group concurrently;
  // a further stream takes over the least recently used set after that set's stream's work).  A set
  // is owned through `claimed`, not through the stream value: the null stream is a stream too.
  struct GroupSet {
    bool claimed = false;
    hipStream_t s = nullptr;       // the owning stream (nullptr: the null stream)
    uint64_t used = 0;             // last use (call count)
    uint32_t* rows = nullptr;      // partition histograms [kMaxMulti][kMaxParts][nb+1] (a burst: one set per batch)
    uint32_t* prefix = nullptr;    // per-partition prefixes (scan-kernel path)
    uint32_t* totals = nullptr;    // totals [nb+1]
  };
  static constexpr int kGroupSets = 4;
  GroupSet gsets[kGroupSets];
  uint64_t gcalls = 0;
  std::vector<nbg_ring_queue*> queues;  // open RX queues (closed by nbg_ring_stop)
  std::vector<nbg_ring_queue*> closed;  // queues nbg_ring_stop closed: freed by nbg_ring_queue_close or with the ring
  bool ended = false;  // the kernel has ended (stop, idle timeout, or a fault)
  // hipStreamQuery is not cheap on a stream with a resident kernel, so the kernel's end is only
  // checked after the completed count has not moved for kStallCheck
  std::chrono::steady_clock::time_point moved{};
};

namespace {

using Clock = std::chrono::steady_clock;

// The uncached device buffer: the stop word, the completion word and the exit count on lines of
// their own, then the blocks' progress words, then the descriptor replicas.
constexpr size_t kDevStop = 0, kDevComp = 64, kDevExit = 128, kDevProg = 192;
size_t ring_desc_off(int grid) { return kDevProg + ((static_cast<size_t>(grid) * 4u + 63u) & ~size_t{63}); }

// Completed batches: the relay reports the minimum over the blocks' counts (mod 2^32, so taken as
// a lag behind `posted`).  Under r->mu.
void ring_refresh(nbg_ring* r) {
  const uint32_t lag = static_cast<uint32_t>(r->posted) - r->ctl->completed;
  const uint64_t c = lag <= r->posted - r->completed ? r->posted - lag : r->completed;
  if (c != r->completed) r->moved = Clock::now();
  r->completed = c;
}

// A queue's completed tickets: its batches complete in ring order.  Under r->mu.
void queue_refresh(nbg_ring_queue* q) {
  while (q->done < q->posted && q->gidx[q->done % NBG_RING_SLOTS] < q->r->completed) ++q->done;
}

constexpr auto kStallCheck = std::chrono::milliseconds(2);

// The kernel has ended?  (hipStreamQuery: the ring kernel is the last work on its stream.)  An ended
// ring no longer holds the device: other handles' calls take the LDS-hungry kernels again and a new
// ring may start, before this one's nbg_ring_stop.  Under r->mu.
bool ring_ended(nbg_ring* r) {
  if (!r->ended && hipStreamQuery(r->stream) != hipErrorNotReady) {
    r->ended = true;
    std::lock_guard<std::mutex> dg(g_dev_ring_mu);
    if (static_cast<size_t>(r->device) < g_dev_ring.size() && g_dev_ring[r->device] == r) g_dev_ring[r->device] = nullptr;
  }
  return r->ended;
}

// The same, but the stream is only queried once the completed count has stalled for kStallCheck
// with batches outstanding (the idle kernel's own exit, stop, or a fault); the error word is free.
bool ring_gone(nbg_ring* r) {
  if (r->ended || r->ctl->error) return true;
  if (r->completed >= r->posted) return false;
  if (Clock::now() - r->moved < kStallCheck) return false;
  return ring_ended(r);
}

int ring_state_error(nbg_ring* r) {
  if (r->ctl->error) return set_error(NBG_ETIMEDOUT, "ring: the kernel ended after %u ms without a post", r->idle_ms);
  return set_error(NBG_EIO, "ring: the kernel has ended (%s)", hipGetErrorString(hipStreamQuery(r->stream)));
}

void ring_pause(Clock::time_point t0) {
  if (Clock::now() - t0 > std::chrono::microseconds(200)) std::this_thread::sleep_for(std::chrono::microseconds(20));
}

// Stop: the open queues become closed ones (their producers may still hold them).  Under r->mu.
void ring_close_queues(nbg_ring* r) {
  for (auto* q : r->queues) {
    q->closed = true;
    r->closed.push_back(q);
  }
  r->queues.clear();
}

// A call that waits on the ring, counted in r->calls for its whole duration.  Under r->mu.
struct RingCall {
  nbg_ring* r;
  explicit RingCall(nbg_ring* r_) : r(r_) {
    std::lock_guard<std::mutex> g(r->mu);
    ++r->calls;
  }
  ~RingCall() {
    std::lock_guard<std::mutex> g(r->mu);
    --r->calls;
  }
};

int ring_leaked_error() {
  return set_error(NBG_EBUSY, "ring: its kernel did not end at nbg_ring_stop (leaked; the device stays busy)");
}

// Wait for the grouping streams' work on the scratch sets and release them.
void ring_release_sets(nbg_ring* r) {
  for (auto& g : r->gsets) {
    if (g.claimed) (void)hipStreamSynchronize(g.s);
    g.claimed = false;
    g.s = nullptr;
    g.used = 0;
  }
  r->gcalls = 0;
}

void ring_free(nbg_ring* r) {
  ring_release_sets(r);  // their kernels use the scratch below
  for (auto& g : r->gsets) {
    (void)hipFree(g.rows);
    (void)hipFree(g.prefix);
    (void)hipFree(g.totals);
  }
  for (auto* q : r->queues) delete q;
  for (auto* q : r->closed) delete q;
  r->queues.clear();
  r->closed.clear();
  if (r->host) (void)hipHostFree(r->host);
  if (r->dev) (void)hipFree(r->dev);
  if (r->stream) (void)hipStreamDestroy(r->stream);
  if (r->ev_start) (void)hipEventDestroy(r->ev_start);
  if (r->ev_end) (void)hipEventDestroy(r->ev_end);
  delete r;
}

// The ring's buffers, private stream and events (nbg_ring_start keeps them across stops).
int ring_alloc(nbg_maglev* h, nbg_ring** out) {
  auto* r = new (std::nothrow) nbg_ring;
  if (!r) return set_error(NBG_ENOMEM, "ring_start: out of memory");
  r->h = h;
  r->device = h->device;
  r->nb = h->nb;
  r->grid = h->cus - 1;  // classify blocks; one more block, on a CU of its own, is the relay
  if (const char* e = std::getenv("NBG_RING_REPS")) {  // measurement: replicas, a power of two <= 256
    const uint32_t v = static_cast<uint32_t>(std::atoi(e));
    if (v && v <= 256 && (v & (v - 1)) == 0) r->reps = v;
  }
  // The kernel runs on a private stream of the highest priority: HIP maps streams onto at most
  // GPU_MAX_HW_QUEUES hardware queues per priority, and work on any stream that shared the ring's
  // queue would wait behind the resident kernel (measured: a third grouping stream did, until the
  // ring's idle exit).
  int least = 0, greatest = 0;
  (void)hipDeviceGetStreamPriorityRange(&least, &greatest);
  if (hipStreamCreateWithPriority(&r->stream, hipStreamNonBlocking, greatest) != hipSuccess) {
    r->stream = nullptr;
    ring_free(r);
    return set_error(NBG_EIO, "ring_start: private stream");
  }
  if (hipEventCreate(&r->ev_start) != hipSuccess || hipEventCreate(&r->ev_end) != hipSuccess) {
    ring_free(r);
    return set_error(NBG_EIO, "ring_start: events");
  }
  r->hbytes = sizeof(RingCtl) + static_cast<size_t>(r->slots) * sizeof(RingDesc);
  r->dbytes = ring_desc_off(r->grid) + static_cast<size_t>(r->reps) * r->slots * sizeof(RingDesc);
  if (hipHostMalloc(reinterpret_cast<void**>(&r->host), r->hbytes, hipHostMallocMapped | hipHostMallocCoherent) !=
      hipSuccess) {
    r->host = nullptr;
    ring_free(r);
    return set_error(NBG_ENOMEM, "ring_start: pinned ring of %zu B", r->hbytes);
  }
  r->ctl = reinterpret_cast<RingCtl*>(r->host);
  r->desc = reinterpret_cast<RingDesc*>(r->host + sizeof(RingCtl));
  if (hipExtMallocWithFlags(reinterpret_cast<void**>(&r->dev), r->dbytes, hipDeviceMallocUncached) != hipSuccess) {
    r->dev = nullptr;
    ring_free(r);
    return set_error(NBG_ENOMEM, "ring_start: uncached device ring of %zu B", r->dbytes);
  }
  const size_t nbins = static_cast<size_t>(h->nb) + 1;
  for (auto& g : r->gsets)
    if (hipMalloc(&g.rows, kMaxMulti * kMaxParts * nbins * 4) != hipSuccess ||
        hipMalloc(&g.prefix, kMaxParts * nbins * 4) != hipSuccess || hipMalloc(&g.totals, nbins * 4) != hipSuccess) {
      ring_free(r);
      return set_error(NBG_ENOMEM, "ring_start: grouping scratch");
    }
  *out = r;
  return NBG_OK;
}

int ring_check_batch(uint8_t* d_pkts, uint64_t n_pkts, uint16_t* d_backend) {
  if (n_pkts >= (1ull << 30)) return set_error(NBG_EINVAL, "ring_post: n_pkts must be < 2^30");
  if (n_pkts && (!d_pkts || !d_backend || (reinterpret_cast<uintptr_t>(d_pkts) & 15u) ||
                 (reinterpret_cast<uintptr_t>(d_backend) & 15u)))
    return set_error(NBG_EINVAL, "ring_post: packet and backend buffers must be 16-B aligned");
  return NBG_OK;
}

// Write batch `posted` into its host slot (the caller found the slot free) and return its ring
// ticket.  Under r->mu.
uint64_t ring_put(nbg_ring* r, uint8_t* d_pkts, uint64_t n_pkts, uint16_t* d_backend) {
  const uint64_t j = r->posted;
  if (r->completed == j) r->moved = Clock::now();  // the stall clock starts with the first outstanding batch
  const uint64_t units = ((n_pkts + 63) / 64 + 7) / 8;  // 512-packet units of 8 waves' tiles
  RingDesc d{};
  d.pkts = reinterpret_cast<uintptr_t>(d_pkts);
  d.backend = reinterpret_cast<uintptr_t>(d_backend);
  d.ulo = r->units;
  d.uhi = r->units + units;
  d.n_pkts = static_cast<uint32_t>(n_pkts);
  d.seq = static_cast<uint32_t>(j + 1);
  d.check = ring_check(d.pkts, d.backend, d.ulo, d.uhi, d.n_pkts, d.seq);
  // one 64-B line: a relay read that overlaps this write fails the check and is retried
  volatile uint64_t* dst = reinterpret_cast<volatile uint64_t*>(r->desc + (j & (r->slots - 1)));
  const uint64_t* src = reinterpret_cast<const uint64_t*>(&d);
  for (int i = 0; i < 8; ++i) dst[i] = src[i];
  std::atomic_thread_fence(std::memory_order_release);
  r->rec[j & (r->slots - 1)] = {d_backend, n_pkts};
  r->posted = j + 1;
  r->units += units;
  return j;
}

// One batch into the ring, waiting for a free slot (the batch NBG_RING_SLOTS back complete); with a
// queue, *ticket is the queue's ticket.  The ring's mutex is held only while the state is touched.
int ring_post_one(nbg_ring* r, nbg_ring_queue* q, uint8_t* d_pkts, uint64_t n_pkts, uint16_t* d_backend,
                  uint64_t* ticket) {
  int rc = ring_check_batch(d_pkts, n_pkts, d_backend);
  if (rc) return rc;
  const auto t0 = Clock::now();
  RingCall call(r);
  for (;;) {
    {
      std::lock_guard<std::mutex> g(r->mu);
      if (r->leaked) return ring_leaked_error();
      if (q && q->closed) return set_error(NBG_EINVAL, "ring_queue_post: the queue was closed by nbg_ring_stop");
      if (r->stopping) return set_error(NBG_EINVAL, "ring_post: the ring is stopping");
      ring_refresh(r);
      if (ring_gone(r)) return ring_state_error(r);
      if (r->posted - r->completed < r->slots) {
        const uint64_t gt = ring_put(r, d_pkts, n_pkts, d_backend);
        if (q) {
          queue_refresh(q);  // frees the entry of the queue's ticket NBG_RING_SLOTS back (complete by now)
          q->gidx[q->posted % NBG_RING_SLOTS] = gt;
          *ticket = q->posted++;
        } else {
          *ticket = gt;
        }
        return NBG_OK;
      }
    }
    if (Clock::now() - t0 > std::chrono::milliseconds(r->idle_ms + 1000u))
      return set_error(NBG_ETIMEDOUT, "ring_post: no slot freed in %u ms", r->idle_ms + 1000u);
    ring_pause(t0);
  }
}

// Stream s's scratch set; a stream without one takes a free set, or the least recently used one
// after everything its previous stream has issued so far.  Under r->mu.
int ring_gset(nbg_ring* r, hipStream_t s, nbg_ring::GroupSet** out) {
  nbg_ring::GroupSet* gs = nullptr;
  for (auto& x : r->gsets)
    if (x.claimed && x.s == s) gs = &x;
  if (!gs) {
    for (auto& x : r->gsets)
      if (!x.claimed) {
        gs = &x;
        break;
      }
    if (!gs) {
      gs = &r->gsets[0];
      for (auto& x : r->gsets)
        if (x.used < gs->used) gs = &x;
      hipEvent_t ev = nullptr;
      NBG_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      const hipError_t e1 = hipEventRecord(ev, gs->s), e2 = hipStreamWaitEvent(s, ev, 0);
      (void)hipEventDestroy(ev);
      if (e1 != hipSuccess || e2 != hipSuccess) return set_error(NBG_EIO, "ring_group: stream order");
    }
    gs->claimed = true;
    gs->s = s;
  }
  gs->used = ++r->gcalls;
  *out = gs;
  return NBG_OK;
}

// The grouping of ring ticket `ticket` on stream s (gated on its completion when not complete yet).
// Under r->mu.
int ring_group_locked(nbg_ring* r, uint64_t ticket, uint32_t* d_perm, uint32_t* d_counts, hipStream_t s) {
  if (ticket >= r->posted)
    return set_error(NBG_EINVAL, "ring_group: ticket %llu was not posted", (unsigned long long)ticket);
  if (r->posted - ticket > r->slots)
    return set_error(NBG_EINVAL, "ring_group: ticket %llu is older than the ring's %u slots", (unsigned long long)ticket,
                     r->slots);
  ring_refresh(r);
  DeviceGuard g(r->device);
  const auto [backend, n_pkts] = r->rec[ticket & (r->slots - 1)];
  const uint32_t nbins = r->nb + 1;
  nbg_ring::GroupSet* gs = nullptr;
  int rc = ring_gset(r, s, &gs);
  if (rc) return rc;
  if (n_pkts == 0) {
    NBG_HIP(hipMemsetAsync(d_counts, 0, nbins * 4, s));
    return NBG_OK;
  }
  if (ticket >= r->completed) {  // not complete yet: the stream waits for it on the device
    const uint32_t* dcomp = reinterpret_cast<const uint32_t*>(r->dev + kDevComp);
    const uint32_t* dexit = reinterpret_cast<const uint32_t*>(r->dev + kDevExit);
    if ((rc = launch_ring_gate(dcomp, dexit, static_cast<uint32_t>(ticket + 1), static_cast<uint32_t>(r->grid), s)))
      return rc;
  }
  const uint64_t per = (n_pkts + kChunk * kMaxParts - 1) / (kChunk * kMaxParts);
  const uint32_t part_pkts = static_cast<uint32_t>(per * kChunk);
  const uint32_t n_parts = static_cast<uint32_t>((n_pkts + part_pkts - 1) / part_pkts);
  HistArgs ha{};
  ha.backend = backend;
  ha.n_pkts = static_cast<uint32_t>(n_pkts);
  ha.nb = r->nb;
  ha.part_pkts = part_pkts;
  ha.n_parts = n_parts;
  ha.part_hist = gs->rows;
  const int scan = pick_group_scan(nbins, n_parts);
  ha.hist16 = scan == kScanDirect && part_pkts < 65536 ? 1u : 0u;  // packed rows for the direct prefix
  if ((rc = launch_hist(ha, s))) return rc;
  if (scan == kScanKernel) {
    ScanArgs sa{};
    sa.part_hist = gs->rows;
    sa.part_prefix = gs->prefix;
    sa.totals = gs->totals;
    sa.n_parts = n_parts;
    sa.nbins = nbins;
    if ((rc = launch_scan(sa, s))) return rc;
  }
  GroupArgs ga{};
  ga.backend = backend;
  ga.n_pkts = static_cast<uint32_t>(n_pkts);
  ga.nb = r->nb;
  uint32_t bits = 0;
  while ((1u << bits) < nbins) ++bits;
  ga.bits = bits;
  ga.n_parts = n_parts;
  ga.part_pkts = part_pkts;
  ga.part_hist = gs->rows;
  ga.part_prefix = gs->prefix;
  ga.totals = gs->totals;
  ga.hist16 = ha.hist16;
  ga.counts = d_counts;
  ga.perm = d_perm;
  return launch_group(ga, scan, s, group_compact(nbins, true));
}

// Batches first .. first + n - 1 grouped by one gate, one hist and one group launch on s (a
// producer's burst: launches per batch would cost more host time than a shard-size batch takes on
// the device).  Falls back to one grouping per batch where the multi-batch launches do not apply
// (an empty batch, grouping through the scan kernel).  Under r->mu.
int ring_group_burst_locked(nbg_ring* r, uint64_t first, uint32_t n, uint32_t* const* d_perm,
                            uint32_t* const* d_counts, hipStream_t s) {
  if (n == 0 || n > kMaxMulti) return set_error(NBG_EINVAL, "ring_group_burst: 1..%u batches", kMaxMulti);
  const uint64_t last = first + n - 1;
  if (last >= r->posted)
    return set_error(NBG_EINVAL, "ring_group_burst: ticket %llu was not posted", (unsigned long long)last);
  if (r->posted - first > r->slots)
    return set_error(NBG_EINVAL, "ring_group_burst: ticket %llu is older than the ring's %u slots",
                     (unsigned long long)first, r->slots);
  for (uint32_t j = 0; j < n; ++j)
    if (!d_perm[j] || !d_counts[j]) return set_error(NBG_EINVAL, "ring_group_burst: null output of batch %u", j);
  const uint32_t nbins = r->nb + 1;
  uint64_t max_n = 0;
  bool empty = false;
  for (uint32_t j = 0; j < n; ++j) {
    const uint64_t m = r->rec[(first + j) & (r->slots - 1)].second;
    max_n = std::max(max_n, m);
    empty = empty || m == 0;
  }
  const uint64_t per = (max_n + kChunk * kMaxParts - 1) / (kChunk * kMaxParts);
  const uint32_t part_pkts = static_cast<uint32_t>(std::max<uint64_t>(per, 1) * kChunk);
  const uint32_t n_parts_max = static_cast<uint32_t>((max_n + part_pkts - 1) / part_pkts);
  const int scan = pick_group_scan(nbins, n_parts_max);
  if (empty || scan == kScanKernel || n == 1) {
    for (uint32_t j = 0; j < n; ++j) {
      const int rc = ring_group_locked(r, first + j, d_perm[j], d_counts[j], s);
      if (rc) return rc;
    }
    return NBG_OK;
  }
  ring_refresh(r);
  DeviceGuard g(r->device);
  nbg_ring::GroupSet* gs = nullptr;
  int rc = ring_gset(r, s, &gs);
  if (rc) return rc;
  if (last >= r->completed) {  // batches complete in ring order: waiting for the last covers all
    const uint32_t* dcomp = reinterpret_cast<const uint32_t*>(r->dev + kDevComp);
    const uint32_t* dexit = reinterpret_cast<const uint32_t*>(r->dev + kDevExit);
    if ((rc = launch_ring_gate(dcomp, dexit, static_cast<uint32_t>(last + 1), static_cast<uint32_t>(r->grid), s)))
      return rc;
  }
  HistMulti hm{};
  GroupMulti gm{};
  uint32_t bits = 0;
  while ((1u << bits) < nbins) ++bits;
  for (uint32_t j = 0; j < n; ++j) {
    const auto [backend, n_pkts] = r->rec[(first + j) & (r->slots - 1)];
    uint32_t* rows = gs->rows + static_cast<size_t>(j) * kMaxParts * nbins;
    HistArgs& ha = hm.h[j];
    ha.backend = backend;
    ha.n_pkts = static_cast<uint32_t>(n_pkts);
    ha.nb = r->nb;
    ha.part_pkts = part_pkts;
    ha.n_parts = static_cast<uint32_t>((n_pkts + part_pkts - 1) / part_pkts);
    ha.part_hist = rows;
    ha.hist16 = part_pkts < 65536 ? 1u : 0u;  // the direct prefix (scan == kScanDirect here)
    GroupArgs& ga = gm.g[j];
    ga.backend = backend;
    ga.n_pkts = static_cast<uint32_t>(n_pkts);
    ga.nb = r->nb;
    ga.bits = bits;
    ga.n_parts = ha.n_parts;
    ga.part_pkts = part_pkts;
    ga.part_hist = rows;
    ga.hist16 = ha.hist16;
    ga.counts = d_counts[j];
    ga.perm = d_perm[j];
  }
  hm.per = n_parts_max;
  gm.per = n_parts_max;
  if ((rc = launch_hist_multi(hm, n, s))) return rc;
  return launch_group_multi(gm, n, scan, s, group_compact(nbins, true));
}

// Wait until `done()` holds, the ring has gone, or timeout_ms (0: none).  `done` runs under r->mu
// after a refresh.
template <typename F>
int ring_wait_for(nbg_ring* r, uint32_t timeout_ms, const char* what, uint64_t ticket, F done) {
  const auto t0 = Clock::now();
  RingCall call(r);
  for (;;) {
    {
      std::lock_guard<std::mutex> g(r->mu);
      if (r->leaked) return ring_leaked_error();
      ring_refresh(r);
      if (done()) return NBG_OK;
      if (ring_gone(r)) {
        ring_refresh(r);  // progress stored before the kernel ended
        if (done()) return NBG_OK;
        return ring_state_error(r);
      }
    }
    if (timeout_ms && Clock::now() - t0 > std::chrono::milliseconds(timeout_ms))
      return set_error(NBG_ETIMEDOUT, "%s: batch %llu not complete after %u ms", what, (unsigned long long)ticket,
                       timeout_ms);
    ring_pause(t0);
  }
}

}  // namespace

extern "C" {

int nbg_ring_start(nbg_maglev* h, uint32_t stride, uint16_t fixed_len, uint32_t flags, uint32_t idle_ms, void* stream,
                   nbg_ring** out) {
  if (!h || !out) return set_error(NBG_EINVAL, "ring_start: null argument");
  *out = nullptr;
  if (h->ring) return set_error(NBG_EBUSY, "ring_start: the handle already runs a ring");
  if (h->wide || h->m > 65537) return set_error(NBG_EINVAL, "ring_start: needs <= 255 backends and M <= 65537");
  if (stride % 16 || stride < 64 || stride >= (1u << 24) || fixed_len < 48)
    return set_error(NBG_EINVAL, "ring_start: fixed slots with stride %% 16 == 0, 64 <= stride < 2^24, fixed_len >= 48");
  if (flags & ~NBG_SWAP_MACS) return set_error(NBG_EINVAL, "ring_start: flags other than NBG_SWAP_MACS");
  if (h->pending) return set_error(NBG_EINVAL, "ring_start: a deferred or lagged group is pending");
  if (h->cus < 2) return set_error(NBG_EINVAL, "ring_start: needs a CU for the relay beside the classify blocks");
  // one ring per GPU: a second one's blocks could never all become resident beside the first
  std::lock_guard<std::mutex> dev_lock(g_dev_ring_mu);
  if (static_cast<size_t>(h->device) < g_dev_hring.size() && g_dev_hring[h->device])
    return set_error(NBG_EBUSY, "ring_start: device %d runs a host-batch server (nbg_host_ring_stop first)", h->device);
  if (static_cast<size_t>(h->device) < g_dev_ring.size() && g_dev_ring[h->device])
    return set_error(NBG_EBUSY,
                     "ring_start: device %d already runs a persistent ring (one per GPU; RX queues share it through "
                     "nbg_ring_queue_open)",
                     h->device);
  DeviceGuard g(h->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  int rc = order_after_last(h, s);  // the ring runs after the handle's earlier work
  if (rc) return rc;
  // a stopped ring's buffers, stream and events are reused (a start then costs a memset and a launch)
  nbg_ring* r = h->ring_spare;
  h->ring_spare = nullptr;
  if (!r && (rc = ring_alloc(h, &r))) return rc;
  r->idle_ms = idle_ms ? idle_ms : 2000u;
  r->moved = Clock::now();
  r->posted = r->units = r->completed = 0;
  r->ended = false;
  r->stopping = false;
  r->stopped = false;
  r->stop_rc = NBG_OK;
  r->rec.assign(r->slots, {nullptr, 0});
  std::memset(r->host, 0, r->hbytes);
  {
    // after everything issued on `stream` so far, in the private stream's order: zero the device
    // ring, then the kernel
    hipEvent_t ev = nullptr;
    const bool ok = hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess &&
                    hipEventRecord(ev, s) == hipSuccess && hipStreamWaitEvent(r->stream, ev, 0) == hipSuccess &&
                    hipMemsetAsync(r->dev, 0, r->dbytes, r->stream) == hipSuccess;
    if (ev) (void)hipEventDestroy(ev);
    if (!ok) {
      ring_free(r);
      return set_error(NBG_EIO, "ring_start: ordering after the caller's stream");
    }
  }
  uint8_t* hdev = nullptr;
  if (hipHostGetDevicePointer(reinterpret_cast<void**>(&hdev), r->host, 0) != hipSuccess) {
    ring_free(r);
    return set_error(NBG_EIO, "ring_start: device address of the pinned ring");
  }
  ClassifyArgs a{};
  a.stride = stride;
  a.fixed_len = fixed_len;
  a.lut = h->d_lut;
  a.m = static_cast<uint32_t>(h->m);
  a.mu = ~0ull / h->m + ((~0ull % h->m) + 1 == h->m ? 1 : 0);  // floor(2^64 / m)
  a.nb = h->nb;
  a.swap = (flags & NBG_SWAP_MACS) ? 1u : 0u;
  a.win_owned = 1;
  a.wb_full = 1;
  a.lean = 1;
  a.lut_lds_bytes = std::min<uint32_t>(h->lut_alloc, 65536u);
  a.lut_tail = h->m > 65536 ? h->lut_host[65536] : 0u;
  RingArgs ra{};
  ra.ctl = reinterpret_cast<RingCtl*>(hdev);
  ra.hdesc = reinterpret_cast<const RingDesc*>(hdev + sizeof(RingCtl));
  ra.dstop = reinterpret_cast<uint32_t*>(r->dev + kDevStop);
  ra.dcomp = reinterpret_cast<uint32_t*>(r->dev + kDevComp);
  ra.dexit = reinterpret_cast<uint32_t*>(r->dev + kDevExit);
  ra.prog = reinterpret_cast<uint32_t*>(r->dev + kDevProg);
  ra.desc = reinterpret_cast<RingDesc*>(r->dev + ring_desc_off(r->grid));
  ra.slots = r->slots;
  ra.reps = r->reps;
  ra.grid = static_cast<uint32_t>(r->grid);
  ra.idle_ticks = static_cast<uint64_t>(r->idle_ms) * 100000u;  // 100 MHz
  (void)hipEventRecord(r->ev_start, r->stream);
  if ((rc = launch_classify_ring(a, ra, a.swap ? 1 : 0, r->grid + 1, r->stream))) {
    ring_free(r);
    return rc;
  }
  (void)hipEventRecord(r->ev_end, r->stream);
  if (static_cast<size_t>(h->device) >= g_dev_ring.size()) g_dev_ring.resize(h->device + 1, nullptr);
  g_dev_ring[h->device] = r;
  h->ring_kernel_ms = -1.f;
  h->ring = r;
  h->last_stream = s;
  h->issued = true;
  *out = r;
  return NBG_OK;
}

int nbg_ring_post_burst(nbg_ring* r, const nbg_ring_batch* batches, uint32_t n_batches, uint32_t* n_posted,
                        uint64_t* first_ticket) {
  if (!r || !n_posted || !first_ticket || (n_batches && !batches))
    return set_error(NBG_EINVAL, "ring_post_burst: null argument");
  *n_posted = 0;
  for (uint32_t i = 0; i < n_batches; ++i) {
    const int rc = ring_check_batch(batches[i].d_pkts, batches[i].n_pkts, batches[i].d_backend);
    if (rc) return rc;
  }
  std::lock_guard<std::mutex> g(r->mu);
  if (r->leaked) return ring_leaked_error();
  if (r->stopping) return set_error(NBG_EINVAL, "ring_post_burst: the ring is stopping");
  *first_ticket = r->posted;
  ring_refresh(r);
  if (ring_gone(r)) return ring_state_error(r);
  const uint64_t room = r->slots - (r->posted - r->completed);
  const uint32_t k = static_cast<uint32_t>(std::min<uint64_t>(room, n_batches));
  for (uint32_t i = 0; i < k; ++i) ring_put(r, batches[i].d_pkts, batches[i].n_pkts, batches[i].d_backend);
  *n_posted = k;
  return NBG_OK;
}

int nbg_ring_post(nbg_ring* r, uint8_t* d_pkts, uint64_t n_pkts, uint16_t* d_backend, uint64_t* ticket) {
  if (!r || !ticket) return set_error(NBG_EINVAL, "ring_post: null argument");
  return ring_post_one(r, nullptr, d_pkts, n_pkts, d_backend, ticket);
}

int nbg_ring_group(nbg_ring* r, uint64_t ticket, uint32_t* d_perm, uint32_t* d_counts, void* stream) {
  if (!r || !d_perm || !d_counts) return set_error(NBG_EINVAL, "ring_group: null argument");
  std::lock_guard<std::mutex> g(r->mu);
  if (r->leaked) return ring_leaked_error();
  return ring_group_locked(r, ticket, d_perm, d_counts, static_cast<hipStream_t>(stream));
}

int nbg_ring_group_burst(nbg_ring* r, uint64_t first_ticket, uint32_t n_batches, uint32_t* const* d_perm,
                         uint32_t* const* d_counts, void* stream) {
  if (!r || !d_perm || !d_counts) return set_error(NBG_EINVAL, "ring_group_burst: null argument");
  std::lock_guard<std::mutex> g(r->mu);
  if (r->leaked) return ring_leaked_error();
  return ring_group_burst_locked(r, first_ticket, n_batches, d_perm, d_counts, static_cast<hipStream_t>(stream));
}

// Diagnostics (not in include/nbgpu.h): the window stride host batch `ticket` was staged at (32, 48,
// 64 or 80; 0 for zero-copy), while its slot still holds it; -1 otherwise.
int nbg_debug_host_win(nbg_maglev* h, uint64_t ticket) {
  if (!h || ticket == 0 || ticket >= h->next_ticket) return -1;
  const auto& t = h->slots[ticket % NBG_HOST_SLOTS];
  return t.ticket == ticket ? static_cast<int>(t.win) : -1;
}

// Diagnostics (not in include/nbgpu.h): the host control line's 16 words.
int nbg_debug_ring_ctl(nbg_ring* r, uint32_t* out) {
  if (!r || !out) return NBG_EINVAL;
  const volatile uint32_t* w = reinterpret_cast<const volatile uint32_t*>(r->ctl);
  for (int i = 0; i < 16; ++i) out[i] = w[i];
  return NBG_OK;
}

int nbg_ring_kernel_ms(nbg_maglev* h, float* ms) {
  if (!h || !ms) return set_error(NBG_EINVAL, "ring_kernel_ms: null argument");
  if (h->ring_kernel_ms < 0.f) return set_error(NBG_EINVAL, "ring_kernel_ms: no stopped ring on this handle");
  *ms = h->ring_kernel_ms;
  return NBG_OK;
}

int nbg_ring_poll(nbg_ring* r, uint64_t* completed) {
  if (!r || !completed) return set_error(NBG_EINVAL, "ring_poll: null argument");
  std::lock_guard<std::mutex> g(r->mu);
  if (r->leaked) return ring_leaked_error();
  ring_refresh(r);
  *completed = r->completed;
  if (r->completed < r->posted && ring_gone(r)) return ring_state_error(r);
  return NBG_OK;
}

int nbg_ring_wait(nbg_ring* r, uint64_t ticket, uint32_t timeout_ms) {
  if (!r) return set_error(NBG_EINVAL, "ring_wait: null ring");
  {
    std::lock_guard<std::mutex> g(r->mu);
    if (r->leaked) return ring_leaked_error();
    if (ticket >= r->posted)
      return set_error(NBG_EINVAL, "ring_wait: ticket %llu was not posted", (unsigned long long)ticket);
  }
  return ring_wait_for(r, timeout_ms, "ring_wait", ticket, [&] { return r->completed > ticket; });
}

int nbg_ring_stop(nbg_ring* r) {
  if (!r) return set_error(NBG_EINVAL, "ring_stop: null ring");
  std::unique_lock<std::mutex> lk(r->mu);
  if (r->leaked) return ring_leaked_error();
  // a repeat stop (or a stale one from another thread) reports the first stop's result: the ring is
  // already in the handle's spare or dead list and must not be detached or listed twice
  while (r->stopping && !r->stopped && !r->leaked) {  // another thread's stop is draining the kernel
    lk.unlock();
    std::this_thread::sleep_for(std::chrono::microseconds(20));
    lk.lock();
  }
  if (r->leaked) return ring_leaked_error();
  if (r->stopped) return r->stop_rc ? set_error(r->stop_rc, "ring_stop: already stopped (%d)", r->stop_rc) : NBG_OK;
  DeviceGuard g(r->device);
  r->stopping = true;  // the lock is released while the kernel drains: no post may follow the stop word
  __atomic_store_n(&const_cast<RingCtl*>(const_cast<volatile RingCtl*>(r->ctl))->stop, 1u, __ATOMIC_RELEASE);
  const auto t0 = Clock::now();
  int rc = NBG_OK;
  while (!ring_ended(r)) {
    if (Clock::now() - t0 > std::chrono::milliseconds(r->idle_ms + 5000u)) {
      // never free memory a running kernel may still read: leak the ring (and the handle's device
      // memory, nbg_maglev_destroy) instead; the device stays marked busy, and every later call on
      // the ring returns NBG_EBUSY without touching the handle
      if (r->h->ring == r) r->h->ring = nullptr;
      r->h->ring_leaked = true;
      r->leaked = true;
      return set_error(NBG_EBUSY, "ring_stop: the kernel did not end (its memory is leaked, the device stays busy)");
    }
    lk.unlock();  // producers blocked in post / wait take the lock to see the kernel end
    ring_pause(t0);
    lk.lock();
  }
  // the kernel has ended, so every call still waiting on the ring returns at its next look: let them
  // leave before the queues close and the scratch is released (or the ring freed)
  while (r->calls) {
    lk.unlock();
    std::this_thread::sleep_for(std::chrono::microseconds(20));
    lk.lock();
  }
  {
    std::lock_guard<std::mutex> dg(g_dev_ring_mu);
    if (static_cast<size_t>(r->device) < g_dev_ring.size() && g_dev_ring[r->device] == r) g_dev_ring[r->device] = nullptr;
  }
  const hipError_t e = hipStreamQuery(r->stream);
  ring_refresh(r);
  if (e != hipSuccess) rc = set_error(NBG_EIO, "ring_stop: %s", hipGetErrorString(e));
  else if (r->completed < r->posted) rc = ring_state_error(r);
  nbg_maglev* h = r->h;
  if (h->ring == r) h->ring = nullptr;
  r->stopped = true;
  r->stop_rc = rc;
  float ms = -1.f;
  if (e == hipSuccess && hipEventElapsedTime(&ms, r->ev_start, r->ev_end) == hipSuccess) h->ring_kernel_ms = ms;
  ring_close_queues(r);
  if (e != hipSuccess) {
    // the stream failed: the ring is not reused, but callers may still hold it and its queues, so it
    // is kept (every call reports the failure) and freed with the handle
    h->ring_dead.push_back(r);
    return rc;
  }
  // keep the buffers, stream and events for the next start; the grouping streams' work on the
  // scratch is finished first
  ring_release_sets(r);
  h->ring_spare = r;
  return rc;
}

int nbg_ring_queue_open(nbg_ring* r, nbg_ring_queue** out) {
  if (!r || !out) return set_error(NBG_EINVAL, "ring_queue_open: null argument");
  *out = nullptr;
  std::lock_guard<std::mutex> g(r->mu);
  if (r->leaked) return ring_leaked_error();
  if (r->queues.size() >= NBG_RING_MAX_QUEUES)
    return set_error(NBG_EBUSY, "ring_queue_open: the ring has %u queues open", NBG_RING_MAX_QUEUES);
  auto* q = new (std::nothrow) nbg_ring_queue;
  if (!q) return set_error(NBG_ENOMEM, "ring_queue_open: out of memory");
  q->r = r;
  r->queues.push_back(q);
  *out = q;
  return NBG_OK;
}

int nbg_ring_queue_close(nbg_ring_queue* q) {
  if (!q) return set_error(NBG_EINVAL, "ring_queue_close: null queue");
  nbg_ring* r = q->r;
  std::lock_guard<std::mutex> g(r->mu);
  if (q->closed) {  // closed by nbg_ring_stop: free it now
    auto it = std::find(r->closed.begin(), r->closed.end(), q);
    if (it == r->closed.end()) return set_error(NBG_EINVAL, "ring_queue_close: not a queue of its ring");
    r->closed.erase(it);
    delete q;
    return NBG_OK;
  }
  auto it = std::find(r->queues.begin(), r->queues.end(), q);
  if (it == r->queues.end()) return set_error(NBG_EINVAL, "ring_queue_close: not an open queue of its ring");
  r->queues.erase(it);
  delete q;
  return NBG_OK;
}

int nbg_ring_queue_post(nbg_ring_queue* q, uint8_t* d_pkts, uint64_t n_pkts, uint16_t* d_backend, uint64_t* ticket) {
  if (!q || !ticket) return set_error(NBG_EINVAL, "ring_queue_post: null argument");
  return ring_post_one(q->r, q, d_pkts, n_pkts, d_backend, ticket);
}

int nbg_ring_queue_poll(nbg_ring_queue* q, uint64_t* completed) {
  if (!q || !completed) return set_error(NBG_EINVAL, "ring_queue_poll: null argument");
  nbg_ring* r = q->r;
  std::lock_guard<std::mutex> g(r->mu);
  if (r->leaked) return ring_leaked_error();
  if (q->closed) return set_error(NBG_EINVAL, "ring_queue_poll: the queue was closed by nbg_ring_stop");
  ring_refresh(r);
  queue_refresh(q);
  *completed = q->done;
  if (q->done < q->posted && ring_gone(r)) return ring_state_error(r);
  return NBG_OK;
}

int nbg_ring_queue_wait(nbg_ring_queue* q, uint64_t ticket, uint32_t timeout_ms) {
  if (!q) return set_error(NBG_EINVAL, "ring_queue_wait: null queue");
  nbg_ring* r = q->r;
  {
    std::lock_guard<std::mutex> g(r->mu);
    if (r->leaked) return ring_leaked_error();
    if (q->closed) return set_error(NBG_EINVAL, "ring_queue_wait: the queue was closed by nbg_ring_stop");
    if (ticket >= q->posted)
      return set_error(NBG_EINVAL, "ring_queue_wait: ticket %llu was not posted on this queue",
                       (unsigned long long)ticket);
  }
  // a queue stop closes while this waits still has its tickets' completion (the ring completes every
  // posted batch before it ends), so the wait reports that rather than the close
  return ring_wait_for(r, timeout_ms, "ring_queue_wait", ticket, [&] {
    queue_refresh(q);
    return q->done > ticket;
  });
}

int nbg_ring_queue_group(nbg_ring_queue* q, uint64_t ticket, uint32_t* d_perm, uint32_t* d_counts, void* stream) {
  if (!q || !d_perm || !d_counts) return set_error(NBG_EINVAL, "ring_queue_group: null argument");
  nbg_ring* r = q->r;
  std::lock_guard<std::mutex> g(r->mu);
  if (r->leaked) return ring_leaked_error();
  if (q->closed) return set_error(NBG_EINVAL, "ring_queue_group: the queue was closed by nbg_ring_stop");
  if (ticket >= q->posted)
    return set_error(NBG_EINVAL, "ring_queue_group: ticket %llu was not posted on this queue", (unsigned long long)ticket);
  if (q->posted - ticket > NBG_RING_SLOTS)
    return set_error(NBG_EINVAL, "ring_queue_group: ticket %llu is older than the queue's last %u", (unsigned long long)ticket,
                     NBG_RING_SLOTS);
  return ring_group_locked(r, q->gidx[ticket % NBG_RING_SLOTS], d_perm, d_counts, static_cast<hipStream_t>(stream));
}

}  // extern "C"

namespace {

// Stage the header windows of a host batch at a `win`-byte stride (the first min(len, win) bytes of
// every frame) and return the stride the batch needs: the path reads 14 + max(20, 4*IHL + 4)
// bytes (utils/flow.rs:53-62) — 38 for IHL 5 — so 48-B windows (three 16-B chunks) serve every
// frame longer than 48 B with IHL <= 7; 64 B up to IHL 11, 80 B beyond.  The IHL byte is read from
// the staged copy, so one pass over the (scattered) mbufs both gathers and sizes; frames shorter
// than the stride are staged whole and take the kernel's byte-wise path.  Software prefetch runs
// kAhead frames ahead: the gather is bound by host memory latency, one cache line per mbuf.
// swap: apply MacHeader::swap_addresses (headers/mac.rs:140-145) to every frame of >= 14 B while its
// line is in cache (the staged copy keeps the bytes as received; the flow hash reads none of the 12
// swapped bytes), so no second pass over the mbufs writes the swap back after the GPU.
//
// base = 8, win = 32 (a direct batch, whose small kernel takes 32-B windows): bytes 8..39 of every frame,
// which hold every byte an IHL-5 parse reads once the MACs are swapped here; 32 comes back when every
// frame longer than 40 B has IHL <= 5, else the stride a whole-window staging needs (the caller stages
// the batch again from byte 0).  A third fewer bytes cross PCIe than with 48-B windows.
uint32_t host_gather(uint8_t* const* pkt_ptrs, const uint16_t* lens, uint64_t n, uint32_t win, uint32_t base,
                     uint8_t* h_win, uint16_t* h_len, bool swap) {
  constexpr uint64_t kAhead = 16;  // 32 and 64 measured no faster (profiles/r06_dropin_tune.json)
  const uint32_t top = base + win;  // frames longer than this are sized by their IP header
  std::atomic<uint32_t> need{top};
  parallel_for(n, [&](uint64_t b, uint64_t e) {
    uint32_t m = top;
    for (uint64_t i = b; i < e; ++i) {
      if (i + kAhead < e) __builtin_prefetch(pkt_ptrs[i + kAhead], 1, 0);  // read, then (swap) written
      const uint32_t l = lens[i], c = l > base ? std::min<uint32_t>(l, top) - base : 0u;
      uint8_t* w = h_win + i * win;
      uint8_t* f = pkt_ptrs[i];
      std::memcpy(w, f + base, c);
      h_len[i] = static_cast<uint16_t>(l);
      if (l > top) m = std::max<uint32_t>(m, 14 + std::max<uint32_t>(20, (w[14 - base] & 0xfu) * 4 + 4));
      if (swap && l >= 14) {
        uint8_t dst[6];
        std::memcpy(dst, f, 6);
        std::memmove(f, f + 6, 6);
        std::memcpy(f + 6, dst, 6);
      }
    }
    uint32_t cur = need.load();
    while (m > cur && !need.compare_exchange_weak(cur, m)) {
    }
  });
  const uint32_t m = need.load();
  if (base == 8 && win == 32 && m <= 40) return 32;
  return m <= 48 ? 48 : (m <= 64 ? 64 : 80);
}

int slot_reserve(nbg_maglev* h, nbg_maglev::HostSlot& t, uint64_t n) {
  if (!t.done) NBG_HIP(hipEventCreateWithFlags(&t.done, hipEventDisableTiming));
  if (!t.h_flag) {
    NBG_HIP(hipHostMalloc(reinterpret_cast<void**>(&t.h_flag), 64, hipHostMallocMapped | hipHostMallocCoherent));
    *reinterpret_cast<volatile uint32_t*>(t.h_flag) = 0;
    NBG_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&t.dh_flag), t.h_flag, 0));
  }
  if (n <= t.cap) return NBG_OK;
  free_slot_buffers(t);
  const uint64_t cap = std::max<uint64_t>(n, 4096);
  const size_t nbins = h->nb + 1;
  const size_t win_bytes = cap * 80 + 64;  // any window stride, + the last packet's 4th chunk
  // mapped and fine-grained: the direct path's kernel reads and writes them over PCIe (no stale
  // lines in the GPU's caches between the slot's batches; the copies of the large-batch path do not
  // care)
  constexpr unsigned kPin = hipHostMallocMapped | hipHostMallocCoherent;
  // NBG_HOST_IN_COARSE=1 (measurement): the staged windows and lengths coarse-grained, so the direct
  // kernel's reads go through the L2 (the dispatch's acquire invalidates it)
  static const unsigned kPinIn = [] {
    const char* e = std::getenv("NBG_HOST_IN_COARSE");
    return e && std::atoi(e) == 1 ? unsigned{hipHostMallocMapped | hipHostMallocNonCoherent} : kPin;
  }();
  NBG_HIP(hipHostMalloc(reinterpret_cast<void**>(&t.h_win), win_bytes, kPinIn));
  NBG_HIP(hipHostMalloc(reinterpret_cast<void**>(&t.h_len), cap * 2, kPinIn));
  NBG_HIP(hipHostMalloc(reinterpret_cast<void**>(&t.h_backend), cap * 2, kPin));
  NBG_HIP(hipHostMalloc(reinterpret_cast<void**>(&t.h_perm), cap * 4, kPin));
  NBG_HIP(hipHostMalloc(reinterpret_cast<void**>(&t.h_counts), nbins * 4, kPin));
  NBG_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&t.dh_win), t.h_win, 0));
  NBG_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&t.dh_len), t.h_len, 0));
  NBG_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&t.dh_backend), t.h_backend, 0));
  NBG_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&t.dh_perm), t.h_perm, 0));
  NBG_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&t.dh_counts), t.h_counts, 0));
  NBG_HIP(hipMalloc(&t.d_win, win_bytes));
  NBG_HIP(hipMalloc(&t.d_len, cap * 2));
  NBG_HIP(hipMalloc(&t.d_backend, cap * 2));
  NBG_HIP(hipMalloc(&t.d_perm, cap * 4));
  NBG_HIP(hipMalloc(&t.d_counts, nbins * 4));
  // the slack past the last window is read, never used; zeroed in stream order before the H2D
  // copies that follow on the same stream (not on the null stream: see SetupStream)
  NBG_HIP(hipMemsetAsync(t.d_win, 0, win_bytes, h->host_compute));
  t.cap = cap;
  return NBG_OK;
}

// The direct batch in slot t has finished: its completion word holds its ticket.
bool flag_set(const nbg_maglev::HostSlot& t) {
  return __atomic_load_n(t.h_flag, __ATOMIC_ACQUIRE) == static_cast<uint32_t>(t.ticket);
}

// Wait for a direct batch's completion word: spin, then yield; the stream is queried now and then, so
// a kernel that failed (its word never set) is reported instead of waited for.  A batch posted to a
// host-batch server whose kernel ended before taking it (its idle exit racing the post) is launched.
int wait_flag(nbg_maglev* h, nbg_maglev::HostSlot& t) {
  for (uint32_t spin = 0; !flag_set(t); ++spin) {
    if (spin < 2048) {
      __builtin_ia32_pause();
      continue;
    }
    std::this_thread::yield();
    if ((spin & 255u) == 0) {
      const hipError_t e = hipStreamQuery(t.watch);
      if (e != hipSuccess && e != hipErrorNotReady) return set_error(NBG_EIO, "host_wait: %s", hipGetErrorString(e));
      if (e == hipSuccess && !flag_set(t)) {
        if (!t.on_ring) return set_error(NBG_EIO, "host_wait: the batch's kernel ended without its completion word");
        t.on_ring = false;  // no block of the ended server touches it: launch it
        t.watch = h->host_compute;
        DeviceGuard g(h->device);
        const int rc = launch_small(t.ra, t.rg, h->wide, h->host_compute, t.dh_flag, static_cast<uint32_t>(t.ticket));
        if (rc) return rc;
      }
    }
  }
  return NBG_OK;
}

// Complete the batch held by slot t: wait for it (completion word or D2H copies) and hand the results
// to the caller's buffers (the MAC swap was applied at submit: in the gather, or by the zero-copy kernel).
int slot_complete(nbg_maglev* h, nbg_maglev::HostSlot& t) {
  if (!t.busy) return NBG_OK;
  t.busy = false;
  if (t.direct) {
    const int rc = wait_flag(h, t);
    if (rc) return rc;
  } else {
    NBG_HIP(hipEventSynchronize(t.done));
  }
  const uint64_t n = t.n;
  if (t.backend_out) std::memcpy(t.backend_out, t.h_backend, n * 2);
  if (t.perm_out) std::memcpy(t.perm_out, t.h_perm, n * 4);
  if (t.counts_out) std::memcpy(t.counts_out, t.h_counts, (h->nb + 1) * 4);
  return NBG_OK;
}


// The arguments the small kernel would be launched with for a host batch (classify_common's small
// path): packets at pkts (+ off[i], or i * stride), lengths len[], outputs in pinned host memory.
void small_args(const nbg_maglev* h, uint8_t* pkts, const uint32_t* off, const uint16_t* len, uint32_t stride,
                uint64_t n, uint32_t flags, uint16_t* backend, uint32_t* perm, uint32_t* counts, ClassifyArgs& a,
                GroupArgs& g, bool win32 = false) {
  a = ClassifyArgs{};
  a.pkts = pkts;
  a.off = off;
  a.len = len;
  a.stride = stride;
  a.n_pkts = static_cast<uint32_t>(n);
  a.tiles_per_wave = 1;
  a.lut = h->d_lut;
  a.m = static_cast<uint32_t>(h->m);
  a.mu = ~0ull / h->m + ((~0ull % h->m) + 1 == h->m ? 1 : 0);  // floor(2^64 / m)
  a.nb = h->nb;
  a.swap = (flags & NBG_SWAP_MACS) ? 1u : 0u;
  a.win_owned = (!off && stride >= 64) || (flags & NBG_OWNED_WINDOWS) ? 1u : 0u;
  a.wb_full = (flags & NBG_WB_PARTIAL) ? 0u : 1u;
  a.win32 = win32 ? 1u : 0u;
  a.backend = backend;
  g = GroupArgs{};
  g.perm = perm;
  g.counts = counts;
}

// Post a direct batch to the handle's host-batch server; false when the server has ended or stops
// (the caller launches the small kernel instead).  Producer threads post concurrently: tickets come
// from one atomic counter, a slot is reused once a block acknowledged its previous descriptor.
bool host_ring_post(nbg_host_ring* r, const ClassifyArgs& a, const GroupArgs& g, uint32_t variant, uint32_t* done,
                    uint32_t done_val) {
  if (r->stopping.load() || __atomic_load_n(&r->ctl->ended, __ATOMIC_ACQUIRE)) return false;
  const uint64_t t = r->next.fetch_add(1);
  auto* d = reinterpret_cast<HostRingDesc*>(r->desc + (t & (r->slots - 1)) * kHostRingDescBytes);
  if (t >= r->slots) {
    const uint32_t want = static_cast<uint32_t>(t - r->slots + 1);
    for (uint32_t spin = 0; __atomic_load_n(&d->ack, __ATOMIC_ACQUIRE) != want; ++spin) {
      // a server that ended (idle exit racing an earlier post) never acknowledges the slot: launch
      if (__atomic_load_n(&r->ctl->ended, __ATOMIC_ACQUIRE)) return false;
      if (spin < 4096) {
        __builtin_ia32_pause();
      } else {
        std::this_thread::yield();  // the slots' batches are in flight: a block takes one every few us
      }
    }
  }
  d->variant = variant;
  d->done_val = done_val;
  d->done = done;
  d->a = a;
  d->g = g;
  __atomic_store_n(&d->seq, static_cast<uint32_t>(t + 1), __ATOMIC_RELEASE);
  __atomic_store_n(&r->ctl->posted, static_cast<uint32_t>(t + 1), __ATOMIC_RELEASE);
  return true;
}

}  // namespace

extern "C" {

int nbg_maglev_host_submit(nbg_maglev* h, uint8_t* const* pkt_ptrs, const uint16_t* lens, uint64_t n,
                           uint32_t flags, uint16_t* backend_out, uint32_t* perm_out, uint32_t* counts_out,
                           uint64_t* ticket) {
  if (!h || !ticket || (!pkt_ptrs && n) || (!lens && n) || (!backend_out && n))
    return set_error(NBG_EINVAL, "host_submit: null argument");
  if (n >= (1ull << 30)) return set_error(NBG_EINVAL, "host_submit: n must be < 2^30");
  if (h->ring) return set_error(NBG_EBUSY, "host_submit: the handle's persistent ring is running");
  if (h->pending && !h->pending_lag)
    return set_error(NBG_EINVAL, "host_submit: a deferred group is pending (nbg_maglev_finish_group)");
  DeviceGuard g(h->device);
  if (!h->host_compute) NBG_HIP(hipStreamCreateWithFlags(&h->host_compute, hipStreamNonBlocking));
  const uint64_t tk = h->next_ticket;
  auto& t = h->slots[tk % NBG_HOST_SLOTS];
  int rc = slot_complete(h, t);  // the slot's previous batch, if its wait has not come yet
  if (rc) return rc;
  if ((rc = slot_reserve(h, t, n))) return rc;
  t.direct = false;
  t.on_ring = false;
  t.win = 0;
  const bool swap = flags & NBG_SWAP_MACS;
  t.n = n;
  t.backend_out = backend_out;
  t.perm_out = perm_out;
  t.counts_out = counts_out;
  t.ticket = tk;
  h->next_ticket = tk + 1;
  if (n == 0) {
    if (counts_out) std::memset(counts_out, 0, (h->nb + 1) * sizeof(uint32_t));
    *ticket = tk;
    return NBG_OK;
  }
  // zero-copy: every frame (and the 64 B the kernel may read from its start) lies in one registered
  // region below 4 GiB: only offsets and lengths cross PCIe; the kernel reads the frames and writes
  // the MAC chunk back in host memory, and no host thread touches a packet
  HostRegionRec reg{};
  if (n <= t.cap && find_region(pkt_ptrs[0], h->device, &reg) && reg.bytes <= (1ull << 32)) {
    std::atomic<bool> inside{true};
    uint32_t* h_off = reinterpret_cast<uint32_t*>(t.h_win);
    parallel_for(n, [&](uint64_t b, uint64_t e) {
      bool ok = true;
      for (uint64_t i = b; i < e; ++i) {
        const uintptr_t a = reinterpret_cast<uintptr_t>(pkt_ptrs[i]);
        ok &= a >= reg.base && a + 64 <= reg.base + reg.bytes;
        h_off[i] = static_cast<uint32_t>(a - reg.base);
        t.h_len[i] = lens[i];
      }
      if (!ok) inside.store(false);
    });
    if (inside.load()) {
      hipStream_t hs = h->host_compute;
      const bool group = perm_out || counts_out;
      const uint32_t zflags = (flags & ~(NBG_DEFER_GROUP | NBG_GROUP_LAG)) | NBG_OWNED_WINDOWS | NBG_WB_PARTIAL;
      if (use_small(n, h->nb + 1, zflags, reg.dev)) {
        // direct: the one small-kernel launch (or the host-batch server) reads the offsets and lengths
        // out of pinned memory and stores its results there (no copy on either side)
        ClassifyArgs a;
        GroupArgs ga;
        small_args(h, reg.dev, reinterpret_cast<const uint32_t*>(t.dh_win), t.dh_len, 0, n, zflags, t.dh_backend,
                   perm_out ? t.dh_perm : nullptr, group ? t.dh_counts : nullptr, a, ga);
        t.on_ring = h->hring && host_ring_post(h->hring, a, ga, small_variant(h->wide, a.m, h->nb, false), t.dh_flag,
                                               static_cast<uint32_t>(tk));
        if (t.on_ring) {
          t.watch = h->hring->stream;
          t.ra = a;
          t.rg = ga;
        } else {
          rc = classify_common(h, reg.dev, reinterpret_cast<const uint32_t*>(t.dh_win), t.dh_len, 0, 0, n, zflags,
                               t.dh_backend, perm_out ? t.dh_perm : nullptr, group ? t.dh_counts : nullptr, nullptr,
                               nullptr, 0, nullptr, hs, t.dh_flag, static_cast<uint32_t>(tk));
          if (rc) return rc;
          t.watch = hs;
        }
        t.direct = true;
        t.busy = true;
        *ticket = tk;
        return NBG_OK;
      }
      NBG_HIP(hipMemcpyAsync(t.d_win, h_off, n * 4, hipMemcpyHostToDevice, hs));
      NBG_HIP(hipMemcpyAsync(t.d_len, t.h_len, n * 2, hipMemcpyHostToDevice, hs));
      rc = nbg_maglev_classify_device_ex(h, reg.dev, reinterpret_cast<const uint32_t*>(t.d_win), t.d_len, 0, 0, n,
                                         (flags & ~(NBG_DEFER_GROUP | NBG_GROUP_LAG)) | NBG_OWNED_WINDOWS | NBG_WB_PARTIAL, t.d_backend,
                                         perm_out ? t.d_perm : nullptr, group ? t.d_counts : nullptr, nullptr, hs);
      if (rc) return rc;
      NBG_HIP(hipMemcpyAsync(t.h_backend, t.d_backend, n * 2, hipMemcpyDeviceToHost, hs));
      if (perm_out) NBG_HIP(hipMemcpyAsync(t.h_perm, t.d_perm, n * 4, hipMemcpyDeviceToHost, hs));
      if (counts_out) NBG_HIP(hipMemcpyAsync(t.h_counts, t.d_counts, (h->nb + 1) * 4, hipMemcpyDeviceToHost, hs));
      NBG_HIP(hipEventRecord(t.done, hs));
      t.busy = true;
      *ticket = tk;
      return NBG_OK;
    }
  }
  // gather, swapping the MACs in the mbufs on the way: a direct batch at 32-B windows (frame bytes
  // 8..39), a copied one at 48-B windows; a batch with longer IP headers is staged again (without
  // swapping) from byte 0 at the stride it needs
  const uint32_t sflags =
      (flags & ~(NBG_DEFER_GROUP | NBG_WB_PARTIAL | NBG_GROUP_LAG | NBG_SWAP_MACS)) | NBG_OWNED_WINDOWS;
  const bool direct = use_small(n, h->nb + 1, sflags, t.dh_win);
  // NBG_HOST_WIN48=1 (measurement): direct batches at 48-B windows, as before the 32-B staging
  static const bool win48 = [] {
    const char* e = std::getenv("NBG_HOST_WIN48");
    return e && std::atoi(e) == 1;
  }();
  uint32_t win = direct && !win48 ? host_gather(pkt_ptrs, lens, n, 32, 8, t.h_win, t.h_len, swap) : 0u;
  if (win != 32) {
    win = host_gather(pkt_ptrs, lens, n, 48, 0, t.h_win, t.h_len, swap && !(direct && !win48));
    if (win > 48) host_gather(pkt_ptrs, lens, n, win, 0, t.h_win, t.h_len, false);
  }
  t.win = win;
  // copies and kernels in submit order on the handle's one host stream (the kernels share the
  // handle's grouping scratch).  No cross-stream event: with the copies on a stream of their own
  // and an event wait on the compute stream, kernels were seen reading windows whose H2D copy had
  // not landed (zero windows, sporadically, with many streams in the process).  The host gathers
  // the next batch while this one runs.
  hipStream_t hs = h->host_compute;
  const bool group = perm_out || counts_out;
  if (direct) {
    // direct: a batch of at most 2,048 packets (NetBricks' own bursts are 32) is classified and
    // grouped by one small-kernel launch that reads the staged windows out of pinned memory and
    // stores backend / perm / counts there.  The copies' fixed costs (a few us each on the DMA
    // engines, four to six per batch) were the whole cost of a small batch
    ClassifyArgs a;
    GroupArgs ga;
    small_args(h, t.dh_win, nullptr, t.dh_len, win, n, sflags, t.dh_backend, perm_out ? t.dh_perm : nullptr,
               group ? t.dh_counts : nullptr, a, ga, win == 32);
    t.on_ring = h->hring && host_ring_post(h->hring, a, ga, small_variant(h->wide, a.m, h->nb, win == 32), t.dh_flag,
                                           static_cast<uint32_t>(tk));
    if (t.on_ring) {
      t.watch = h->hring->stream;
      t.ra = a;
      t.rg = ga;
    } else {
      rc = classify_common(h, t.dh_win, nullptr, t.dh_len, win, 0, n, sflags, t.dh_backend,
                           perm_out ? t.dh_perm : nullptr, group ? t.dh_counts : nullptr, nullptr, nullptr, 0, nullptr,
                           hs, t.dh_flag, static_cast<uint32_t>(tk), win == 32);
      if (rc) return rc;
      t.watch = hs;
    }
    t.direct = true;
    t.busy = true;
    *ticket = tk;
    return NBG_OK;
  }
  NBG_HIP(hipMemcpyAsync(t.d_win, t.h_win, n * win, hipMemcpyHostToDevice, hs));
  NBG_HIP(hipMemcpyAsync(t.d_len, t.h_len, n * 2, hipMemcpyHostToDevice, hs));
  rc = nbg_maglev_classify_device_ex(h, t.d_win, nullptr, t.d_len, win, 0, n, sflags, t.d_backend,
                                     perm_out ? t.d_perm : nullptr, group ? t.d_counts : nullptr, nullptr, hs);
  if (rc) return rc;
  NBG_HIP(hipMemcpyAsync(t.h_backend, t.d_backend, n * 2, hipMemcpyDeviceToHost, hs));
  if (perm_out) NBG_HIP(hipMemcpyAsync(t.h_perm, t.d_perm, n * 4, hipMemcpyDeviceToHost, hs));
  if (counts_out) NBG_HIP(hipMemcpyAsync(t.h_counts, t.d_counts, (h->nb + 1) * 4, hipMemcpyDeviceToHost, hs));
  NBG_HIP(hipEventRecord(t.done, hs));
  t.busy = true;
  *ticket = tk;
  return NBG_OK;
}

int nbg_host_register(void* base, uint64_t bytes, int device, uint8_t** dev_base) {
  if (!base || !bytes || !dev_base) return set_error(NBG_EINVAL, "host_register: null argument");
  int rc = check_device(device);
  if (rc) return rc;
  DeviceGuard g(device);
  NBG_HIP(hipHostRegister(base, bytes, hipHostRegisterMapped));
  void* d = nullptr;
  const hipError_t e = hipHostGetDevicePointer(&d, base, 0);
  if (e != hipSuccess) {
    (void)hipHostUnregister(base);
    return set_error(NBG_EIO, "host_register: hipHostGetDevicePointer: %s", hipGetErrorString(e));
  }
  *dev_base = static_cast<uint8_t*>(d);
  std::lock_guard<std::mutex> lk(g_regions_mu);
  g_regions.push_back({reinterpret_cast<uintptr_t>(base), bytes, *dev_base, device});
  return NBG_OK;
}

int nbg_host_unregister(void* base, int device) {
  if (!base) return set_error(NBG_EINVAL, "host_unregister: null base");
  int rc = check_device(device);
  if (rc) return rc;
  DeviceGuard g(device);
  {
    std::lock_guard<std::mutex> lk(g_regions_mu);
    for (size_t i = 0; i < g_regions.size(); ++i)
      if (g_regions[i].base == reinterpret_cast<uintptr_t>(base) && g_regions[i].device == device) {
        g_regions.erase(g_regions.begin() + static_cast<std::ptrdiff_t>(i));
        break;
      }
  }
  NBG_HIP(hipHostUnregister(base));
  return NBG_OK;
}

int nbg_device_local_cpus(int device, int32_t* cpus, uint32_t cap, uint32_t* n) {
  if (!n || (!cpus && cap)) return set_error(NBG_EINVAL, "device_local_cpus: null argument");
  *n = 0;
  const int rc = check_device(device);
  if (rc) return rc;
  char bus[64] = {0};
  NBG_HIP(hipDeviceGetPCIBusId(bus, static_cast<int>(sizeof bus) - 1, device));
  for (char* c = bus; *c; ++c) *c = static_cast<char>(std::tolower(static_cast<unsigned char>(*c)));
  const std::string path = std::string("/sys/bus/pci/devices/") + bus + "/local_cpulist";
  FILE* f = std::fopen(path.c_str(), "r");
  if (!f) return set_error(NBG_EIO, "device_local_cpus: cannot read %s", path.c_str());
  char line[4096] = {0};
  const bool got = std::fgets(line, sizeof line, f) != nullptr;
  std::fclose(f);
  if (!got) return set_error(NBG_EIO, "device_local_cpus: %s is empty", path.c_str());
  // "0-63,128-191": ranges and single CPUs, comma separated
  uint32_t count = 0;
  for (const char* p = line; *p && *p != '\n';) {
    char* end = nullptr;
    const long lo = std::strtol(p, &end, 10);
    if (end == p || lo < 0) return set_error(NBG_EIO, "device_local_cpus: cannot parse %s", line);
    long hi = lo;
    p = end;
    if (*p == '-') {
      hi = std::strtol(p + 1, &end, 10);
      if (end == p + 1 || hi < lo) return set_error(NBG_EIO, "device_local_cpus: cannot parse %s", line);
      p = end;
    }
    for (long c = lo; c <= hi; ++c, ++count)
      if (count < cap) cpus[count] = static_cast<int32_t>(c);
    if (*p == ',') ++p;
  }
  *n = count;
  return count ? NBG_OK : set_error(NBG_EIO, "device_local_cpus: %s lists no CPU", path.c_str());
}

int nbg_host_ring_start(int device, uint32_t blocks, uint32_t idle_ms, nbg_host_ring** out) {
  if (!out) return set_error(NBG_EINVAL, "host_ring_start: null argument");
  *out = nullptr;
  int rc = check_device(device);
  if (rc) return rc;
  DeviceGuard g(device);
  int cus = 0;
  NBG_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
  if (blocks == 0) blocks = 64;  // 16 pipelines: 32 -> 626, 64 -> 673 Mpps (profiles/r06_dropin_win32.json)
  if (blocks > static_cast<uint32_t>(cus) / 2)
    return set_error(NBG_EINVAL, "host_ring_start: %u blocks (one per CU, at most half of the %d CUs)", blocks, cus);
  // one resident server per device, and not beside a persistent RX ring (whose blocks need every CU)
  std::lock_guard<std::mutex> dev_lock(g_dev_ring_mu);
  if (static_cast<size_t>(device) < g_dev_ring.size() && g_dev_ring[device])
    return set_error(NBG_EBUSY, "host_ring_start: device %d runs a persistent RX ring", device);
  if (static_cast<size_t>(device) < g_dev_hring.size() && g_dev_hring[device])
    return set_error(NBG_EBUSY, "host_ring_start: device %d already runs a host-batch server", device);
  auto* r = new (std::nothrow) nbg_host_ring;
  if (!r) return set_error(NBG_ENOMEM, "host_ring_start: out of memory");
  r->device = device;
  r->blocks = blocks;
  r->slots = 256;
  r->idle_ms = idle_ms ? idle_ms : 2000u;
  auto fail = [&](int code, const char* what) {
    if (r->stream) (void)hipStreamDestroy(r->stream);
    if (r->host) (void)hipHostFree(r->host);
    if (r->claim) (void)hipFree(r->claim);
    delete r;
    return set_error(code, "host_ring_start: %s", what);
  };
  if (static_cast<size_t>(device) < g_hring_stream.size() && g_hring_stream[device]) {
    r->stream = g_hring_stream[device];
    g_hring_stream[device] = nullptr;
  } else {
    int least = 0, greatest = 0;
    (void)hipDeviceGetStreamPriorityRange(&least, &greatest);
    if (hipStreamCreateWithPriority(&r->stream, hipStreamNonBlocking, greatest) != hipSuccess) {
      r->stream = nullptr;
      return fail(NBG_EIO, "private stream");
    }
  }
  const size_t hbytes = 64 + static_cast<size_t>(r->slots) * kHostRingDescBytes;
  if (hipHostMalloc(reinterpret_cast<void**>(&r->host), hbytes, hipHostMallocMapped | hipHostMallocCoherent) !=
      hipSuccess) {
    r->host = nullptr;
    return fail(NBG_ENOMEM, "pinned descriptor ring");
  }
  std::memset(r->host, 0, hbytes);
  r->ctl = reinterpret_cast<HostRingCtl*>(r->host);
  r->desc = r->host + 64;
  if (hipMalloc(&r->claim, 64) != hipSuccess) {
    r->claim = nullptr;
    return fail(NBG_ENOMEM, "claim counter");
  }
  uint8_t* hdev = nullptr;
  if (hipMemsetAsync(r->claim, 0, 64, r->stream) != hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&hdev), r->host, 0) != hipSuccess)
    return fail(NBG_EIO, "setup");
  HostRingArgs a{};
  a.ctl = reinterpret_cast<HostRingCtl*>(hdev);
  a.desc = hdev + 64;
  a.claim = r->claim;
  a.slots = r->slots;
  a.idle_ticks = static_cast<uint64_t>(r->idle_ms) * 100000u;  // 100 MHz
  if ((rc = launch_host_ring(a, blocks, r->stream))) {
    (void)hipStreamSynchronize(r->stream);
    return fail(rc, nbg_last_error());
  }
  if (static_cast<size_t>(device) >= g_dev_hring.size()) g_dev_hring.resize(device + 1, nullptr);
  g_dev_hring[device] = r;
  *out = r;
  return NBG_OK;
}

int nbg_host_ring_stop(nbg_host_ring* r) {
  if (!r) return set_error(NBG_EINVAL, "host_ring_stop: null server");
  if (r->leaked) return set_error(NBG_EBUSY, "host_ring_stop: its kernel did not end at an earlier stop (leaked)");
  if (r->attached.load())
    return set_error(NBG_EBUSY, "host_ring_stop: %u handles still use it (nbg_maglev_set_host_ring(h, NULL) first)",
                     r->attached.load());
  DeviceGuard g(r->device);
  r->stopping = true;
  __atomic_store_n(&r->ctl->stop, 1u, __ATOMIC_RELEASE);
  const auto t0 = std::chrono::steady_clock::now();
  while (hipStreamQuery(r->stream) == hipErrorNotReady) {
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(r->idle_ms + 5000u)) {
      r->leaked = true;  // never free what a running kernel may touch
      return set_error(NBG_EBUSY, "host_ring_stop: the kernel did not end (its memory is leaked)");
    }
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  const hipError_t e = hipStreamQuery(r->stream);
  {
    std::lock_guard<std::mutex> dev_lock(g_dev_ring_mu);
    if (static_cast<size_t>(r->device) < g_dev_hring.size() && g_dev_hring[r->device] == r)
      g_dev_hring[r->device] = nullptr;
    if (static_cast<size_t>(r->device) >= g_hring_stream.size()) g_hring_stream.resize(r->device + 1, nullptr);
    if (!g_hring_stream[r->device]) g_hring_stream[r->device] = r->stream;
    else (void)hipStreamDestroy(r->stream);
  }
  (void)hipHostFree(r->host);
  (void)hipFree(r->claim);
  delete r;
  if (e != hipSuccess) return set_error(NBG_EIO, "host_ring_stop: %s", hipGetErrorString(e));
  return NBG_OK;
}

int nbg_maglev_set_host_ring(nbg_maglev* h, nbg_host_ring* r) {
  if (!h) return set_error(NBG_EINVAL, "set_host_ring: null handle");
  if (r && r->device != h->device) return set_error(NBG_EINVAL, "set_host_ring: the server runs on another device");
  if (r && (r->stopping.load() || r->leaked)) return set_error(NBG_EINVAL, "set_host_ring: the server was stopped");
  if (h->hring == r) return NBG_OK;
  // batches already posted to the old server complete through their completion words as before
  if (h->hring) h->hring->attached.fetch_sub(1);
  h->hring = r;
  if (r) r->attached.fetch_add(1);
  return NBG_OK;
}

int nbg_maglev_host_wait(nbg_maglev* h, uint64_t ticket) {
  if (!h) return set_error(NBG_EINVAL, "host_wait: null handle");
  if (ticket == 0 || ticket >= h->next_ticket) return set_error(NBG_EINVAL, "host_wait: unknown ticket %llu",
                                                                (unsigned long long)ticket);
  auto& t = h->slots[ticket % NBG_HOST_SLOTS];
  if (t.ticket != ticket) return NBG_OK;  // its slot was reused: the batch was completed then
  DeviceGuard g(h->device);
  return slot_complete(h, t);
}

int nbg_maglev_host_query(nbg_maglev* h, uint64_t ticket, int* done) {
  if (!h || !done) return set_error(NBG_EINVAL, "host_query: null argument");
  if (ticket == 0 || ticket >= h->next_ticket) return set_error(NBG_EINVAL, "host_query: unknown ticket %llu",
                                                                (unsigned long long)ticket);
  auto& t = h->slots[ticket % NBG_HOST_SLOTS];
  if (t.ticket != ticket || !t.busy) {  // completed by its wait, or by the submit that reused its slot
    *done = 1;
    return NBG_OK;
  }
  if (t.direct) {  // a plain load of the completion word: no runtime call
    *done = flag_set(t) ? 1 : 0;
    return NBG_OK;
  }
  DeviceGuard g(h->device);
  const hipError_t e = hipEventQuery(t.done);
  if (e == hipErrorNotReady) {
    *done = 0;
    return NBG_OK;
  }
  if (e != hipSuccess) return set_error(NBG_EIO, "host_query: %s", hipGetErrorString(e));
  *done = 1;
  return NBG_OK;
}

int nbg_maglev_classify_host(nbg_maglev* h, uint8_t* const* pkt_ptrs, const uint16_t* lens, uint64_t n,
                             uint32_t flags, uint16_t* backend_out, uint32_t* perm_out, uint32_t* counts_out) {
  uint64_t tk = 0;
  int rc = nbg_maglev_host_submit(h, pkt_ptrs, lens, n, flags, backend_out, perm_out, counts_out, &tk);
  return rc ? rc : nbg_maglev_host_wait(h, tk);
}

}  // extern "C"
