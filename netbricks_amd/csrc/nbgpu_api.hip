// C-ABI of the Maglev flow-steering path (include/nbgpu.h).
//
// Handle lifecycle mirrors the reference's one-time pipeline construction
// (test/maglev/src/nf.rs:84-111: Maglev::new + operator chain) and the per-batch
// producer task (framework/src/operators/group_by.rs:43-55).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <new>
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

struct nbg_maglev {
  int device = 0;
  uint32_t nb = 0;
  uint64_t m = 0;
  std::vector<uint16_t> lut_host;
  void* d_lut = nullptr;      // u8 (nb <= 256) or u16 entries, padded to 16 B
  bool wide = false;
  uint32_t lut_bytes = 0;     // padded device LUT bytes
  // per-call scratch
  uint64_t cap_tiles = 0;
  unsigned long long* d_desc = nullptr;
  uint32_t* d_tile_prefix = nullptr;
  uint32_t* d_group_base = nullptr;
  uint32_t* d_counts = nullptr;     // used when the caller passes no counts buffer
  unsigned long long* d_ticket = nullptr;
  uint32_t* d_err = nullptr;
  uint32_t epoch = 0;
  hipStream_t last_stream = nullptr;
  int grid_lds = 0, grid_global = 0;
  // host-path staging (pinned host + device)
  uint64_t host_cap = 0;
  uint32_t host_win = 0;
  uint8_t* h_win = nullptr;
  uint16_t* h_len = nullptr;
  uint8_t* h_mac = nullptr;
  uint8_t* d_win = nullptr;
  uint16_t* d_len = nullptr;
  uint16_t* d_backend = nullptr;
  uint32_t* d_perm = nullptr;
  hipStream_t host_stream = nullptr;
};

namespace {

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

void free_scratch(nbg_maglev* h) {
  (void)hipFree(h->d_desc);
  (void)hipFree(h->d_tile_prefix);
  h->d_desc = nullptr;
  h->d_tile_prefix = nullptr;
  h->cap_tiles = 0;
}

void free_host_path(nbg_maglev* h) {
  (void)hipHostFree(h->h_win);
  (void)hipHostFree(h->h_len);
  (void)hipHostFree(h->h_mac);
  (void)hipFree(h->d_win);
  (void)hipFree(h->d_len);
  (void)hipFree(h->d_backend);
  (void)hipFree(h->d_perm);
  h->h_win = nullptr;
  h->h_len = nullptr;
  h->h_mac = nullptr;
  h->d_win = nullptr;
  h->d_len = nullptr;
  h->d_backend = nullptr;
  h->d_perm = nullptr;
  h->host_cap = 0;
  h->host_win = 0;
}

int ensure_scratch(nbg_maglev* h, uint64_t n_pkts) {
  const uint64_t tiles = (n_pkts + kTile - 1) / kTile;
  if (tiles <= h->cap_tiles) return NBG_OK;
  free_scratch(h);
  const uint64_t cap = std::max<uint64_t>(tiles, 64);
  const size_t words = static_cast<size_t>(cap) * (h->nb + 1);
  NBG_HIP(hipMalloc(&h->d_desc, words * sizeof(unsigned long long)));
  NBG_HIP(hipMalloc(&h->d_tile_prefix, words * sizeof(uint32_t)));
  NBG_HIP(hipMemset(h->d_desc, 0, words * sizeof(unsigned long long)));
  h->cap_tiles = cap;
  return NBG_OK;
}

int upload(nbg_maglev* h) {
  DeviceGuard g(h->device);
  h->wide = h->nb > 256;
  const size_t esz = h->wide ? 2 : 1;
  h->lut_bytes = static_cast<uint32_t>((h->m * esz + 15) & ~uint64_t(15));
  std::vector<uint8_t> buf(h->lut_bytes, 0);
  if (h->wide) {
    std::memcpy(buf.data(), h->lut_host.data(), h->m * 2);
  } else {
    for (uint64_t j = 0; j < h->m; ++j) buf[j] = static_cast<uint8_t>(h->lut_host[j]);
  }
  NBG_HIP(hipMalloc(&h->d_lut, h->lut_bytes));
  NBG_HIP(hipMemcpy(h->d_lut, buf.data(), h->lut_bytes, hipMemcpyHostToDevice));
  NBG_HIP(hipMalloc(&h->d_group_base, (h->nb + 1) * sizeof(uint32_t)));
  NBG_HIP(hipMalloc(&h->d_counts, (h->nb + 1) * sizeof(uint32_t)));
  NBG_HIP(hipMalloc(&h->d_ticket, 2 * sizeof(unsigned long long)));
  NBG_HIP(hipMalloc(&h->d_err, sizeof(uint32_t)));
  NBG_HIP(hipMemset(h->d_ticket, 0, 2 * sizeof(unsigned long long)));
  NBG_HIP(hipMemset(h->d_err, 0, sizeof(uint32_t)));
  int rc = max_classify_grid(h->wide, true, h->lut_bytes, h->device, &h->grid_lds);
  if (rc) return rc;
  return max_classify_grid(h->wide, false, 0, h->device, &h->grid_global);
}

// LDS staging pays when the LUT fits two blocks per CU (<= 72 KiB).
bool use_lds_lut(const nbg_maglev* h, uint32_t flags) {
  return !(flags & NBG_LUT_GLOBAL) && h->lut_bytes <= 72 * 1024;
}

int finish_create(nbg_maglev* h, int device, nbg_maglev** out) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    delete h;
    return set_error(NBG_ENODEV, "no HIP device available (the Maglev path has no CPU fallback)");
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
  {
    DeviceGuard g(h->device);
    free_scratch(h);
    free_host_path(h);
    (void)hipFree(h->d_lut);
    (void)hipFree(h->d_group_base);
    (void)hipFree(h->d_counts);
    (void)hipFree(h->d_ticket);
    (void)hipFree(h->d_err);
    if (h->host_stream) (void)hipStreamDestroy(h->host_stream);
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
  DeviceGuard g(h->device);
  return ensure_scratch(h, max_pkts);
}

int nbg_maglev_classify_device(nbg_maglev* h, uint8_t* d_pkts, const uint32_t* d_off, const uint16_t* d_len,
                               uint32_t stride, uint16_t fixed_len, uint64_t n_pkts, uint32_t flags,
                               uint16_t* d_backend, uint32_t* d_perm, uint32_t* d_counts, void* stream) {
  if (!h) return set_error(NBG_EINVAL, "classify: null handle");
  if (n_pkts >= (1ull << 30)) return set_error(NBG_EINVAL, "classify: n_pkts must be < 2^30");
  if (n_pkts == 0) {
    if (d_counts) NBG_HIP(hipMemsetAsync(d_counts, 0, (h->nb + 1) * sizeof(uint32_t), (hipStream_t)stream));
    return NBG_OK;
  }
  if (!d_pkts || !d_backend) return set_error(NBG_EINVAL, "classify: null packet or backend buffer");
  if (!d_off && stride == 0) return set_error(NBG_EINVAL, "classify: stride 0 without offsets");
  if (!d_off && static_cast<unsigned __int128>(n_pkts) * stride > (1ull << 40))
    return set_error(NBG_EINVAL, "classify: batch too large");
  DeviceGuard g(h->device);
  const bool group = d_perm || d_counts;
  if (group) {
    int rc = ensure_scratch(h, n_pkts);
    if (rc) return rc;
  }
  const bool lds = use_lds_lut(h, flags);
  const uint32_t n_tiles = static_cast<uint32_t>((n_pkts + kTile - 1) / kTile);
  int grid = std::min<int>(lds ? h->grid_lds : h->grid_global, static_cast<int>(n_tiles));

  ClassifyArgs a{};
  a.pkts = d_pkts;
  a.off = d_off;
  a.len = d_len;
  a.stride = stride;
  a.fixed_len = fixed_len;
  a.n_pkts = static_cast<uint32_t>(n_pkts);
  a.n_tiles = n_tiles;
  a.lut = h->d_lut;
  a.m = static_cast<uint32_t>(h->m);
  a.lut_lds_bytes = lds ? h->lut_bytes : 0;
  a.mu = ~0ull / h->m + ((~0ull % h->m) + 1 == h->m ? 1 : 0);  // floor(2^64 / m)
  a.nb = h->nb;
  a.swap = (flags & NBG_SWAP_MACS) ? 1u : 0u;
  a.backend = d_backend;
  if (group) {
    h->epoch = (h->epoch + 1) & 0x3fffffffu;
    if (h->epoch == 0) h->epoch = 1;
    a.desc = h->d_desc;
    a.tile_prefix = h->d_tile_prefix;
    a.group_base = h->d_group_base;
    a.counts = d_counts ? d_counts : h->d_counts;
    a.ticket = h->d_ticket;
    a.epoch = h->epoch;
    a.err = h->d_err;
  }
  int rc = launch_classify(a, h->wide, lds, grid, stream);
  if (rc) return rc;
  if (d_perm) {
    ScatterArgs s{};
    s.backend = d_backend;
    s.n_pkts = static_cast<uint32_t>(n_pkts);
    s.nb = h->nb;
    uint32_t bits = 0;
    while ((1u << bits) < h->nb + 1) ++bits;
    s.bits = bits;
    s.tile_prefix = h->d_tile_prefix;
    s.group_base = h->d_group_base;
    s.perm = d_perm;
    rc = launch_scatter(s, n_tiles, stream);
    if (rc) return rc;
  }
  h->last_stream = static_cast<hipStream_t>(stream);
  return NBG_OK;
}

int nbg_maglev_check(nbg_maglev* h) {
  if (!h) return set_error(NBG_EINVAL, "check: null handle");
  DeviceGuard g(h->device);
  NBG_HIP(hipStreamSynchronize(h->last_stream));
  uint32_t err = 0;
  NBG_HIP(hipMemcpy(&err, h->d_err, sizeof(err), hipMemcpyDeviceToHost));
  if (err) return set_error(NBG_ETIMEDOUT, "look-back spin limit reached (device flag %u)", err);
  return NBG_OK;
}

int nbg_maglev_classify_host(nbg_maglev* h, uint8_t* const* pkt_ptrs, const uint16_t* lens, uint64_t n,
                             uint32_t flags, uint16_t* backend_out, uint32_t* perm_out, uint32_t* counts_out) {
  if (!h || (!pkt_ptrs && n) || (!lens && n) || (!backend_out && n))
    return set_error(NBG_EINVAL, "classify_host: null argument");
  if (n >= (1ull << 30)) return set_error(NBG_EINVAL, "classify_host: n must be < 2^30");
  DeviceGuard g(h->device);
  if (!h->host_stream) NBG_HIP(hipStreamCreateWithFlags(&h->host_stream, hipStreamNonBlocking));
  if (n == 0) {
    if (counts_out) std::memset(counts_out, 0, (h->nb + 1) * sizeof(uint32_t));
    return NBG_OK;
  }
  // Header window per packet: bytes the path can read = 14 + max(20, 4*IHL + 4) <= 78.
  uint32_t need = 64;
  for (uint64_t i = 0; i < n; ++i) {
    if (lens[i] > 64 && lens[i] >= 15) {
      const uint32_t w = 14 + std::max<uint32_t>(20, (pkt_ptrs[i][14] & 0xfu) * 4 + 4);
      if (w > need) need = w;
    }
  }
  const uint32_t win = need <= 64 ? 64 : 80;
  if (n > h->host_cap || win != h->host_win) {
    free_host_path(h);
    const uint64_t cap = std::max<uint64_t>(n, 4096);
    NBG_HIP(hipHostMalloc(reinterpret_cast<void**>(&h->h_win), cap * win, hipHostMallocDefault));
    NBG_HIP(hipHostMalloc(reinterpret_cast<void**>(&h->h_len), cap * 2, hipHostMallocDefault));
    NBG_HIP(hipHostMalloc(reinterpret_cast<void**>(&h->h_mac), cap * 12, hipHostMallocDefault));
    NBG_HIP(hipMalloc(&h->d_win, cap * win));
    NBG_HIP(hipMalloc(&h->d_len, cap * 2));
    NBG_HIP(hipMalloc(&h->d_backend, cap * 2));
    NBG_HIP(hipMalloc(&h->d_perm, cap * 4));
    h->host_cap = cap;
    h->host_win = win;
  }
  for (uint64_t i = 0; i < n; ++i) {
    const uint32_t c = std::min<uint32_t>(lens[i], win);
    std::memcpy(h->h_win + i * win, pkt_ptrs[i], c);
    h->h_len[i] = lens[i];
  }
  hipStream_t s = h->host_stream;
  NBG_HIP(hipMemcpyAsync(h->d_win, h->h_win, n * win, hipMemcpyHostToDevice, s));
  NBG_HIP(hipMemcpyAsync(h->d_len, h->h_len, n * 2, hipMemcpyHostToDevice, s));
  uint32_t* d_counts = counts_out || perm_out ? h->d_counts : nullptr;
  int rc = nbg_maglev_classify_device(h, h->d_win, nullptr, h->d_len, win, 0, n, flags, h->d_backend,
                                      perm_out ? h->d_perm : nullptr, d_counts, s);
  if (rc) return rc;
  NBG_HIP(hipMemcpyAsync(backend_out, h->d_backend, n * 2, hipMemcpyDeviceToHost, s));
  if (perm_out) NBG_HIP(hipMemcpyAsync(perm_out, h->d_perm, n * 4, hipMemcpyDeviceToHost, s));
  if (counts_out) NBG_HIP(hipMemcpyAsync(counts_out, h->d_counts, (h->nb + 1) * 4, hipMemcpyDeviceToHost, s));
  const bool swap = flags & NBG_SWAP_MACS;
  if (swap) NBG_HIP(hipMemcpy2DAsync(h->h_mac, 12, h->d_win, win, 12, n, hipMemcpyDeviceToHost, s));
  NBG_HIP(hipStreamSynchronize(s));
  if (swap) {
    for (uint64_t i = 0; i < n; ++i)
      if (lens[i] >= 14) std::memcpy(pkt_ptrs[i], h->h_mac + i * 12, 12);
  }
  uint32_t err = 0;
  NBG_HIP(hipMemcpy(&err, h->d_err, sizeof(err), hipMemcpyDeviceToHost));
  if (err) return set_error(NBG_ETIMEDOUT, "look-back spin limit reached");
  return NBG_OK;
}

}  // extern "C"
