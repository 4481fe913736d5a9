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

// Kernel geometry shared by the classify and scatter kernels.
constexpr int kBlock = 256;          // threads per workgroup (4 waves)
constexpr int kPktsPerThread = 4;    // packets per thread per tile
constexpr int kTile = kBlock * kPktsPerThread;  // packets per tile (look-back unit)

struct ClassifyArgs {
  uint8_t* pkts;
  const uint32_t* off;      // nullable
  const uint16_t* len;      // nullable
  uint32_t stride;
  uint32_t fixed_len;
  uint32_t n_pkts;
  uint32_t n_tiles;
  const void* lut;          // u8 or u16 entries
  uint32_t m;               // table size
  uint32_t lut_lds_bytes;   // bytes of LUT staged in LDS (0 = global gather)
  uint64_t mu;              // floor(2^64 / m) for Barrett
  uint32_t nb;              // backends; bins = nb + 1 (sentinel bin = nb)
  uint32_t swap;
  uint16_t* backend;
  // grouping (nullable when no perm requested)
  unsigned long long* desc;   // [n_tiles][nb+1] look-back words
  uint32_t* tile_prefix;      // [n_tiles][nb+1] exclusive prefix over earlier tiles
  uint32_t* group_base;       // [nb+1] exclusive prefix over groups
  uint32_t* counts;           // [nb+1]
  unsigned long long* ticket; // [0] tile ticket, [1] exit count; reset by the last block
  uint32_t epoch;
  uint32_t* err;
};

struct ScatterArgs {
  const uint16_t* backend;
  uint32_t n_pkts;
  uint32_t nb;
  uint32_t bits;              // ceil(log2(nb+1))
  const uint32_t* tile_prefix;
  const uint32_t* group_base;
  uint32_t* perm;
};

// Launchers (maglev_kernels.hip).  `wide_lut` = u16 entries; `lds_lut` = stage in LDS.
int launch_classify(const ClassifyArgs& a, bool wide_lut, bool lds_lut, int grid, void* stream);
int launch_scatter(const ScatterArgs& a, uint32_t n_tiles, void* stream);
int max_classify_grid(bool wide_lut, bool lds_lut, uint32_t lds_bytes, int device, int* grid);

}  // namespace nbg
