// Host-side Maglev LUT construction (control plane, once per backend set).
//
// Restates Maglev::new (test/maglev/src/nf.rs:70-76):
//   offset_skip_for_name  nf.rs:21-31  offset = XXH64(name||0xFF, 0) % M,
//                                      skip   = FNV1a64(name||0xFF) % (M-1) + 1
//   generate_permutations nf.rs:33-42  perm[i][j] = (offset_i + j*skip_i) % M
//   generate_lut          nf.rs:44-68  round-robin fill with the 0x8000 "empty" sentinel
// The reference materialises N x M usize permutations (5.2 GB at N=1000, M=655373);
// here a permutation entry is evaluated on demand, so memory is O(M).
//
// The hashers are the `fnv` crate's FnvHasher and twox-hash 1.x `XxHash` (seed 0);
// Rust's `impl Hash for str` writes the bytes and then one 0xFF byte.
#include "nbgpu_internal.h"

#include <cstring>
#include <vector>

namespace nbg {

namespace {

constexpr uint64_t kP1 = 0x9E3779B185EBCA87ULL;
constexpr uint64_t kP2 = 0xC2B2AE3D27D4EB4FULL;
constexpr uint64_t kP3 = 0x165667B19E3779F9ULL;
constexpr uint64_t kP4 = 0x85EBCA77C2B2AE63ULL;
constexpr uint64_t kP5 = 0x27D4EB2F165667C5ULL;

inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
inline uint64_t rd64(const uint8_t* p) { uint64_t v; std::memcpy(&v, p, 8); return v; }
inline uint32_t rd32(const uint8_t* p) { uint32_t v; std::memcpy(&v, p, 4); return v; }
inline uint64_t xround(uint64_t acc, uint64_t in) { return rotl(acc + in * kP2, 31) * kP1; }
inline uint64_t xmerge(uint64_t acc, uint64_t v) { return (acc ^ xround(0, v)) * kP1 + kP4; }

}  // namespace

uint64_t fnv1a64(const uint8_t* p, size_t n) {
  uint64_t h = 0xcbf29ce484222325ULL;
  for (size_t i = 0; i < n; ++i) {
    h ^= p[i];
    h *= 0x100000001b3ULL;
  }
  return h;
}

// XXH64 (published xxHash algorithm, little-endian input reads).
uint64_t xxh64(const uint8_t* p, size_t n, uint64_t seed) {
  const uint8_t* end = p + n;
  uint64_t h;
  if (n >= 32) {
    uint64_t v1 = seed + kP1 + kP2, v2 = seed + kP2, v3 = seed, v4 = seed - kP1;
    const uint8_t* limit = end - 32;
    do {
      v1 = xround(v1, rd64(p));
      v2 = xround(v2, rd64(p + 8));
      v3 = xround(v3, rd64(p + 16));
      v4 = xround(v4, rd64(p + 24));
      p += 32;
    } while (p <= limit);
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    h = xmerge(h, v1);
    h = xmerge(h, v2);
    h = xmerge(h, v3);
    h = xmerge(h, v4);
  } else {
    h = seed + kP5;
  }
  h += static_cast<uint64_t>(n);
  while (p + 8 <= end) {
    h ^= xround(0, rd64(p));
    h = rotl(h, 27) * kP1 + kP4;
    p += 8;
  }
  if (p + 4 <= end) {
    h ^= static_cast<uint64_t>(rd32(p)) * kP1;
    h = rotl(h, 23) * kP2 + kP3;
    p += 4;
  }
  while (p < end) {
    h ^= (*p) * kP5;
    h = rotl(h, 11) * kP1;
    ++p;
  }
  h ^= h >> 33;
  h *= kP2;
  h ^= h >> 29;
  h *= kP3;
  h ^= h >> 32;
  return h;
}

int build_lut(const char* const* names, const uint32_t* lens, uint32_t n, uint64_t m, std::vector<uint32_t>& entry) {
  if (n == 0 || m < 2) return set_error(NBG_EINVAL, "maglev: need >=1 backend and table_size >= 2");
  std::vector<uint64_t> offset(n), skip(n), next(n, 0);
  std::vector<uint8_t> buf;
  for (uint32_t i = 0; i < n; ++i) {
    if (!names[i] && lens[i]) return set_error(NBG_EINVAL, "maglev: null backend name");
    buf.assign(names[i], names[i] + lens[i]);
    buf.push_back(0xff);  // Rust `str: Hash` terminator byte
    offset[i] = xxh64(buf.data(), buf.size(), 0) % m;
    skip[i] = fnv1a64(buf.data(), buf.size()) % (m - 1) + 1;
  }
  constexpr uint32_t kEmpty = 0x8000;  // nf.rs:46
  entry.assign(m, kEmpty);
  // (offset + j*skip) % M without overflow: keep c and step modulo M.
  std::vector<uint64_t> cur(n);
  for (uint32_t i = 0; i < n; ++i) cur[i] = offset[i];
  auto advance = [&](uint32_t i) {
    ++next[i];
    cur[i] += skip[i];
    if (cur[i] >= m) cur[i] -= m;
  };
  uint64_t filled = 0;
  while (filled < m) {
    for (uint32_t i = 0; i < n; ++i) {
      while (entry[cur[i]] != kEmpty) {
        advance(i);
        // permutations[i][m] would be out of bounds: the reference panics (nf.rs:52-54)
        if (next[i] >= m)
          return set_error(NBG_EINVAL, "maglev: permutation of backend %u exhausted (table size %llu not coprime "
                           "to its skip; use a prime table size)", i, (unsigned long long)m);
      }
      if (entry[cur[i]] == kEmpty) {
        entry[cur[i]] = i;
        advance(i);
        ++filled;
      }
      if (filled >= m) break;
    }
  }
  return NBG_OK;
}

}  // namespace nbg

extern "C" int nbg_lut_build_host(const char* const* names, const uint32_t* name_lens, uint32_t n_backends,
                                  uint64_t table_size, uint16_t* out) {
  if (!names || !name_lens || !out) return nbg::set_error(NBG_EINVAL, "nbg_lut_build_host: null argument");
  if (n_backends > 65534) return nbg::set_error(NBG_EINVAL, "nbg_lut_build_host: n_backends > 65534");
  std::vector<uint32_t> e;
  int rc = nbg::build_lut(names, name_lens, n_backends, table_size, e);
  if (rc) return rc;
  for (uint64_t j = 0; j < table_size; ++j) out[j] = static_cast<uint16_t>(e[j]);
  return NBG_OK;
}
