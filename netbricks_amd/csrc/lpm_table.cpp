// DIR-24-8 LPM table builder: the product restatement of test/lpm's IPLookup.
//
//   IPLookup::default / insert / construct_table   test/lpm/src/nf.rs:24-86
//   lookup_entry                                   test/lpm/src/nf.rs:88-98
//
// tbl24 has TBL24_SIZE = 2^24 + 1 u16 entries (nf.rs:19).  A route of length <= 24 fills
// tbl24[(k >> 8) .. (k >> 8) + 2^(24-len)) with its gate; the start is NOT masked to the
// prefix (nf.rs:52-53), which this restatement keeps.  Longer routes get a 256-entry block
// of tbl_long (also 2^24 + 1 entries in the reference), marked in tbl24 with
// OVERFLOW_MASK | (block >> 8) truncated to u16 (nf.rs:75).  Lengths are processed
// 0..=32 in order; inside one length the reference iterates a HashMap (nf.rs:51,60), whose
// order is not reproducible outside Rust — routes of one length are applied here in
// ascending prefix order, which gives the reference's lookup results whenever routes of one
// length do not overlap with different gates (always true for masked prefixes).
#include <cstring>
#include <map>
#include <vector>

#include "nbgpu_internal.h"

namespace nbg {

int build_lpm(const uint32_t* prefixes, const uint8_t* lens, const uint16_t* gates, uint64_t n,
              std::vector<uint16_t>& tbl24, std::vector<uint16_t>& tbl_long, uint64_t& long_used) {
  constexpr uint64_t kTbl24 = (1ull << 24) + 1;  // TBL24_SIZE (nf.rs:19)
  constexpr uint16_t kOverflow = 0x8000;          // OVERFLOW_MASK (nf.rs:21)
  std::vector<std::map<uint32_t, uint16_t>> raw(33);  // RAW_SIZE = 33 (nf.rs:20)
  for (uint64_t i = 0; i < n; ++i) {
    if (lens[i] > 32) return set_error(NBG_EINVAL, "lpm: route %llu has length %u > 32", (unsigned long long)i, lens[i]);
    raw[lens[i]][prefixes[i]] = gates[i];  // HashMap::insert replaces (nf.rs:46)
  }
  tbl24.assign(kTbl24, 0);
  tbl_long.assign(kTbl24, 0);
  uint64_t cur = 0;  // current_tbl_long
  for (uint32_t len = 0; len <= 24; ++len) {
    for (const auto& kv : raw[len]) {
      const uint64_t start = kv.first >> 8, end = start + (1ull << (24 - len));
      if (end > kTbl24)
        return set_error(NBG_EINVAL, "lpm: /%u route %08x fills tbl24 past its end (reference panics)", len, kv.first);
      for (uint64_t p = start; p < end; ++p) tbl24[p] = kv.second;
    }
  }
  for (uint32_t len = 25; len <= 32; ++len) {
    for (const auto& kv : raw[len]) {
      const uint64_t addr = kv.first;
      const uint16_t t24 = tbl24[addr >> 8];
      if ((t24 & kOverflow) == 0) {
        if (cur + 256 > kTbl24) return set_error(NBG_EINVAL, "lpm: tbl_long exhausted (reference panics)");
        const uint64_t start = cur + (addr & 0xff), end = start + (1ull << (32 - len));
        for (uint64_t j = cur; j < cur + 256; ++j) tbl_long[j] = (j < start || j >= end) ? t24 : kv.second;
        tbl24[addr >> 8] = static_cast<uint16_t>(static_cast<uint16_t>(cur >> 8) | kOverflow);
        cur += 256;
      } else {
        const uint64_t start = (static_cast<uint64_t>(t24 & ~kOverflow) << 8) + (addr & 0xff);
        const uint64_t end = start + (1ull << (32 - len));
        if (end > kTbl24) return set_error(NBG_EINVAL, "lpm: /%u route %08x writes past tbl_long", len, kv.first);
        for (uint64_t j = start; j < end; ++j) tbl_long[j] = kv.second;
      }
    }
  }
  long_used = cur;
  return NBG_OK;
}

}  // namespace nbg

extern "C" int nbg_lpm_build_host(const uint32_t* prefixes, const uint8_t* lens, const uint16_t* gates, uint64_t n,
                                  uint16_t* tbl24, uint16_t* tbl_long, uint64_t long_cap, uint64_t* long_used) {
  if ((!prefixes || !lens || !gates) && n) return nbg::set_error(NBG_EINVAL, "nbg_lpm_build_host: null argument");
  if (!tbl24 || !long_used) return nbg::set_error(NBG_EINVAL, "nbg_lpm_build_host: null output");
  std::vector<uint16_t> t24, tl;
  uint64_t used = 0;
  const int rc = nbg::build_lpm(prefixes, lens, gates, n, t24, tl, used);
  if (rc) return rc;
  *long_used = used;
  if (used > long_cap || (used && !tbl_long))
    return nbg::set_error(NBG_EINVAL, "nbg_lpm_build_host: tbl_long needs %llu entries", (unsigned long long)used);
  std::memcpy(tbl24, t24.data(), t24.size() * sizeof(uint16_t));
  if (used) std::memcpy(tbl_long, tl.data(), used * sizeof(uint16_t));
  return NBG_OK;
}
