// Synthetic packet traces for tests and the benchmark (DESIGN.md "Synthetic traces").
//
// splitmix64 PRNG.  Flow table first (n_flows 5-tuples), then per packet a flow
// index and the frame bytes.  Frames are Ethernet II / IPv4 (IHL 5, valid header
// checksum) / UDP, like the 64-B UDP frames BASELINE.json's configs name.
#include <cstring>
#include <vector>

#include "nbgpu_internal.h"

namespace {

struct SplitMix {
  uint64_t s;
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
  }
};

struct Tuple {
  uint32_t src, dst;
  uint16_t sport, dport;
};

Tuple random_tuple(SplitMix& r) {
  Tuple t;
  t.src = 0x0A000000u | static_cast<uint32_t>(r.next() & 0xFFFFFFu);  // 10.0.0.0/8
  t.dst = 0xC0A80000u | static_cast<uint32_t>(r.next() & 0xFFFFu);    // 192.168.0.0/16
  t.sport = static_cast<uint16_t>(1024 + r.next() % 64512);             // [1024, 65535]
  t.dport = static_cast<uint16_t>(1 + r.next() % 65535);                // [1, 65535]
  return t;
}

inline void be16(uint8_t* p, uint32_t v) {
  p[0] = static_cast<uint8_t>(v >> 8);
  p[1] = static_cast<uint8_t>(v);
}
inline void be32(uint8_t* p, uint32_t v) {
  be16(p, v >> 16);
  be16(p + 2, v);
}

void write_frame(uint8_t* f, uint32_t len, const Tuple& t, uint32_t id, SplitMix& r) {
  static const uint8_t kEth[14] = {0x02, 0, 0, 0, 0, 0x01, 0x02, 0, 0, 0, 0, 0x02, 0x08, 0x00};
  std::memcpy(f, kEth, 14);
  uint8_t* ip = f + 14;
  ip[0] = 0x45;
  ip[1] = 0;
  be16(ip + 2, len - 14);
  be16(ip + 4, id & 0xFFFF);
  be16(ip + 6, 0x4000);  // DF
  ip[8] = 64;
  ip[9] = 17;  // UDP
  be16(ip + 10, 0);
  be32(ip + 12, t.src);
  be32(ip + 16, t.dst);
  uint32_t sum = 0;
  for (int k = 0; k < 20; k += 2) sum += (ip[k] << 8) | ip[k + 1];
  while (sum >> 16) sum = (sum & 0xFFFF) + (sum >> 16);
  be16(ip + 10, ~sum & 0xFFFF);
  uint8_t* udp = ip + 20;
  be16(udp, t.sport);
  be16(udp + 2, t.dport);
  be16(udp + 4, len - 34);
  be16(udp + 6, 0);
  for (uint32_t k = 42; k < len; k += 8) {
    const uint64_t v = r.next();
    const uint32_t c = len - k < 8 ? len - k : 8;
    std::memcpy(f + k, &v, c);
  }
}

}  // namespace

extern "C" uint64_t nbg_trace_layout(uint64_t n, int mode, uint64_t seed, uint32_t* off, uint16_t* len) {
  SplitMix r{seed ^ 0x1A7E5EEDULL};
  uint64_t pos = 0;
  for (uint64_t i = 0; i < n; ++i) {
    uint32_t l = 60;
    if (mode == 1) {  // IMIX 7:4:1 of 64/576/1500-B wire frames (FCS stripped)
      const uint64_t k = r.next() % 12;
      l = k < 7 ? 60 : (k < 11 ? 572 : 1496);
    }
    if (off) off[i] = static_cast<uint32_t>(pos);
    if (len) len[i] = static_cast<uint16_t>(l);
    pos += (l + 63) & ~63u;
  }
  return pos;
}

extern "C" int nbg_trace_fill(uint8_t* buf, const uint32_t* off, const uint16_t* len, uint64_t n, uint64_t seed,
                              uint32_t n_flows, uint32_t flags) {
  if (!buf || !off || !len) return nbg::set_error(NBG_EINVAL, "nbg_trace_fill: null argument");
  if (n_flows == 0) n_flows = 1;
  SplitMix r{seed};
  const bool unique = flags & NBG_TRACE_UNIQUE;
  std::vector<Tuple> flows;
  if (!unique) {
    flows.resize(n_flows);
    for (auto& t : flows) t = random_tuple(r);
  }
  for (uint64_t i = 0; i < n; ++i) {
    const Tuple t = unique ? random_tuple(r) : flows[r.next() % n_flows];
    uint8_t* f = buf + off[i];
    const uint32_t l = len[i];
    const uint32_t slot = (l + 63) & ~63u;
    write_frame(f, l, t, static_cast<uint32_t>(i), r);
    std::memset(f + l, 0, slot - l);
  }
  return NBG_OK;
}
