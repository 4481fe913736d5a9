// A pcap-file port: the `dpdk:eth_pcap0,rx_pcap=...,tx_pcap=...` PMD that the reference's
// example NFs use for testing (test/macswap/check.sh:3, README "Example NFs").  recv() hands
// out the capture's frames in bursts; send() appends frames to the output capture.
#pragma once

#include <sys/mman.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "operators.hpp"

namespace nb {

struct PcapRecord {
  uint32_t ts_sec = 0, ts_usec = 0;
  std::vector<uint8_t> data;
};

inline std::vector<PcapRecord> read_pcap(const std::string& path) {
  std::vector<PcapRecord> out;
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("cannot open " + path);
  uint32_t gh[6];
  if (std::fread(gh, 4, 6, f) != 6 || (gh[0] != 0xA1B2C3D4u && gh[0] != 0xA1B23C4Du)) {
    std::fclose(f);
    throw std::runtime_error("not a little-endian pcap: " + path);
  }
  uint32_t rh[4];
  while (std::fread(rh, 4, 4, f) == 4) {
    PcapRecord r;
    r.ts_sec = rh[0];
    r.ts_usec = rh[1];
    r.data.resize(rh[2]);
    if (rh[2] && std::fread(r.data.data(), 1, rh[2], f) != rh[2]) break;
    out.push_back(std::move(r));
  }
  std::fclose(f);
  return out;
}

inline void write_pcap(const std::string& path, const std::vector<PcapRecord>& recs) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) throw std::runtime_error("cannot create " + path);
  const uint32_t gh[6] = {0xA1B2C3D4u, 0x00040002u, 0, 0, 65535, 1 /* LINKTYPE_ETHERNET */};
  std::fwrite(gh, 4, 6, f);
  for (auto& r : recs) {
    const uint32_t rh[4] = {r.ts_sec, r.ts_usec, static_cast<uint32_t>(r.data.size()),
                            static_cast<uint32_t>(r.data.size())};
    std::fwrite(rh, 4, 4, f);
    std::fwrite(r.data.data(), 1, r.data.size(), f);
  }
  std::fclose(f);
}

// One port with an rx capture (consumed once) and a tx capture (collected in send order).
class PcapPort : public PacketRx, public PacketTx {
 public:
  // The frames live in one contiguous mempool of fixed data rooms (as a DPDK mempool's do), so the
  // pool can be registered for zero-copy GPU access (mempool() + nbg_host_register).
  explicit PcapPort(const std::string& rx_path, uint32_t data_room = 2048) {
    auto recs = read_pcap(rx_path);
    room_ = data_room;
    for (auto& r : recs) room_ = std::max<size_t>(room_, (r.data.size() + 63) & ~size_t{63});
    mem_.assign(recs.size() * room_ + 4096, 0);
    base_ = mem_.data() + ((4096 - reinterpret_cast<uintptr_t>(mem_.data()) % 4096) % 4096);  // page-aligned
    uint8_t* base = base_;
    size_t tx_room = 0;
    for (auto& r : recs) {
      auto m = std::make_unique<MBuf>();
      m->room = base + pool_.size() * room_;
      std::memcpy(m->room, r.data.data(), r.data.size());
      m->data_len = static_cast<uint16_t>(r.data.size());
      m->port_seq = pool_.size();
      ts_.push_back({r.ts_sec, r.ts_usec});
      pool_.push_back(std::move(m));
      tx_room += 16 + r.data.size();
    }
    tx_bytes_.assign(tx_room, 0);
    tx_index_.reserve(pool_.size());
  }
  // the mempool's memory: every frame's data room lies in [data, data + bytes)
  std::pair<uint8_t*, size_t> mempool() { return {base_, pool_.size() * room_}; }
  uint32_t recv(MBuf** pkts, uint32_t cap) override {
    uint32_t n = 0;
    while (n < cap && next_ < pool_.size()) pkts[n++] = pool_[next_++].get();
    return n;
  }
  // Appends each frame, with its pcap record header, to one dump buffer (the pcap PMD's
  // pcap_dump into a stdio buffer); write_tx() puts the buffer behind a pcap file header.
  uint32_t send(MBuf** pkts, uint32_t n) override {
    // The buffer is sized and touched for one copy of the rx capture up front (outside any timed
    // loop); sending more than that grows it.
    size_t add = 0;
    for (uint32_t i = 0; i < n; ++i) add += 16 + pkts[i]->data_len;
    if (tx_used_ + add > tx_bytes_.size()) tx_bytes_.resize(std::max(2 * tx_bytes_.size(), tx_used_ + add));
    uint8_t* out = tx_bytes_.data() + tx_used_;
    for (uint32_t i = 0; i < n; ++i) {
      const uint32_t len = pkts[i]->data_len;
      const uint32_t rh[4] = {0, 0, len, len};
      std::memcpy(out, rh, 16);
      std::memcpy(out + 16, pkts[i]->data(), len);
      out += 16 + len;
      tx_index_.push_back(pkts[i]->port_seq);
    }
    tx_used_ += add;
    return n;
  }
  void write_tx(const std::string& path) const {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot create " + path);
    const uint32_t gh[6] = {0xA1B2C3D4u, 0x00040002u, 0, 0, 65535, 1 /* LINKTYPE_ETHERNET */};
    std::fwrite(gh, 4, 6, f);
    std::fwrite(tx_bytes_.data(), 1, tx_used_, f);
    std::fclose(f);
  }
  bool rx_done() const { return next_ >= pool_.size(); }
  size_t rx_total() const { return pool_.size(); }
  const std::vector<size_t>& tx_index() const { return tx_index_; }  // rx position of each sent frame

 private:
  std::vector<uint8_t> mem_;
  uint8_t* base_ = nullptr;
  size_t room_ = 2048;
  std::vector<std::unique_ptr<MBuf>> pool_;
  std::vector<std::pair<uint32_t, uint32_t>> ts_;
  size_t next_ = 0;
  std::vector<uint8_t> tx_bytes_;
  size_t tx_used_ = 0;
  std::vector<size_t> tx_index_;
};

// A replay port for throughput runs: the reference's VirtualPort (interface/port/virt_port.rs:27-52:
// recv hands out mbufs, send frees them) over a capture's frames.  The frames are copied into one
// mempool of at least min_pool mbufs (the capture repeated; 2-KiB data rooms, as DPDK's); recv hands
// out free mbufs in pool order until `total` packets were received, send returns them to the pool
// (the free list is FIFO, so a frame is received again only after it was sent).
class LoopPort : public PacketRx, public PacketTx {
 public:
  // huge: the mempool in 2-MiB transparent huge pages, as a DPDK mempool lives in hugepages (for the
  // GPU's reads of a registered pool, and the host's, one TLB entry per 2 MiB instead of per 4 KiB)
  // object: the stride of the pool's objects (0: the data room itself).  A DPDK mempool object is
  // larger than its data room (the 128-B rte_mbuf, 128 B of headroom, the mempool's own header) and
  // rte_mempool pads objects so that consecutive ones do not start on the same cache sets; a stride
  // of exactly 2 KiB would put every frame's first line into 1/32 of the L2's sets.
  LoopPort(const std::vector<PcapRecord>& recs, uint64_t total, size_t min_pool = 65536, uint32_t data_room = 2048,
           bool huge = true, uint32_t object = 0)
      : total_(total) {
    if (recs.empty()) throw std::invalid_argument("LoopPort: empty capture");
    room_ = data_room;
    for (auto& r : recs) room_ = std::max<size_t>(room_, (r.data.size() + 63) & ~size_t{63});
    if (object) room_ = std::max<size_t>(room_, (object + 63) & ~size_t{63});
    const size_t n = (std::max(min_pool, recs.size()) + recs.size() - 1) / recs.size() * recs.size();
    constexpr size_t kHuge = 2u << 20;
    map_bytes_ = (n * room_ + 2 * kHuge - 1) / kHuge * kHuge;
    void* m = mmap(nullptr, map_bytes_, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (m == MAP_FAILED) throw std::runtime_error("LoopPort: mmap of the mempool failed");
    map_ = static_cast<uint8_t*>(m);
    base_ = map_ + (kHuge - reinterpret_cast<uintptr_t>(map_) % kHuge) % kHuge;  // 2-MiB aligned
    if (huge) huge_ = madvise(base_, static_cast<size_t>(map_ + map_bytes_ - base_) / kHuge * kHuge, MADV_HUGEPAGE) == 0;
    pool_.resize(n);
    free_.resize(n);
    for (size_t i = 0; i < n; ++i) {
      const auto& r = recs[i % recs.size()];
      MBuf& m = pool_[i];
      m.room = base_ + i * room_;
      std::memcpy(m.room, r.data.data(), r.data.size());
      m.data_len = static_cast<uint16_t>(r.data.size());
      m.port_seq = i;
      free_[i] = &m;
    }
    tail_ = n;
  }
  ~LoopPort() override {
    if (map_) munmap(map_, map_bytes_);
  }
  LoopPort(const LoopPort&) = delete;
  LoopPort& operator=(const LoopPort&) = delete;
  std::pair<uint8_t*, size_t> mempool() { return {base_, pool_.size() * room_}; }
  bool huge_pages() const { return huge_; }
  uint32_t recv(MBuf** pkts, uint32_t cap) override {
    uint32_t n = 0;
    while (n < cap && received_ < total_ && head_ != tail_) {
      pkts[n++] = free_[head_++ % free_.size()];
      ++received_;
    }
    return n;
  }
  uint32_t send(MBuf** pkts, uint32_t n) override {  // rte_eth_tx_burst + the NIC freeing the mbufs
    for (uint32_t i = 0; i < n; ++i) {
      MBuf::write_metadata_slot(pkts[i], kHeaderSlot, 0);
      free_[tail_++ % free_.size()] = pkts[i];
    }
    sent_ += n;
    return n;
  }
  bool rx_done() const { return received_ >= total_; }
  uint64_t rx_total() const { return received_; }
  uint64_t tx_total() const { return sent_; }
  size_t pool_size() const { return pool_.size(); }

 private:
  uint64_t total_, received_ = 0, sent_ = 0;
  uint8_t* map_ = nullptr;
  size_t map_bytes_ = 0;
  bool huge_ = false;
  uint8_t* base_ = nullptr;
  size_t room_ = 2048;
  std::vector<MBuf> pool_;
  std::vector<MBuf*> free_;  // ring: [head_, tail_) are free
  uint64_t head_ = 0, tail_ = 0;
};

}  // namespace nb
