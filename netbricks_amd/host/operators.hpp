// Host-side mirror of the NetBricks batch-operator surface for the Maglev path, backed by
// the MI355X C-ABI (include/nbgpu.h).  Same names and meaning as the reference:
//
//   ReceiveBatch::new(port)          framework/src/operators/receive_batch.rs:9-98
//   .parse::<MacHeader>()            framework/src/operators/mod.rs:59-64, parsed_batch.rs
//   .transform(swap_addresses)       framework/src/operators/transform_batch.rs:11-118
//   .group_by(ct, group_fn, sched)   framework/src/operators/group_by.rs:13-113
//   GroupBy::get_group(i)            group_by.rs:102-112 (+ RestoreHeader, restore_header.rs)
//   merge(batches)                   framework/src/operators/merge_batch.rs:10-111
//   .compose() / .send(port)         composition_batch.rs:13-60, send_batch.rs:10-125
//   MpscQueue (1024 slots)           framework/src/queues/mpsc_mbuf_queue.rs:22-265
//   StandaloneScheduler              framework/src/scheduler/standalone_scheduler.rs:127-158
//
// The per-packet closures of test/maglev (nf.rs:94-106) cannot cross an FFI boundary per
// packet, so the transform and group functions of this path are *descriptors* (MacSwap,
// MaglevGroup) that the GPU group_by recognises: its producer task accumulates received
// bursts into one batch, submits parse + swap + flow hash + LUT lookup + stable grouping as one
// nbg_maglev_host_submit (up to NBG_HOST_SLOTS batches in flight), and enqueues each finished
// batch's mbufs into the per-group FIFOs in arrival order — exactly what GroupByProducer::execute
// (group_by.rs:43-55) does packet by packet.
#pragma once

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <functional>
#include <memory>
#include <numeric>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#if defined(__x86_64__)
#include <x86intrin.h>
#endif

#include "../../include/nbgpu.h"

namespace nb {

// ---- timing -------------------------------------------------------------------------------
// The throughput runs time every scheduler task and producer phase, hundreds of reads per 992-packet
// batch (a consumer execution moves one burst of one group), so the read itself must be cheap: the
// invariant TSC on x86-64 (one instruction, ~10-20 ns against ~20-40 for steady_clock::now, measured),
// converted with a rate calibrated once against steady_clock.
struct TscClock {
  using tick = uint64_t;
  static tick now() {
#if defined(__x86_64__)
    return __rdtsc();
#else
    return static_cast<tick>(std::chrono::steady_clock::now().time_since_epoch().count());
#endif
  }
  static double seconds_per_tick() {
    static const double spt = [] {
#if defined(__x86_64__)
      const auto c0 = std::chrono::steady_clock::now();
      const tick t0 = now();
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
      const tick t1 = now();
      const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - c0).count();
      return s / static_cast<double>(t1 - t0);
#else
      return static_cast<double>(std::chrono::steady_clock::period::num) / std::chrono::steady_clock::period::den;
#endif
    }();
    return spt;
  }
  static double since(tick t0) { return static_cast<double>(now() - t0) * seconds_per_tick(); }
};

// ---- packets ----------------------------------------------------------------------------
// Stand-in for rte_mbuf: data pointer + data_len + the metadata slots NetBricks uses to save the
// parsed header and offset (interface/packet.rs:54-57: HEADER_SLOT 0, OFFSET_SLOT 1).
constexpr size_t kHeaderSlot = 0, kOffsetSlot = 1;
struct MBuf {
  std::vector<uint8_t> storage;  // data room (DPDK: >= 2 KiB, so 64-B windows are owned)
  uint8_t* room = nullptr;       // or a data room inside a port's mempool (then storage is empty)
  uint16_t data_len = 0;
  uintptr_t meta[2] = {0, 0};    // HEADER_SLOT, OFFSET_SLOT
  uint64_t port_seq = 0;         // position in the receiving port's stream (bookkeeping)
  uint8_t* data() { return room ? room : storage.data(); }
  uint8_t* data_address(size_t off) { return data() + off; }  // native/zcsi/mbuf.rs:34-37
  // native/zcsi/mbuf.rs:8-21
  static uintptr_t read_metadata_slot(const MBuf* m, size_t slot) { return m->meta[slot]; }
  static void write_metadata_slot(MBuf* m, size_t slot, uintptr_t v) { m->meta[slot] = v; }
};

// Packet<MacHeader, _>: the MAC header view a consumer gets back (interface/packet.rs:22-30).
struct MacPacket {
  MBuf* mbuf;
  uint8_t* header;  // the MAC header (dst 0..5, src 6..11, ethertype 12..13)
  size_t offset;    // the header's offset from the data start
  uint8_t* payload() const { return header + 14; }  // MacHeader::offset() == 14 (headers/mac.rs:96-106)
};

// Packet::save_header_and_offset (interface/packet.rs:211-221) of the packet that
// parse::<MacHeader>() makes from a received mbuf: the header is the data start and its offset is 0
// (ReceiveBatch packets start at offset 0, packet_batch.rs:233; parse_header sets
// offset = self.offset() + NullHeader::offset() = 0, packet.rs:392-399, null_header.rs:18-20).
inline void save_header_and_offset(MBuf* m) {
  MBuf::write_metadata_slot(m, kHeaderSlot, reinterpret_cast<uintptr_t>(m->data_address(0)));
  MBuf::write_metadata_slot(m, kOffsetSlot, 0);
}

// Packet::restore_saved_header (interface/packet.rs:414-424): None when the header slot is null.
inline bool restore_saved_header(MBuf* m, MacPacket* out) {
  const uintptr_t hdr = MBuf::read_metadata_slot(m, kHeaderSlot);
  if (hdr == 0) return false;
  *out = MacPacket{m, reinterpret_cast<uint8_t*>(hdr), MBuf::read_metadata_slot(m, kOffsetSlot)};
  return true;
}

struct PacketRx {  // interface/mod.rs:11-13
  virtual ~PacketRx() = default;
  virtual uint32_t recv(MBuf** pkts, uint32_t cap) = 0;
};
struct PacketTx {  // interface/mod.rs:15-17
  virtual ~PacketTx() = default;
  virtual uint32_t send(MBuf** pkts, uint32_t n) = 0;
};

class NbError : public std::runtime_error {
 public:
  NbError(int code, const std::string& what) : std::runtime_error(what), code(code) {}
  int code;
};

inline void check(int rc, const char* where) {
  if (rc != NBG_OK) throw NbError(rc, std::string(where) + ": " + nbg_last_error());
}

// ---- queues -------------------------------------------------------------------------------
// Single-producer ring of mbuf pointers with the reference's capacity rule (mask + tail - head,
// mpsc_mbuf_queue.rs:91-115): a full queue refuses the packet and the producer drops it.
class MpscQueue {
 public:
  explicit MpscQueue(uint32_t size = 1024) : ring_(size), mask_(size - 1) {
    if (size & (size - 1)) throw std::invalid_argument("queue size must be a power of two");
  }
  bool enqueue_one(MBuf* m) {
    if (mask_ + tail_ - head_ == 0) return false;  // free slots = mask + consumer_tail - producer_head
    ring_[head_++ & mask_] = m;
    return true;
  }
  uint32_t dequeue(MBuf** out, uint32_t cap) {  // mpsc_mbuf_queue.rs:197-212
    uint32_t n = 0;
    while (n < cap && tail_ != head_) out[n++] = ring_[tail_++ & mask_];
    return n;
  }
  uint64_t size() const { return head_ - tail_; }
  uint64_t free_slots() const { return mask_ + tail_ - head_; }

 private:
  std::vector<MBuf*> ring_;
  uint64_t mask_, head_ = 0, tail_ = 0;
};

// ---- scheduler ----------------------------------------------------------------------------
struct Executable {  // scheduler/mod.rs: trait Executable
  virtual ~Executable() = default;
  virtual void execute() = 0;
};

// Run-to-completion round robin over tasks (standalone_scheduler.rs:127-158).
class StandaloneScheduler {
 public:
  size_t add_task(std::shared_ptr<Executable> t) {
    tasks_.push_back(std::move(t));
    return tasks_.size() - 1;
  }
  void execute_round() {
    if (!timed_) {
      for (auto& t : tasks_) t->execute();
      return;
    }
    ticks_.resize(tasks_.size());
    for (size_t i = 0; i < tasks_.size(); ++i) {
      const TscClock::tick t0 = TscClock::now();
      tasks_[i]->execute();
      ticks_[i] += TscClock::now() - t0;
    }
  }
  // per-task wall time accumulated over execute_round() (for throughput breakdowns; off by default)
  void set_timed(bool on) {
    if (on) TscClock::seconds_per_tick();  // calibrated before the run, not inside it
    timed_ = on;
  }
  double task_seconds(size_t i) const {
    return i < ticks_.size() ? static_cast<double>(ticks_[i]) * TscClock::seconds_per_tick() : 0.0;
  }

 private:
  std::vector<std::shared_ptr<Executable>> tasks_;
  std::vector<TscClock::tick> ticks_;
  bool timed_ = false;
};

// ---- batches ------------------------------------------------------------------------------
constexpr uint32_t kBurst = 32;  // ReceiveBatch::new -> PacketBatch::new(32), receive_batch.rs:26

// A batch source: act() fills `pkts`, done() releases them (the Act trait, operators/act.rs).
struct Batch {
  virtual ~Batch() = default;
  virtual void act() = 0;
  virtual void done() = 0;
  std::vector<MBuf*> pkts;
};

struct ReceiveBatch : Batch {  // receive_batch.rs:9-98
  explicit ReceiveBatch(std::shared_ptr<PacketRx> q) : queue(std::move(q)) {}
  void act() override {
    pkts.resize(kBurst);
    pkts.resize(queue->recv(pkts.data(), kBurst));
    received += pkts.size();
  }
  void done() override { pkts.clear(); }
  std::shared_ptr<PacketRx> queue;
  uint64_t received = 0;
};

struct MacHeader {};  // headers/mac.rs:69-75; offset() == 14 under feature "performance"
struct MacSwap {};    // MacHeader::swap_addresses (mac.rs:140-145) as a transform descriptor

// ParsedBatch<MacHeader> (parsed_batch.rs) + TransformBatch(MacSwap): on this path both are
// folded into the group_by kernel, so the chain only records what to apply.
struct ParsedMacBatch {
  std::shared_ptr<Batch> parent;
  bool swap = false;
};

inline ParsedMacBatch parse_mac(std::shared_ptr<Batch> parent) { return ParsedMacBatch{std::move(parent), false}; }
inline ParsedMacBatch transform(ParsedMacBatch p, MacSwap) {
  p.swap = true;
  return p;
}

// RestoreHeader (operators/restore_header.rs:9-67) over a group's consumer batch: every received
// mbuf gets its saved header back; a null header slot is the reference's `.unwrap()` panic
// (restore_header.rs:64), thrown here as NbError.
struct RestoreHeader : Batch {
  explicit RestoreHeader(std::shared_ptr<Batch> p) : parent(std::move(p)) {}
  void act() override {
    parent->act();
    pkts = parent->pkts;
    packets.resize(pkts.size());
    for (size_t i = 0; i < pkts.size(); ++i)
      if (!restore_saved_header(pkts[i], &packets[i]))
        throw NbError(NBG_EINVAL, "RestoreHeader: null saved header (restore_header.rs:64 unwrap)");
  }
  void done() override {
    parent->done();
    pkts.clear();
    packets.clear();
  }
  std::shared_ptr<Batch> parent;
  std::vector<MacPacket> packets;
};

// The enqueue half of GroupByProducer::execute (group_by.rs:46-51) for a whole classified batch —
// the same steps, in the same order, as the Rust GpuMaglevProducer in INTEGRATION.md: walk the
// groups in perm order; a would-panic packet (group ct = queues.size(): the reference panics on
// it) is freed, never enqueued; every other packet gets save_header_and_offset and then
// enqueue_one into its group's queue, where a full queue loses it (mpsc_mbuf_queue.rs:91-115).
struct EnqueueStats {
  uint64_t dropped = 0, would_panic = 0, stalls = 0;
};
// Where the enqueue of a classified batch stands: group g, its j-th packet, perm position k.
struct EnqueueCursor {
  size_t g = 0, k = 0;
  uint32_t j = 0;
};
// Enqueue from `c` on.  stall = false: a full queue loses the packet (the reference), and the batch
// always completes.  stall = true (backpressure): the enqueue stops at the first packet whose queue is
// full and returns false; the next call resumes there (per-group FIFO order holds: nothing behind the
// stopped packet is enqueued before it).
inline bool enqueue_grouped_from(MBuf* const* batch, const uint32_t* perm, const uint32_t* counts,
                                 std::vector<std::shared_ptr<MpscQueue>>& queues, EnqueueStats& st, EnqueueCursor& c,
                                 bool stall) {
  const size_t ct = queues.size();
  const size_t n = std::accumulate(counts, counts + ct + 1, size_t{0});
  for (; c.g <= ct; ++c.g, c.j = 0) {
    for (; c.j < counts[c.g]; ++c.j, ++c.k) {
      if (c.k + 8 < n) __builtin_prefetch(batch[perm[c.k + 8]], 1, 0);  // the mbufs come in group order
      MBuf* m = batch[perm[c.k]];
      if (c.g == ct) {  // mbuf_free (native/zcsi/zcsi.rs:44): the port owns the storage here
        ++st.would_panic;
        continue;
      }
      if (stall && queues[c.g]->free_slots() == 0) {
        ++st.stalls;
        return false;
      }
      save_header_and_offset(m);
      if (!queues[c.g]->enqueue_one(m)) ++st.dropped;
    }
  }
  return true;
}
inline void enqueue_grouped(MBuf* const* batch, const uint32_t* perm, const uint32_t* counts,
                            std::vector<std::shared_ptr<MpscQueue>>& queues, EnqueueStats& st) {
  EnqueueCursor c;
  enqueue_grouped_from(batch, perm, counts, queues, st, c, false);
}

// The Maglev group function of test/maglev (nf.rs:101-106): lut[flow_hash % M].
class MaglevGroup {
 public:
  MaglevGroup(const std::vector<std::string>& backends, uint64_t lut_size, int device = 0) {
    std::vector<const char*> names;
    std::vector<uint32_t> lens;
    for (auto& b : backends) {
      names.push_back(b.data());
      lens.push_back(static_cast<uint32_t>(b.size()));
    }
    nbg_maglev* h = nullptr;
    check(nbg_maglev_create(names.data(), lens.data(), static_cast<uint32_t>(names.size()), lut_size, device, &h),
          "nbg_maglev_create");
    h_.reset(h, nbg_maglev_destroy);
  }
  nbg_maglev* handle() const { return h_.get(); }
  uint32_t backends() const { return nbg_maglev_backends(h_.get()); }

 private:
  std::shared_ptr<nbg_maglev> h_;
};

// The group queues keep the reference's 1024 slots (new_mpsc_queue_pair, mpsc_mbuf_queue.rs:261-265;
// 1023 usable), so one GPU batch may hold at most 1023 packets: then even a batch whose packets all
// land in one group fits an empty queue.
constexpr uint32_t kQueueSlots = 1024;
constexpr uint32_t kMaxGpuBatch = kQueueSlots - 1;

// When the producer pulls the next batch from its port, and what a full group queue does.
//   kBackpressure (default; a deliberate deviation): a batch is pulled only when every group queue has
//     room for a whole batch, and the enqueue of a classified batch waits at a full queue (resumed by
//     the producer's next execution, after the consumers ran) instead of dropping: no packet is ever
//     lost, and per-group FIFO order holds.  Packets wait in the port (the NIC's RX ring) and in the
//     producer's in-flight batches, as they do in DPDK when a pipeline falls behind.
//   kDropOnFull (the reference): a batch is pulled whenever the pipeline has a free slot; a packet
//     whose queue is full is lost (GroupByProducer ignores enqueue_one's result, group_by.rs:50;
//     enqueue_sp refuses it, mpsc_mbuf_queue.rs:91-115).
enum class Admission { kBackpressure, kDropOnFull };

// Packets per GPU batch: at most kMaxGpuBatch, whole 32-packet bursts (receive_batch.rs:26).
inline uint32_t cap_batch(uint32_t want) { return std::max(kBurst, std::min(want, kMaxGpuBatch) / kBurst * kBurst); }

inline bool admit_batch(const std::vector<std::shared_ptr<MpscQueue>>& queues, uint32_t max_batch, Admission a) {
  if (a == Admission::kDropOnFull) return true;
  for (auto& q : queues)
    if (q->free_slots() < max_batch) return false;
  return true;
}

// Where a GPU producer's time goes (seconds over the run): pulling RX bursts into a batch, the submit
// (gather + launch), completion polls, the wait (results + MAC write-back), the per-group enqueue.
struct ProducerProfile {
  double pull = 0, submit = 0, query = 0, wait = 0, enqueue = 0;
  uint64_t queries = 0;
};

// Batches a producer keeps in flight on the GPU (nbg_maglev_host_submit's staging slots).
constexpr uint32_t kMaxDepth = NBG_HOST_SLOTS;

// GroupBy (group_by.rs:15-113) with the GPU producer: ct queues, get_group(i) for i < ct.  Packets
// the reference would panic on (the would-panic sentinel group) are freed by the producer and
// counted (would_panic()); everything else keeps the reference semantics.  max_batch is capped at
// kMaxGpuBatch (1023; 992 = 31 whole bursts) so that the reference's 1024-slot queues can always
// take a batch.  The producer is pipelined: up to `depth` batches are on the GPU at once
// (nbg_maglev_host_submit), each delivered to the queues — in submit order, so per-group FIFO order
// holds across batches — by the first execute() that finds it complete (nbg_maglev_host_query); the
// scheduler's other tasks (the consumers) run while a batch is on the GPU or waits at a full queue.
class GroupBy {
 public:
  GroupBy(ParsedMacBatch parent, uint32_t groups, MaglevGroup fn, StandaloneScheduler& sched,
          uint32_t max_batch = kMaxGpuBatch, Admission admission = Admission::kBackpressure,
          uint32_t depth = kMaxDepth)
      : groups_(groups) {
    if (groups != fn.backends()) throw std::invalid_argument("group_by: groups != Maglev backends");
    if (max_batch == 0) throw std::invalid_argument("group_by: max_batch must be >= 1");
    if (depth == 0 || depth > kMaxDepth) throw std::invalid_argument("group_by: depth must be 1..NBG_HOST_SLOTS");
    max_batch = cap_batch(max_batch);
    for (uint32_t i = 0; i < groups; ++i) queues_.push_back(std::make_shared<MpscQueue>(kQueueSlots));
    producer_ = std::make_shared<Producer>(std::move(parent), std::move(fn), queues_, max_batch, admission, depth);
    task_ = sched.add_task(producer_);
  }
  uint32_t len() const { return groups_; }
  uint32_t max_batch() const { return producer_->max_batch; }
  uint32_t depth() const { return producer_->depth; }

  // get_group(i): RestoreHeader over a ReceiveBatch of the group's MPSC consumer (group_by.rs:102-112).
  std::shared_ptr<RestoreHeader> get_group(uint32_t i) {
    if (i >= groups_) return nullptr;
    struct Consumer : PacketRx {
      std::shared_ptr<MpscQueue> q;
      uint32_t recv(MBuf** p, uint32_t cap) override { return q->dequeue(p, cap); }
    };
    auto c = std::make_shared<Consumer>();
    c->q = queues_[i];
    return std::make_shared<RestoreHeader>(std::make_shared<ReceiveBatch>(c));
  }
  uint64_t dropped() const { return producer_->stats.dropped; }
  uint64_t stalls() const { return producer_->stats.stalls; }
  uint64_t would_panic() const { return producer_->stats.would_panic; }
  uint64_t processed() const { return producer_->processed; }  // packets delivered to the queues
  uint64_t in_flight() const { return producer_->in_flight_pkts; }
  uint64_t batches() const { return producer_->batches; }
  const ProducerProfile& profile() const { return producer_->prof; }
  void set_profiled(bool on) {
    if (on) TscClock::seconds_per_tick();
    producer_->timed = on;
  }
  nbg_maglev* handle() const { return producer_->fn.handle(); }

 private:
  struct InFlight {
    std::vector<MBuf*> batch;
    std::vector<uint8_t*> ptrs;
    std::vector<uint16_t> lens, backend;
    std::vector<uint32_t> perm, counts;
    uint64_t ticket = 0;
    bool waited = false;  // results and MAC rewrite landed (host_wait returned)
    EnqueueCursor cur;    // how far its enqueue got
  };

  struct Producer : Executable {
    Producer(ParsedMacBatch p, MaglevGroup f, std::vector<std::shared_ptr<MpscQueue>> q, uint32_t max_batch,
             Admission admission, uint32_t depth)
        : parent(std::move(p)), fn(std::move(f)), queues(std::move(q)), max_batch(max_batch), admission(admission),
          depth(depth), slots(depth) {
      for (auto& b : slots) {
        b.batch.reserve(max_batch);
        b.ptrs.resize(max_batch);
        b.lens.resize(max_batch);
        b.backend.resize(max_batch);
        b.perm.resize(max_batch);
        b.counts.resize(queues.size() + 1);
      }
    }
    // GroupByProducer::execute (group_by.rs:43-55) for whole batches: deliver every batch the GPU has
    // finished (oldest first), then pull bursts until a new batch is full or the port is idle and
    // submit it, if the pipeline has a free slot and the queues admit it.
    void execute() override {
      while (n_in_flight) {
        InFlight& b = slots[head];
        if (!b.waited) {
          int done = 0;
          const Clock::tick t0 = tnow();
          check(nbg_maglev_host_query(fn.handle(), b.ticket, &done), "nbg_maglev_host_query");
          prof.query += since(t0);
          ++prof.queries;
          if (!done) break;
        }
        if (!deliver(b)) break;  // a full queue (backpressure): resumed at the next execution
      }
      if (n_in_flight == depth) return;
      // every queue has room for a whole batch: checked over all ct queues only until it holds, then
      // kept until this producer enqueues again (the consumers only ever free slots)
      if (!room) room = admit_batch(queues, max_batch, admission);
      if (!room) return;
      const Clock::tick t0 = tnow();
      InFlight& b = slots[(head + n_in_flight) % depth];
      b.batch.clear();
      for (;;) {  // whole bursts only: max_batch is a multiple of kBurst
        parent.parent->act();
        auto& r = parent.parent->pkts;
        b.batch.insert(b.batch.end(), r.begin(), r.end());
        const bool idle = r.size() < kBurst;
        parent.parent->done();
        if (idle || b.batch.size() + kBurst > max_batch) break;
      }
      if (b.batch.empty()) return;
      const size_t n = b.batch.size();
      for (size_t i = 0; i < n; ++i) {
        b.ptrs[i] = b.batch[i]->data();
        b.lens[i] = b.batch[i]->data_len;
      }
      const Clock::tick t1 = tnow();
      prof.pull += static_cast<double>(t1 - t0) * TscClock::seconds_per_tick();
      check(nbg_maglev_host_submit(fn.handle(), b.ptrs.data(), b.lens.data(), n, parent.swap ? NBG_SWAP_MACS : 0u,
                                   b.backend.data(), b.perm.data(), b.counts.data(), &b.ticket),
            "nbg_maglev_host_submit");
      b.waited = false;
      b.cur = EnqueueCursor{};
      prof.submit += since(t1);
      ++n_in_flight;
      in_flight_pkts += n;
      ++batches;
    }
    // The enqueue half: results and the MAC rewrite land (host_wait), then the per-group FIFOs.
    // false: stopped at a full queue (backpressure); the batch stays at the head
    bool deliver(InFlight& b) {
      if (!b.waited) {
        const Clock::tick t0 = tnow();
        check(nbg_maglev_host_wait(fn.handle(), b.ticket), "nbg_maglev_host_wait");
        prof.wait += since(t0);
        b.waited = true;
      }
      const Clock::tick t1 = tnow();
      const bool all = enqueue_grouped_from(b.batch.data(), b.perm.data(), b.counts.data(), queues, stats, b.cur,
                                            admission == Admission::kBackpressure);
      room = false;
      prof.enqueue += since(t1);
      if (!all) return false;
      processed += b.batch.size();
      in_flight_pkts -= b.batch.size();
      head = (head + 1) % depth;
      --n_in_flight;
      return true;
    }
    ParsedMacBatch parent;
    MaglevGroup fn;
    std::vector<std::shared_ptr<MpscQueue>> queues;
    uint32_t max_batch;
    Admission admission;
    uint32_t depth;
    std::vector<InFlight> slots;  // a ring of `depth` batches: [head, head + n_in_flight) are on the GPU
    bool room = false;            // admit_batch held and no enqueue since
    uint32_t head = 0, n_in_flight = 0;
    uint64_t in_flight_pkts = 0;
    EnqueueStats stats;
    uint64_t processed = 0, batches = 0;
    ProducerProfile prof;
    bool timed = true;  // the per-phase profile (off: no clock reads at all)
    using Clock = TscClock;
    Clock::tick tnow() const { return timed ? Clock::now() : 0; }
    double since(Clock::tick t) const { return timed ? TscClock::since(t) : 0.0; }
  };

  uint32_t groups_;
  std::vector<std::shared_ptr<MpscQueue>> queues_;
  std::shared_ptr<Producer> producer_;
  size_t task_ = 0;
};

// MergeBatch + CompositionBatch + SendBatch (merge_batch.rs:44-57, send_batch.rs:66-78): each
// execution receives one burst from the current group, sends it, and rotates the group.
class MergeSend : public Executable {
 public:
  MergeSend(std::vector<std::shared_ptr<Batch>> parents, std::shared_ptr<PacketTx> port)
      : parents_(std::move(parents)), port_(std::move(port)) {}
  void execute() override {
    auto& b = *parents_[which_];
    b.act();
    if (!b.pkts.empty()) sent += port_->send(b.pkts.data(), static_cast<uint32_t>(b.pkts.size()));
    b.done();
    which_ = (which_ + 1) % parents_.size();
  }
  uint64_t sent = 0;

 private:
  std::vector<std::shared_ptr<Batch>> parents_;
  std::shared_ptr<PacketTx> port_;
  size_t which_ = 0;
};

// test/maglev/src/nf.rs:84-111 with the GPU group_by: returns the merged, composed
// pipeline of all groups, ready to be sent (main.rs:33-37 `.send(port)`).
struct MaglevPipeline {
  std::shared_ptr<GroupBy> groups;
  std::shared_ptr<MergeSend> tx;
};

inline MaglevPipeline maglev(std::shared_ptr<Batch> parent, StandaloneScheduler& s,
                             const std::vector<std::string>& backends, std::shared_ptr<PacketTx> port,
                             uint64_t lut_size = 65537, uint32_t max_batch = kMaxGpuBatch,
                             Admission admission = Admission::kBackpressure, uint32_t depth = kMaxDepth) {
  const uint32_t ct = static_cast<uint32_t>(backends.size());
  MaglevGroup lut(backends, lut_size);  // Maglev::new(backends, 65537), nf.rs:90
  auto groups = std::make_shared<GroupBy>(transform(parse_mac(std::move(parent)), MacSwap{}), ct, lut, s,
                                          max_batch, admission, depth);
  std::vector<std::shared_ptr<Batch>> outs;
  for (uint32_t i = 0; i < ct; ++i) outs.push_back(groups->get_group(i));  // nf.rs:109
  auto tx = std::make_shared<MergeSend>(outs, std::move(port));
  s.add_task(tx);
  return {groups, tx};
}

}  // namespace nb
