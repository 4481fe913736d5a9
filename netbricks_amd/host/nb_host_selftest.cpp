// CPU-only self test of the host operator pieces that need no GPU: MPSC queue semantics
// (capacity mask = 1023 of 1024 slots, FIFO, refusal when full: mpsc_mbuf_queue.rs:91-115),
// the producer's grouped enqueue with save_header_and_offset and the consumer's RestoreHeader
// (packet.rs:211-221,414-424, restore_header.rs:62-65), and pcap read/write round trips.
// Exit code 0 = pass.
#include <cstdio>
#include <cstdlib>

#include "operators.hpp"
#include "pcap_port.hpp"

#define EXPECT(c)                                                        \
  do {                                                                   \
    if (!(c)) {                                                          \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      return 1;                                                          \
    }                                                                    \
  } while (0)

int main(int argc, char** argv) {
  nb::MpscQueue q(1024);
  std::vector<nb::MBuf> bufs(1100);
  uint32_t accepted = 0;
  for (auto& b : bufs) accepted += q.enqueue_one(&b);
  EXPECT(accepted == 1023);
  nb::MBuf* out[32];
  EXPECT(q.dequeue(out, 32) == 32);
  EXPECT(out[0] == &bufs[0] && out[31] == &bufs[31]);
  EXPECT(q.enqueue_one(&bufs[1099]));
  uint32_t total = 32;
  for (uint32_t n; (n = q.dequeue(out, 32)) > 0;) total += n;
  EXPECT(total == 1024);
  {
    // a classified batch of 6 frames over 2 groups + the would-panic group: perm/counts as the
    // C-ABI returns them (groups in order, arrival order inside each group)
    std::vector<nb::MBuf> m(6);
    for (size_t i = 0; i < m.size(); ++i) {
      m[i].storage.assign(64, 0);
      m[i].data_len = 60;
      for (int k = 0; k < 12; ++k) m[i].storage[k] = static_cast<uint8_t>(16 * i + k);  // dst 0..5, src 6..11
      m[i].storage[12] = 0x08;
    }
    std::vector<nb::MBuf*> batch;
    for (auto& b : m) batch.push_back(&b);
    const uint32_t perm[6] = {1, 4, 0, 2, 5, 3};  // group 0: 1, 4; group 1: 0, 2, 5; would-panic: 3
    const uint32_t counts[3] = {2, 3, 1};
    std::vector<std::shared_ptr<nb::MpscQueue>> qs = {std::make_shared<nb::MpscQueue>(1024),
                                                      std::make_shared<nb::MpscQueue>(1024)};
    nb::EnqueueStats st;
    nb::enqueue_grouped(batch.data(), perm, counts, qs, st);
    EXPECT(st.would_panic == 1 && st.dropped == 0 && qs[0]->size() == 2 && qs[1]->size() == 3);
    EXPECT(m[3].meta[0] == 0);  // freed, never enqueued: no saved header
    // consumer side: ReceiveBatch over the queue -> RestoreHeader -> re-parse the MAC header
    struct Rx : nb::PacketRx {
      std::shared_ptr<nb::MpscQueue> q;
      uint32_t recv(nb::MBuf** p, uint32_t cap) override { return q->dequeue(p, cap); }
    };
    const uint32_t want[2][3] = {{1, 4, 0}, {0, 2, 5}};
    for (int g = 0; g < 2; ++g) {
      auto rx = std::make_shared<Rx>();
      rx->q = qs[g];
      nb::RestoreHeader rh(std::make_shared<nb::ReceiveBatch>(rx));
      rh.act();
      EXPECT(rh.packets.size() == counts[g]);
      for (size_t j = 0; j < rh.packets.size(); ++j) {
        const nb::MacPacket& p = rh.packets[j];
        EXPECT(p.mbuf == &m[want[g][j]]);
        EXPECT(p.header == m[want[g][j]].data() && p.offset == 0);
        EXPECT(p.header[0] == 16 * want[g][j] && p.header[6] == 16 * want[g][j] + 6);  // dst, src
        EXPECT(p.payload() == m[want[g][j]].data() + 14);
      }
      rh.done();
    }
    // a zeroed header slot is the reference's unwrap panic (restore_header.rs:64)
    nb::MBuf bare;
    bare.storage.assign(64, 0);
    auto q = std::make_shared<nb::MpscQueue>(1024);
    q->enqueue_one(&bare);
    auto rx = std::make_shared<Rx>();
    rx->q = q;
    nb::RestoreHeader rh(std::make_shared<nb::ReceiveBatch>(rx));
    bool threw = false;
    try {
      rh.act();
    } catch (const nb::NbError&) {
      threw = true;
    }
    EXPECT(threw);
  }
  {
    // The reference's drop on a full queue: one batch of 1500 packets that all land in group 0 of
    // 1024-slot queues (mpsc_mbuf_queue.rs:261) keeps 1023 and loses 477 (enqueue_sp refuses,
    // group_by.rs:50 ignores the refusal).
    std::vector<nb::MBuf> m(1500);
    std::vector<nb::MBuf*> batch;
    std::vector<uint32_t> perm(m.size());
    for (size_t i = 0; i < m.size(); ++i) {
      m[i].storage.assign(64, 0);
      batch.push_back(&m[i]);
      perm[i] = static_cast<uint32_t>(i);
    }
    const uint32_t counts[3] = {1500, 0, 0};
    std::vector<std::shared_ptr<nb::MpscQueue>> qs = {std::make_shared<nb::MpscQueue>(nb::kQueueSlots),
                                                      std::make_shared<nb::MpscQueue>(nb::kQueueSlots)};
    EXPECT(nb::admit_batch(qs, 1500, nb::Admission::kDropOnFull));
    nb::EnqueueStats st;
    nb::enqueue_grouped(batch.data(), perm.data(), counts, qs, st);
    EXPECT(st.dropped == 477 && qs[0]->size() == 1023 && qs[1]->size() == 0);
    nb::MBuf* out[32];
    EXPECT(qs[0]->dequeue(out, 32) == 32 && out[0] == &m[0] && out[31] == &m[31]);  // the first 1023 kept, in order
  }
  {
    // Capped batches with backpressure: batches of cap_batch() packets (whole bursts, <= 1023) are
    // admitted only when every 1024-slot queue can take a whole batch, so even the worst case —
    // every packet of every batch in one group, a consumer draining one 32-packet burst of one group
    // per round (merge_batch.rs:44-57) — drops nothing and keeps FIFO order.  The same schedule with
    // the reference's drop-on-full admission loses packets.
    EXPECT(nb::cap_batch(4096) == 992 && nb::cap_batch(1023) == 992 && nb::cap_batch(100) == 96 &&
           nb::cap_batch(10) == 32);
    for (int mode = 0; mode < 2; ++mode) {
      const auto adm = mode == 0 ? nb::Admission::kBackpressure : nb::Admission::kDropOnFull;
      const uint32_t cap = nb::cap_batch(4096), total = 20000, groups = 3;
      std::vector<nb::MBuf> m(total);
      std::vector<std::shared_ptr<nb::MpscQueue>> qs;
      for (uint32_t g = 0; g < groups; ++g) qs.push_back(std::make_shared<nb::MpscQueue>(nb::kQueueSlots));
      nb::EnqueueStats st;
      uint32_t next = 0, delivered = 0, which = 0;
      std::vector<uint32_t> last_seen(groups, 0);
      bool in_order = true;
      for (int round = 0; round < 200000 && (next < total || delivered + st.dropped < total); ++round) {
        if (next < total && nb::admit_batch(qs, cap, adm)) {
          const uint32_t n = std::min(cap, total - next);
          const uint32_t g = (next / cap) % 2;  // every packet of a batch in one group (0 or 1)
          std::vector<nb::MBuf*> batch;
          std::vector<uint32_t> perm(n);
          for (uint32_t i = 0; i < n; ++i) {
            m[next + i].port_seq = next + i + 1;
            batch.push_back(&m[next + i]);
            perm[i] = i;
          }
          uint32_t counts[4] = {0, 0, 0, 0};
          counts[g] = n;
          nb::enqueue_grouped(batch.data(), perm.data(), counts, qs, st);
          next += n;
        }
        nb::MBuf* out[32];
        const uint32_t got = qs[which]->dequeue(out, 32);
        for (uint32_t i = 0; i < got; ++i) {
          in_order &= out[i]->port_seq > last_seen[which];
          last_seen[which] = static_cast<uint32_t>(out[i]->port_seq);
        }
        delivered += got;
        which = (which + 1) % groups;
      }
      EXPECT(in_order);
      if (mode == 0) EXPECT(st.dropped == 0 && delivered == total);
      else EXPECT(st.dropped > 0 && delivered + st.dropped == total);
    }
  }
  {
    // Backpressure: a batch of 1500 packets of one group stops at the full 1024-slot queue (1023
    // in), resumes where it stopped once the consumer drained a burst, and ends with every packet
    // delivered once, in order, nothing dropped.
    std::vector<nb::MBuf> m(1500);
    std::vector<nb::MBuf*> batch;
    std::vector<uint32_t> perm(m.size());
    for (size_t i = 0; i < m.size(); ++i) {
      m[i].storage.assign(64, 0);
      m[i].port_seq = i;
      batch.push_back(&m[i]);
      perm[i] = static_cast<uint32_t>(i);
    }
    const uint32_t counts[2] = {1500, 0};
    std::vector<std::shared_ptr<nb::MpscQueue>> qs = {std::make_shared<nb::MpscQueue>(nb::kQueueSlots)};
    nb::EnqueueStats st;
    nb::EnqueueCursor cur;
    EXPECT(!nb::enqueue_grouped_from(batch.data(), perm.data(), counts, qs, st, cur, true));
    EXPECT(qs[0]->size() == 1023 && cur.k == 1023 && st.stalls == 1 && st.dropped == 0);
    nb::MBuf* out[32];
    uint64_t next = 0, rounds = 0;
    bool done = false, in_order = true;
    while (next < 1500 && rounds++ < 1000) {
      if (!done) done = nb::enqueue_grouped_from(batch.data(), perm.data(), counts, qs, st, cur, true);
      for (uint32_t n = qs[0]->dequeue(out, 32), i = 0; i < n; ++i) in_order &= out[i]->port_seq == next++;
    }
    EXPECT(done && in_order && next == 1500 && st.dropped == 0);
  }
  if (argc > 2) {  // pcap round trip: argv[1] in, argv[2] out
    auto recs = nb::read_pcap(argv[1]);
    EXPECT(!recs.empty());
    nb::write_pcap(argv[2], recs);
    auto again = nb::read_pcap(argv[2]);
    EXPECT(again.size() == recs.size());
    for (size_t i = 0; i < recs.size(); ++i) EXPECT(again[i].data == recs[i].data);
    nb::PcapPort port(argv[1]);
    nb::MBuf* p[32];
    size_t got = 0;
    for (uint32_t n; (n = port.recv(p, 32)) > 0;) {
      port.send(p, n);
      got += n;
    }
    EXPECT(got == recs.size() && port.tx_index().back() == recs.size() - 1);
  }
  {  // LoopPort (nb_maglev --loop's replay): pool rounded up to whole captures, objects at the given
     // stride, every frame handed out in capture order and recycled by send
    std::vector<nb::PcapRecord> recs(100);
    for (size_t i = 0; i < recs.size(); ++i) recs[i].data.assign(60, static_cast<uint8_t>(i));
    nb::LoopPort port(recs, 1000, 150, 2048, false, 2368);
    EXPECT(port.pool_size() == 200);
    EXPECT(port.mempool().second == 200u * 2368u);
    std::vector<nb::MBuf*> got(32);
    uint64_t seen = 0;
    while (!port.rx_done()) {
      const uint32_t n = port.recv(got.data(), 32);
      EXPECT(n > 0);
      for (uint32_t i = 0; i < n; ++i, ++seen) {
        EXPECT(got[i]->data_len == 60 && got[i]->data()[0] == static_cast<uint8_t>(seen % 200 % 100));
        EXPECT((got[i]->data() - port.mempool().first) % 2368 == 0);
      }
      EXPECT(port.send(got.data(), n) == n);
    }
    EXPECT(seen == 1000 && port.tx_total() == 1000);
  }
  {  // the profile clock: monotonic, calibrated to a plausible rate
    const auto t0 = nb::TscClock::now();
    const double s = nb::TscClock::seconds_per_tick();
    EXPECT(s > 1e-12 && s < 1e-6);
    EXPECT(nb::TscClock::now() >= t0);
  }
  std::printf("nb_host_selftest ok\n");
  return 0;
}
