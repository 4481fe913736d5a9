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
  std::printf("nb_host_selftest ok\n");
  return 0;
}
