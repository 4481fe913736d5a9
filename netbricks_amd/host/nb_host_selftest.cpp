// CPU-only self test of the host operator pieces that need no GPU: MPSC queue semantics
// (capacity mask = 1023 of 1024 slots, FIFO, refusal when full: mpsc_mbuf_queue.rs:91-115)
// and pcap read/write round trips.  Exit code 0 = pass.
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
