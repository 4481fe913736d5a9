// CPU-only timing of the drop-in path's host side without the GPU: a LoopPort replay, the producer's
// enqueue of a classified batch (enqueue_grouped_from with a synthetic perm / counts, 65 groups) and the
// consumer (GroupBy::get_group's RestoreHeader over each group's queue, MergeSend to the port), on one
// thread as nb_maglev --loop runs them.  Measurement tool (no GPU, no oracle): ns per packet of each
// half, for A/B builds of operators.hpp.
//   g++ -O2 -std=c++17 -I. -o /tmp/consumer_bench tools/consumer_bench.cpp && /tmp/consumer_bench [packets] [mbuf stride]
#include <chrono>
#include <cstdio>
#include <memory>
#include <random>
#include <vector>

#include "netbricks_amd/host/operators.hpp"
#include "netbricks_amd/host/pcap_port.hpp"

namespace {
struct QueueRx : nb::PacketRx {  // GroupBy::get_group's consumer side
  std::shared_ptr<nb::MpscQueue> q;
  uint32_t recv(nb::MBuf** p, uint32_t cap) override { return q->dequeue(p, cap); }
};
}  // namespace

int main(int argc, char** argv) {
  const uint32_t groups = 65, batch = 992;
  const uint64_t total = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 20000000ull;
  std::vector<nb::PcapRecord> recs(10000);
  for (auto& r : recs) r.data.assign(60, 0x11);
  const uint32_t stride = argc > 2 ? static_cast<uint32_t>(std::strtoul(argv[2], nullptr, 10)) : 0u;
  auto port = std::make_shared<nb::LoopPort>(recs, total, 8192, 2048, true, stride);
  std::vector<std::shared_ptr<nb::MpscQueue>> queues;
  std::vector<std::shared_ptr<nb::Batch>> outs;
  for (uint32_t g = 0; g < groups; ++g) {
    queues.push_back(std::make_shared<nb::MpscQueue>(nb::kQueueSlots));
    auto rx = std::make_shared<QueueRx>();
    rx->q = queues.back();
    outs.push_back(std::make_shared<nb::RestoreHeader>(std::make_shared<nb::ReceiveBatch>(rx)));
  }
  nb::MergeSend tx(outs, port);
  nb::ReceiveBatch rxb(port);
  std::mt19937 rng(7);
  std::vector<nb::MBuf*> b;
  std::vector<uint32_t> perm(batch), counts(groups + 1), bin(batch);
  nb::EnqueueStats st;
  double t_prod = 0, t_cons = 0;
  uint64_t rounds = 0, sent_before = 0;
  using C = nb::TscClock;
  while (!port->rx_done() || tx.sent < port->rx_total()) {
    const auto t0 = C::now();
    bool room = true;
    for (auto& q : queues) room = room && q->free_slots() >= batch;
    if (room && !port->rx_done()) {
      b.clear();
      while (b.size() + nb::kBurst <= batch) {
        rxb.act();
        b.insert(b.end(), rxb.pkts.begin(), rxb.pkts.end());
        const bool idle = rxb.pkts.size() < nb::kBurst;
        rxb.done();
        if (idle) break;
      }
      // a synthetic classification: each packet's group at random, perm in group order (stable)
      std::fill(counts.begin(), counts.end(), 0u);
      for (size_t i = 0; i < b.size(); ++i) ++counts[bin[i] = rng() % groups];
      std::vector<uint32_t> base(groups + 1, 0);
      for (uint32_t g = 1; g <= groups; ++g) base[g] = base[g - 1] + counts[g - 1];
      for (size_t i = 0; i < b.size(); ++i) perm[base[bin[i]]++] = static_cast<uint32_t>(i);
      nb::EnqueueCursor c;
      nb::enqueue_grouped_from(b.data(), perm.data(), counts.data(), queues, st, c, true);
    }
    const auto t1 = C::now();
    tx.execute();
    const auto t2 = C::now();
    t_prod += static_cast<double>(t1 - t0) * C::seconds_per_tick();
    t_cons += static_cast<double>(t2 - t1) * C::seconds_per_tick();
    ++rounds;
    if (tx.sent == sent_before && port->rx_done() && tx.sent >= port->rx_total()) break;
    sent_before = tx.sent;
  }
  const double n = static_cast<double>(port->rx_total());
  std::printf("{\"packets\": %.0f, \"rounds\": %llu, \"producer_ns_per_pkt\": %.2f, \"consumer_ns_per_pkt\": %.2f, "
              "\"consumer_ns_per_execute\": %.1f, \"mpps_one_thread\": %.1f}\n",
              n, static_cast<unsigned long long>(rounds), 1e9 * t_prod / n, 1e9 * t_cons / n, 1e9 * t_cons / rounds,
              n / (t_prod + t_cons) / 1e6);
  return 0;
}
