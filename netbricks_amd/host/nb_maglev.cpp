// nb_maglev: the test/maglev NF (test/maglev/src/main.rs:23-42, nf.rs:84-111) on the MI355X
// path, driven from a pcap port (the eth_pcap PMD of the reference's example tests).
//
//   nb_maglev --rx in.pcap --tx out.pcap [--backends N | --names a,b,c] [--table 65537]
//             [--batch 992] [--order order.txt] [--zero-copy 1] [--drop-on-full 1]
//
// Default backends are the reference's ["Larry", "Curly", "Moe"] (main.rs:36).  Prints one
// JSON line with rx/tx/dropped counts and the per-group packet counts; --order writes the rx
// index of every transmitted frame (one per line) for order checks.  --zero-copy 1 registers the
// port's mempool (nbg_host_register), so the GPU reads and rewrites the frames in place over PCIe.
// The group queues have the reference's 1024 slots; --batch is capped at 992 (whole bursts, at most
// 1023).  By default the producer waits while a queue could not take a whole batch; --drop-on-full 1
// pulls regardless and drops on a full queue, as the reference's producer does (group_by.rs:50).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <sstream>
#include <string>
#include <vector>

#include "operators.hpp"
#include "pcap_port.hpp"

int main(int argc, char** argv) {
  std::string rx, tx, order;
  std::vector<std::string> names = {"Larry", "Curly", "Moe"};
  uint64_t table = 65537;
  uint32_t batch = nb::kMaxGpuBatch;
  bool zero_copy = false, drop_on_full = false;
  for (int i = 1; i + 1 < argc; i += 2) {
    const std::string k = argv[i], v = argv[i + 1];
    if (k == "--rx") rx = v;
    else if (k == "--tx") tx = v;
    else if (k == "--order") order = v;
    else if (k == "--table") table = std::strtoull(v.c_str(), nullptr, 10);
    else if (k == "--batch") batch = static_cast<uint32_t>(std::strtoul(v.c_str(), nullptr, 10));
    else if (k == "--zero-copy") zero_copy = std::atoi(v.c_str()) != 0;
    else if (k == "--drop-on-full") drop_on_full = std::atoi(v.c_str()) != 0;
    else if (k == "--backends") {
      names.clear();
      for (int b = 0, n = std::atoi(v.c_str()); b < n; ++b) names.push_back("backend-" + std::to_string(b));
    } else if (k == "--names") {
      names.clear();
      std::stringstream ss(v);
      for (std::string t; std::getline(ss, t, ',');) names.push_back(t);
    } else {
      std::fprintf(stderr, "unknown option %s\n", k.c_str());
      return 2;
    }
  }
  if (rx.empty()) {
    std::fprintf(stderr, "usage: nb_maglev --rx in.pcap [--tx out.pcap] [--backends N|--names a,b] ...\n");
    return 2;
  }
  try {
    auto port = std::make_shared<nb::PcapPort>(rx);
    auto pool = port->mempool();
    if (zero_copy && pool.second) {
      uint8_t* dev = nullptr;
      nb::check(nbg_host_register(pool.first, pool.second, 0, &dev), "nbg_host_register");
    }
    nb::StandaloneScheduler sched;
    sched.set_timed(true);
    auto pipe = nb::maglev(std::make_shared<nb::ReceiveBatch>(port), sched, names, port, table, batch,
                           drop_on_full ? nb::Admission::kDropOnFull : nb::Admission::kBackpressure);
    // run until the capture is consumed and every group queue has drained
    const auto t0 = std::chrono::steady_clock::now();
    for (int idle = 0; idle < 2 * static_cast<int>(names.size() + 2);) {
      const uint64_t before = pipe.tx->sent + pipe.groups->processed();
      sched.execute_round();
      const bool progress = pipe.tx->sent + pipe.groups->processed() != before;
      idle = (port->rx_done() && !progress) ? idle + 1 : 0;
    }
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (!tx.empty()) port->write_tx(tx);
    if (!order.empty()) {
      FILE* f = std::fopen(order.c_str(), "w");
      for (size_t i : port->tx_index()) std::fprintf(f, "%zu\n", i);
      std::fclose(f);
    }
    if (zero_copy && pool.second) nb::check(nbg_host_unregister(pool.first, 0), "nbg_host_unregister");
    std::printf("{\"rx\": %zu, \"tx\": %llu, \"dropped\": %llu, \"would_panic\": %llu, \"backends\": %zu, "
                "\"zero_copy\": %s, \"max_batch\": %u, \"drop_on_full\": %s, \"seconds\": %.6f, \"mpps\": %.2f, "
                "\"group_by_seconds\": %.6f, \"merge_send_seconds\": %.6f}\n",
                port->rx_total(), static_cast<unsigned long long>(pipe.tx->sent),
                static_cast<unsigned long long>(pipe.groups->dropped()),
                static_cast<unsigned long long>(pipe.groups->would_panic()), names.size(), zero_copy ? "true" : "false",
                pipe.groups->max_batch(), drop_on_full ? "true" : "false", secs, secs > 0 ? port->rx_total() / secs / 1e6 : 0.0, sched.task_seconds(0), sched.task_seconds(1));
  } catch (const nb::NbError& e) {
    std::fprintf(stderr, "nb_maglev: %s\n", e.what());
    return e.code == NBG_ENODEV ? 3 : 1;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "nb_maglev: %s\n", e.what());
    return 1;
  }
  return 0;
}
