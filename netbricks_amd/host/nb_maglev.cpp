// nb_maglev: the test/maglev NF (test/maglev/src/main.rs:23-42, nf.rs:84-111) on the MI355X
// path, driven from a pcap port (the eth_pcap PMD of the reference's example tests).
//
//   nb_maglev --rx in.pcap --tx out.pcap [--backends N | --names a,b,c] [--table 65537]
//             [--batch 4096] [--order order.txt]
//
// Default backends are the reference's ["Larry", "Curly", "Moe"] (main.rs:36).  Prints one
// JSON line with rx/tx/dropped counts and the per-group packet counts; --order writes the rx
// index of every transmitted frame (one per line) for order checks.
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
  uint32_t batch = 4096;
  for (int i = 1; i + 1 < argc; i += 2) {
    const std::string k = argv[i], v = argv[i + 1];
    if (k == "--rx") rx = v;
    else if (k == "--tx") tx = v;
    else if (k == "--order") order = v;
    else if (k == "--table") table = std::strtoull(v.c_str(), nullptr, 10);
    else if (k == "--batch") batch = static_cast<uint32_t>(std::strtoul(v.c_str(), nullptr, 10));
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
    nb::StandaloneScheduler sched;
    auto pipe = nb::maglev(std::make_shared<nb::ReceiveBatch>(port), sched, names, port, table, batch);
    // run until the capture is consumed and every group queue has drained
    for (int idle = 0; idle < 2 * static_cast<int>(names.size() + 2);) {
      const uint64_t before = pipe.tx->sent + pipe.groups->processed();
      sched.execute_round();
      const bool progress = pipe.tx->sent + pipe.groups->processed() != before;
      idle = (port->rx_done() && !progress) ? idle + 1 : 0;
    }
    if (!tx.empty()) nb::write_pcap(tx, port->tx());
    if (!order.empty()) {
      FILE* f = std::fopen(order.c_str(), "w");
      for (size_t i : port->tx_index()) std::fprintf(f, "%zu\n", i);
      std::fclose(f);
    }
    std::printf("{\"rx\": %zu, \"tx\": %llu, \"dropped\": %llu, \"would_panic\": %llu, \"backends\": %zu}\n",
                port->rx_total(), static_cast<unsigned long long>(pipe.tx->sent),
                static_cast<unsigned long long>(pipe.groups->dropped()),
                static_cast<unsigned long long>(pipe.groups->would_panic()), names.size());
  } catch (const nb::NbError& e) {
    std::fprintf(stderr, "nb_maglev: %s\n", e.what());
    return e.code == NBG_ENODEV ? 3 : 1;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "nb_maglev: %s\n", e.what());
    return 1;
  }
  return 0;
}
