// nb_maglev: the test/maglev NF (test/maglev/src/main.rs:23-42, nf.rs:84-111) on the MI355X
// path, driven from a pcap port (the eth_pcap PMD of the reference's example tests).
//
//   nb_maglev --rx in.pcap --tx out.pcap [--backends N | --names a,b,c] [--table 65537]
//             [--batch 992] [--depth 3] [--order order.txt] [--zero-copy 1] [--drop-on-full 1]
//   nb_maglev --rx in.pcap --loop TOTAL [--pipelines P] [--hw-queues Q] [--host-ring B] [...]  (throughput run)
//
// Default backends are the reference's ["Larry", "Curly", "Moe"] (main.rs:36).  Prints one
// JSON line with rx/tx/dropped counts and the per-group packet counts; --order writes the rx
// index of every transmitted frame (one per line) for order checks.  --zero-copy 1 registers the
// port's mempool (nbg_host_register), so the GPU reads and rewrites the frames in place over PCIe.
// The group queues have the reference's 1024 slots; --batch is capped at 992 (whole bursts, at most
// 1023).  --depth batches are on the GPU at once (1..NBG_HOST_SLOTS = 8, nbg_maglev_host_submit's slots).  By default
// the producer pulls a batch only while every queue could take a whole one, and a classified batch's
// enqueue waits at a full queue (backpressure: nothing is dropped); --drop-on-full 1 pulls whenever
// the pipeline has room and drops on a full queue, as the reference's producer does (group_by.rs:50).
//
// --loop TOTAL: each of P pipelines (--pipelines, default 1) runs on a thread of its own, pinned to
// one of the process's CPUs, with its own replay port (LoopPort: the capture's frames in a pool of
// --pool mbufs (default: 8,192, or the batches in flight plus 2,048 if more; rounded up to whole copies
// of the capture) with 2-KiB data rooms in
// transparent huge pages, as DPDK's mempools are in hugepages; --hugepages 0 for 4-KiB pages; received
// until TOTAL packets, freed by send — the reference's VirtualPort), its own
// scheduler, its own Maglev handle and stream: the reference's one pipeline per RX queue and core
// (scheduler/context.rs:55-69,241-255).  The JSON line then gives each pipeline's Mpps (rx packets
// over its wall time, producer and consumer tasks included) and the aggregate (all packets over the
// slowest pipeline's time).  --host-ring B attaches every pipeline's handle to one host-batch server
// of B blocks (nbg_host_ring_*: one persistent kernel takes the batches; no kernel launch per batch).
// Pipeline p runs on the p-th CPU local to the GPU (--local-cpus 0: of all the process may use), CPUs
// that other processes keep busy last, the rest dealt over their L3 caches (--spread-l3 0: in the
// kernel's order).
// The JSON's per-phase profile and producer seconds come from TSC reads around every task execution and
// producer phase; --profile 0 turns them off (the NF rate without them: within ~2 %).
#include <pthread.h>
#include <sched.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "operators.hpp"
#include "pcap_port.hpp"

namespace {

struct LoopResult {
  nb::ProducerProfile prof;
  double seconds = 0, producer_seconds = 0;
  bool huge = false;
  size_t pool = 0;
  uint64_t rx = 0, tx = 0, dropped = 0, would_panic = 0, batches = 0, stalls = 0;
  std::string error;
};

// The CPUs the pipelines are pinned to, in order: the process's allowed CPUs that are local to the GPU
// (nbg_device_local_cpus: its socket's physical cores first), or every allowed CPU when none is (or
// local = false).  A producer thread on the GPU's socket keeps its staged windows and the completion
// words it polls on the GPU's side of the inter-socket link, as DPDK puts lcores on the NIC's socket.
std::vector<int> pipeline_cpus(bool local) {
  std::vector<int> out;
  cpu_set_t allowed;
  if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return out;
  if (local) {
    std::vector<int32_t> near(1024);
    uint32_t n = 0;
    if (nbg_device_local_cpus(0, near.data(), static_cast<uint32_t>(near.size()), &n) == NBG_OK)
      for (uint32_t i = 0; i < std::min<uint32_t>(n, static_cast<uint32_t>(near.size())); ++i)
        if (near[i] >= 0 && near[i] < CPU_SETSIZE && CPU_ISSET(near[i], &allowed)) out.push_back(near[i]);
  }
  if (out.empty())
    for (int c = 0; c < CPU_SETSIZE; ++c)
      if (CPU_ISSET(c, &allowed)) out.push_back(c);
  return out;
}

// The same CPUs dealt round-robin over their L3 caches (sysfs cache/index3 of each CPU; the order
// within one L3 kept): 16 pipelines then take two cores on each of eight 8-core CCDs instead of all
// eight cores of two, so each thread has an L3 share and a CCD link share four times as large.
std::vector<int> spread_over_l3(const std::vector<int>& cpus) {
  std::vector<std::string> keys;
  std::vector<std::vector<int>> groups;
  for (int c : cpus) {
    std::string key = "?";
    const std::string path = "/sys/devices/system/cpu/cpu" + std::to_string(c) + "/cache/index3/shared_cpu_list";
    if (FILE* f = std::fopen(path.c_str(), "r")) {
      char line[256] = {0};
      if (std::fgets(line, sizeof line, f)) key = line;
      std::fclose(f);
    }
    size_t g = 0;
    while (g < keys.size() && keys[g] != key) ++g;
    if (g == keys.size()) {
      keys.push_back(key);
      groups.emplace_back();
    }
    groups[g].push_back(c);
  }
  std::vector<int> out;
  for (size_t i = 0; out.size() < cpus.size(); ++i)
    for (auto& g : groups)
      if (i < g.size()) out.push_back(g[i]);
  return out;
}

// The CPUs other processes kept busy over a 100-ms sample of /proc/stat (more than 20 % of their time:
// a shared host's other jobs) apart from the idle ones, the order otherwise kept: the pipelines take
// idle cores first.  The aggregate is set by the slowest pipeline's core, so a DPDK lcore gets an
// isolated one.
std::pair<std::vector<int>, std::vector<int>> idle_first(const std::vector<int>& cpus) {
  auto sample = [](std::vector<std::pair<uint64_t, uint64_t>>& v) {  // (busy, total) jiffies per CPU
    v.assign(CPU_SETSIZE, {0, 0});
    FILE* f = std::fopen("/proc/stat", "r");
    if (!f) return false;
    char line[512];
    while (std::fgets(line, sizeof line, f)) {
      int c = -1;
      unsigned long long u, n, sy, id, io, irq, sirq, st;
      if (std::sscanf(line, "cpu%d %llu %llu %llu %llu %llu %llu %llu %llu", &c, &u, &n, &sy, &id, &io, &irq, &sirq,
                      &st) == 9 && c >= 0 && c < CPU_SETSIZE)
        v[c] = {u + n + sy + irq + sirq + st, u + n + sy + id + io + irq + sirq + st};
    }
    std::fclose(f);
    return true;
  };
  std::vector<std::pair<uint64_t, uint64_t>> a, b;
  if (!sample(a)) return {cpus, {}};
  std::this_thread::sleep_for(std::chrono::milliseconds(100));
  if (!sample(b)) return {cpus, {}};
  std::vector<int> idle, busy;
  for (int c : cpus) {
    const uint64_t tot = b[c].second - a[c].second, use = b[c].first - a[c].first;
    (tot && use * 5 > tot ? busy : idle).push_back(c);
  }
  return {idle, busy};
}

void pin_to(int k, const std::vector<int>& cpus) {
  if (cpus.empty()) return;
  cpu_set_t one;
  CPU_ZERO(&one);
  CPU_SET(cpus[static_cast<size_t>(k) % cpus.size()], &one);
  pthread_setaffinity_np(pthread_self(), sizeof(one), &one);
}

int run_loop(const std::string& rx, const std::vector<std::string>& names, uint64_t table, uint32_t batch,
             uint32_t depth, bool zero_copy, bool drop_on_full, uint64_t total, int pipelines, bool huge,
             nbg_host_ring* server, size_t pool_mbufs, bool profiled, bool local, bool spread, uint32_t object) {
  const auto recs = nb::read_pcap(rx);
  const auto near = idle_first(pipeline_cpus(local));  // (idle, busy)
  std::vector<int> cpus = spread ? spread_over_l3(near.first) : near.first;
  for (int c : spread ? spread_over_l3(near.second) : near.second) cpus.push_back(c);
  std::vector<LoopResult> res(pipelines);
  std::atomic<int> ready{0};
  std::atomic<bool> go{false};
  std::vector<std::thread> th;
  for (int p = 0; p < pipelines; ++p)
    th.emplace_back([&, p] {
      LoopResult& r = res[p];
      bool counted = false;
      try {
        pin_to(p, cpus);
        const size_t mbufs = pool_mbufs ? pool_mbufs
                                        : std::max<size_t>(8192, size_t{depth} * nb::cap_batch(batch) + 2048);
        auto port = std::make_shared<nb::LoopPort>(recs, total, mbufs, 2048, huge, object);
        auto pool = port->mempool();
        uint8_t* dev = nullptr;
        if (zero_copy) nb::check(nbg_host_register(pool.first, pool.second, 0, &dev), "nbg_host_register");
        nb::StandaloneScheduler sched;
        sched.set_timed(profiled);
        auto pipe = nb::maglev(std::make_shared<nb::ReceiveBatch>(port), sched, names, port, table, batch,
                               drop_on_full ? nb::Admission::kDropOnFull : nb::Admission::kBackpressure, depth);
        pipe.groups->set_profiled(profiled);
        if (server) nb::check(nbg_maglev_set_host_ring(pipe.groups->handle(), server), "nbg_maglev_set_host_ring");
        ++ready;
        counted = true;
        while (!go.load()) std::this_thread::yield();
        const auto t0 = std::chrono::steady_clock::now();
        for (int idle = 0; idle < 2 * static_cast<int>(names.size() + 2);) {
          const uint64_t before = port->tx_total() + pipe.groups->processed();
          sched.execute_round();
          const bool progress = port->tx_total() + pipe.groups->processed() != before;
          idle = (port->rx_done() && pipe.groups->in_flight() == 0 && !progress) ? idle + 1 : 0;
        }
        r.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        r.producer_seconds = sched.task_seconds(0);
        r.rx = port->rx_total();
        r.huge = port->huge_pages();
        r.pool = port->pool_size();
        r.tx = port->tx_total();
        r.dropped = pipe.groups->dropped();
        r.would_panic = pipe.groups->would_panic();
        r.batches = pipe.groups->batches();
        r.stalls = pipe.groups->stalls();
        r.prof = pipe.groups->profile();
        if (zero_copy) nb::check(nbg_host_unregister(pool.first, 0), "nbg_host_unregister");
      } catch (const std::exception& e) {
        r.error = e.what();
        if (!counted) ++ready;
      }
    });
  while (ready.load() < pipelines) std::this_thread::sleep_for(std::chrono::milliseconds(1));
  go = true;
  for (auto& t : th) t.join();
  double tmax = 0;
  nb::ProducerProfile pr;  // summed over pipelines
  uint64_t rx_all = 0, tx_all = 0, dropped = 0, panic = 0, batches = 0, stalls = 0;
  std::string per, prod, err;
  bool huge_all = true;
  for (auto& r : res) {
    if (!r.error.empty()) err = r.error;
    huge_all = huge_all && r.huge;
    tmax = std::max(tmax, r.seconds);
    rx_all += r.rx;
    tx_all += r.tx;
    dropped += r.dropped;
    panic += r.would_panic;
    batches += r.batches;
    stalls += r.stalls;
    pr.pull += r.prof.pull;
    pr.submit += r.prof.submit;
    pr.query += r.prof.query;
    pr.wait += r.prof.wait;
    pr.enqueue += r.prof.enqueue;
    pr.queries += r.prof.queries;
    char b[64];
    std::snprintf(b, sizeof b, "%s%.2f", per.empty() ? "" : ", ", r.seconds > 0 ? r.rx / r.seconds / 1e6 : 0.0);
    per += b;
    std::snprintf(b, sizeof b, "%s%.4f", prod.empty() ? "" : ", ", r.producer_seconds);
    prod += b;
  }
  if (!err.empty()) {
    std::fprintf(stderr, "nb_maglev: %s\n", err.c_str());
    return 1;
  }
  std::string cpu_list;
  for (int p = 0; p < pipelines && !cpus.empty(); ++p)
    cpu_list += (p ? "," : "") + std::to_string(cpus[static_cast<size_t>(p) % cpus.size()]);
  std::printf("{\"mode\": \"loop\", \"pipelines\": %d, \"backends\": %zu, \"max_batch\": %u, \"depth\": %u, "
              "\"host_ring\": %s, \"profiled\": %s, \"cpus\": \"%s\", \"pool_mbufs\": %zu, \"mbuf_stride\": %u, \"huge_pages\": %s, \"hw_queues\": \"%s\", \"zero_copy\": %s, \"drop_on_full\": %s, \"rx_per_pipeline\": %llu, \"rx\": %llu, \"tx\": %llu, "
              "\"dropped\": %llu, \"would_panic\": %llu, \"batches\": %llu, \"enqueue_stalls\": %llu, \"seconds_max\": %.6f, "
              "\"aggregate_mpps\": %.2f, \"per_pipeline_mpps\": [%s], \"producer_seconds\": [%s], "
              "\"us_per_batch\": {\"pull\": %.2f, \"submit\": %.2f, \"query\": %.2f, \"queries\": %.1f, "
              "\"wait\": %.2f, \"enqueue\": %.2f}}\n",
              pipelines, names.size(), nb::cap_batch(batch), depth, server ? "true" : "false", profiled ? "true" : "false", cpu_list.c_str(), res[0].pool, object, huge_all ? "true" : "false",
              std::getenv("GPU_MAX_HW_QUEUES") ? std::getenv("GPU_MAX_HW_QUEUES") : "", zero_copy ? "true" : "false",
              drop_on_full ? "true" : "false", static_cast<unsigned long long>(total),
              static_cast<unsigned long long>(rx_all), static_cast<unsigned long long>(tx_all),
              static_cast<unsigned long long>(dropped), static_cast<unsigned long long>(panic),
              static_cast<unsigned long long>(batches), static_cast<unsigned long long>(stalls), tmax, tmax > 0 ? rx_all / tmax / 1e6 : 0.0, per.c_str(),
              prod.c_str(), 1e6 * pr.pull / std::max<uint64_t>(batches, 1), 1e6 * pr.submit / std::max<uint64_t>(batches, 1),
              1e6 * pr.query / std::max<uint64_t>(batches, 1), static_cast<double>(pr.queries) / std::max<uint64_t>(batches, 1),
              1e6 * pr.wait / std::max<uint64_t>(batches, 1), 1e6 * pr.enqueue / std::max<uint64_t>(batches, 1));
  return tx_all + dropped + panic == rx_all ? 0 : 1;
}

}  // namespace

int main(int argc, char** argv) {
  std::string rx, tx, order;
  std::vector<std::string> names = {"Larry", "Curly", "Moe"};
  uint64_t table = 65537, loop = 0;
  uint32_t batch = nb::kMaxGpuBatch, depth = nb::kMaxDepth;
  int pipelines = 1, hw_queues = 0, ring_blocks = -1;
  // mbufs per replay port (0: at least 8,192 and the batches in flight plus two queues' worth,
  // depth x batch + 2,048), rounded up to whole copies of the capture by LoopPort.  The reference's default pool is 2,047 mbufs
  // (DEFAULT_POOL_SIZE, config/config_reader.rs:8) for a producer that holds no batch in flight; a
  // pool far larger than needed only spreads the mbufs' lines over more cache (64k mbufs: 297 against
  // 370 Mpps at 16 pipelines, profiles/r06_dropin_pool.json)
  size_t pool_mbufs = 0;
  bool profiled = true, local = true, spread = true;
  // mempool object stride: 128-B rte_mbuf + 128-B headroom + 2,048-B data room + 64-B object header
  // (37 lines: consecutive frames fall on different cache sets, as rte_mempool spreads them)
  uint32_t object = 2368;
  bool zero_copy = false, drop_on_full = false, huge = true;
  for (int i = 1; i + 1 < argc; i += 2) {
    const std::string k = argv[i], v = argv[i + 1];
    if (k == "--rx") rx = v;
    else if (k == "--tx") tx = v;
    else if (k == "--order") order = v;
    else if (k == "--table") table = std::strtoull(v.c_str(), nullptr, 10);
    else if (k == "--batch") batch = static_cast<uint32_t>(std::strtoul(v.c_str(), nullptr, 10));
    else if (k == "--depth") depth = static_cast<uint32_t>(std::strtoul(v.c_str(), nullptr, 10));
    else if (k == "--loop") loop = std::strtoull(v.c_str(), nullptr, 10);
    else if (k == "--pipelines") pipelines = std::atoi(v.c_str());
    else if (k == "--hw-queues") hw_queues = std::atoi(v.c_str());
    else if (k == "--hugepages") huge = std::atoi(v.c_str()) != 0;
    else if (k == "--host-ring") ring_blocks = std::atoi(v.c_str());
    else if (k == "--pool") pool_mbufs = std::strtoull(v.c_str(), nullptr, 10);
    else if (k == "--profile") profiled = std::atoi(v.c_str()) != 0;
    else if (k == "--local-cpus") local = std::atoi(v.c_str()) != 0;
    else if (k == "--spread-l3") spread = std::atoi(v.c_str()) != 0;
    else if (k == "--mbuf-stride") object = static_cast<uint32_t>(std::strtoul(v.c_str(), nullptr, 10));
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
  if (hw_queues < 0 || hw_queues > 32) {
    std::fprintf(stderr, "--hw-queues: 0 (default: the pipeline count, at least 4) .. 32\n");
    return 2;
  }
  if (rx.empty() || pipelines < 1 || pipelines > 64) {
    std::fprintf(stderr, "usage: nb_maglev --rx in.pcap [--tx out.pcap] [--backends N|--names a,b] ...\n");
    return 2;
  }
  // HIP maps a process's streams onto GPU_MAX_HW_QUEUES hardware queues (4 by default), and kernels
  // of streams that share a queue run one after another: each pipeline's stream gets a queue of its
  // own (set before the first HIP call; an explicit environment setting is kept)
  if (!std::getenv("GPU_MAX_HW_QUEUES")) {
    const int q = hw_queues ? hw_queues : std::min(32, std::max(4, pipelines));
    setenv("GPU_MAX_HW_QUEUES", std::to_string(q).c_str(), 1);
  }
  try {
    // --host-ring B: every pipeline's direct batches go to one host-batch server of B blocks (0 = the
    // library's default) instead of a kernel launch each; -1 (default) = no server
    nbg_host_ring* server = nullptr;
    if (ring_blocks >= 0)
      nb::check(nbg_host_ring_start(0, static_cast<uint32_t>(ring_blocks), 5000, &server), "nbg_host_ring_start");
    struct StopServer {
      nbg_host_ring* s;
      ~StopServer() {
        if (s && nbg_host_ring_stop(s) != NBG_OK) std::fprintf(stderr, "nb_maglev: %s\n", nbg_last_error());
      }
    } stop_server{server};
    if (loop) return run_loop(rx, names, table, batch, depth, zero_copy, drop_on_full, loop, pipelines, huge, server, pool_mbufs, profiled, local, spread, object);
    auto port = std::make_shared<nb::PcapPort>(rx);
    auto pool = port->mempool();
    if (zero_copy && pool.second) {
      uint8_t* dev = nullptr;
      nb::check(nbg_host_register(pool.first, pool.second, 0, &dev), "nbg_host_register");
    }
    nb::StandaloneScheduler sched;
    sched.set_timed(true);
    auto pipe = nb::maglev(std::make_shared<nb::ReceiveBatch>(port), sched, names, port, table, batch,
                           drop_on_full ? nb::Admission::kDropOnFull : nb::Admission::kBackpressure, depth);
    if (server) nb::check(nbg_maglev_set_host_ring(pipe.groups->handle(), server), "nbg_maglev_set_host_ring");
    // run until the capture is consumed, no batch is on the GPU and every group queue has drained
    const auto t0 = std::chrono::steady_clock::now();
    for (int idle = 0; idle < 2 * static_cast<int>(names.size() + 2);) {
      const uint64_t before = pipe.tx->sent + pipe.groups->processed();
      sched.execute_round();
      const bool progress = pipe.tx->sent + pipe.groups->processed() != before;
      idle = (port->rx_done() && pipe.groups->in_flight() == 0 && !progress) ? idle + 1 : 0;
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
                "\"zero_copy\": %s, \"max_batch\": %u, \"depth\": %u, \"drop_on_full\": %s, \"seconds\": %.6f, "
                "\"mpps\": %.2f, \"group_by_seconds\": %.6f, \"merge_send_seconds\": %.6f}\n",
                port->rx_total(), static_cast<unsigned long long>(pipe.tx->sent),
                static_cast<unsigned long long>(pipe.groups->dropped()),
                static_cast<unsigned long long>(pipe.groups->would_panic()), names.size(), zero_copy ? "true" : "false",
                pipe.groups->max_batch(), pipe.groups->depth(), drop_on_full ? "true" : "false", secs,
                secs > 0 ? port->rx_total() / secs / 1e6 : 0.0, sched.task_seconds(0), sched.task_seconds(1));
  } catch (const nb::NbError& e) {
    std::fprintf(stderr, "nb_maglev: %s\n", e.what());
    return e.code == NBG_ENODEV ? 3 : 1;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "nb_maglev: %s\n", e.what());
    return 1;
  }
  return 0;
}
