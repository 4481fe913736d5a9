#!/usr/bin/env python3
"""Throughput of the drop-in operator path (north_star: test/maglev's ReceiveBatch -> parse ->
transform -> group_by surface): nb_maglev --loop, the C++ mirror of test/maglev (operators.hpp) with
the pipelined GPU group_by producer, at the reference's own queue limit (1024-slot group queues,
992-packet batches = 31 RX bursts, framework/src/queues/mpsc_mbuf_queue.rs:261-265,
framework/src/operators/group_by.rs:43-55).

1, 4 and 16 pipelines, one thread + Maglev handle + stream each (one pipeline per RX queue and core,
scheduler/context.rs:55-69,241-255), each replaying a C1-style capture (10k 64-B UDP frames, 65
backends / 65537) through a LoopPort (the reference's VirtualPort: recv hands out mbufs, send frees
them).  Producer and consumer (merge + send) tasks share each pipeline's thread, as in the reference.
Every pipeline's batches go to the device's host-batch server (nbg_host_ring_*, 64 blocks), up to 8
in flight per pipeline; each pipeline's thread is pinned to a CPU on the GPU's socket and its port's
mempool holds 10,000 mbufs (nb_maglev's defaults).

This process never initialises the GPU: it writes the capture (host trace generator) and runs
nb_maglev as child processes.  Prints one JSON line.
"""
import argparse
import json
import os
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
NB = os.path.join(ROOT, "netbricks_amd", "host", "nb_maglev")
SERVER_BLOCKS = 64  # the host-batch server's blocks (16 pipelines: 32 -> 468/387, 48 -> 492/494, 64 -> 543/491,
                    # 96 -> 417/431 Mpps in two rounds, profiles/r06_dropin_server_sweep.json)


def write_c1_pcap(path, n=10000, seed=2024):
    import netbricks_amd as nb  # host-only: the trace generator needs no GPU

    buf, off, ln = nb.make_trace(n, 0, seed=seed)
    with open(path, "wb") as f:
        f.write(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 1))
        for i, (o, l) in enumerate(zip(off.tolist(), ln.tolist())):
            f.write(struct.pack("<IIII", i, 0, l, l))
            f.write(buf[o:o + l].tobytes())


def run(pcap, pipelines, total, batch=992, depth=None, zero_copy=False, drop_on_full=False, hw_queues=0, huge=True,
        server=-1, pool=None, profile=True, local_cpus=True, spread=True, env=None, timeout=120):
    args = [(env or {}).get("NB_BIN", NB), "--rx", pcap, "--backends", "65", "--batch", str(batch), "--loop", str(total),
            "--pipelines", str(pipelines), "--zero-copy", "1" if zero_copy else "0",
            "--drop-on-full", "1" if drop_on_full else "0", "--hw-queues", str(hw_queues),
            "--hugepages", "1" if huge else "0", "--host-ring", str(server)]
    if depth:
        args += ["--depth", str(depth)]
    if pool:
        args += ["--pool", str(pool)]
    args += (env or {}).get("NB_EXTRA_ARGS", "").split()  # an A/B of nb_maglev options (--ab-env)
    if not profile:
        args += ["--profile", "0"]
    if not local_cpus:
        args += ["--local-cpus", "0"]
    if not spread:
        args += ["--spread-l3", "0"]
    r = subprocess.run(["timeout", "-k", "5", str(timeout)] + args, capture_output=True, text=True,
                       env=dict(os.environ, **(env or {})))
    if r.returncode != 0:
        return {"error": f"rc={r.returncode}: {r.stderr[-300:]}"}
    return json.loads(r.stdout.strip().splitlines()[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--total", type=int, default=20_000_000, help="packets received per pipeline")
    ap.add_argument("--pipelines", default="1,4,16")
    ap.add_argument("--extra", action="store_true",
                    help="also zero-copy, depth 3, drop-on-full, 4-KiB pages, and a kernel launch per batch")
    ap.add_argument("--write-pcap", help="only write the C1-style capture to this path")
    ap.add_argument("--tune", action="store_true", help="only the host-gather prefetch distance and server size A/B")
    ap.add_argument("--ab-lib", help="only an A/B of this tree's libnbgpu.so against the one in this directory "
                                     "(LD_LIBRARY_PATH; nb_maglev's RUNPATH yields to it) at 16 and 1 pipelines, 3 rounds")
    ap.add_argument("--ab-bin", help="only an A/B of this tree's nb_maglev against this binary (16 and 1 pipelines, "
                                     "3 alternating rounds)")
    ap.add_argument("--ab-env", help="only an A/B of this tree against KEY=VALUE in the environment (16 and 1 "
                                     "pipelines, 3 alternating rounds)")
    ap.add_argument("--depth-sweep", action="store_true",
                    help="only batches in flight per pipeline (4, 8) x server blocks (48, 64) at 16 pipelines")
    ap.add_argument("--server-sweep", action="store_true",
                    help="only the host-batch server's block count at 16 pipelines (and 4), 2 rounds")
    ap.add_argument("--ab-spread", action="store_true",
                    help="only the thread placement A/B at 16 pipelines (spread over L3 caches or not), 3 rounds")
    ap.add_argument("--pool-sweep", action="store_true",
                    help="only the mempool size A/B (mbufs per pipeline's port) at 1, 4 and 16 pipelines")
    args = ap.parse_args()
    if args.write_pcap:
        write_c1_pcap(args.write_pcap)
        return
    out = {}
    with tempfile.TemporaryDirectory() as d:
        pcap = os.path.join(d, "c1.pcap")
        write_c1_pcap(pcap)
        # the rows: every pipeline's batches through the device's host-batch server (32 blocks), 4 in
        # flight per pipeline, staged 48-B windows; then (extra) each choice against its alternative
        runs = [(f"p{p}", dict(pipelines=int(p), server=SERVER_BLOCKS)) for p in args.pipelines.split(",")]
        if args.tune:
            runs = [(f"p16_server_ahead{a}", dict(pipelines=16, server=32, env={"NBG_GATHER_AHEAD": str(a)}))
                    for a in (16, 32, 64)]
            runs += [("p16_server64", dict(pipelines=16, server=64)), ("p16_server16", dict(pipelines=16, server=16)),
                     ("p16_server_depth2", dict(pipelines=16, server=32, depth=2)),
                     ("p1_zero_copy", dict(pipelines=1, zero_copy=True)),
                     ("p1_zero_copy_ahead32", dict(pipelines=1, zero_copy=True, env={"NBG_GATHER_AHEAD": "32"}))]
        if args.ab_lib or args.ab_env or args.ab_bin:
            alt = ({"LD_LIBRARY_PATH": os.path.abspath(args.ab_lib)} if args.ab_lib
                   else {"NB_BIN": os.path.abspath(args.ab_bin), "LD_LIBRARY_PATH": os.path.join(ROOT, "netbricks_amd")}
                   if args.ab_bin
                   else dict([args.ab_env.split("=", 1)]))
            runs = [(f"p{p}_{'alt' if k % 2 else 'tree'}_r{k // 2}",
                     dict(pipelines=p, server=SERVER_BLOCKS, env=alt if k % 2 else None))
                    for p in (16, 1) for k in range(6)]
        if args.depth_sweep:
            runs = [(f"p16_depth{d}_server{b}_r{k}", dict(pipelines=16, server=b, depth=d))
                    for k in range(2) for b in (48, 64) for d in (4, 8)]
            runs += [(f"p1_depth{d}", dict(pipelines=1, server=64, depth=d)) for d in (4, 8)]
        if args.server_sweep:
            runs = [(f"p16_server{b}_r{k}", dict(pipelines=16, server=b)) for k in range(2) for b in (32, 48, 64, 96)]
            runs += [(f"p4_server{b}", dict(pipelines=4, server=b)) for b in (16, 32)]
        if args.ab_spread:
            runs = [(f"p16_{'spread' if sp else 'packed'}_r{k}", dict(pipelines=16, server=32, spread=sp))
                    for k in range(3) for sp in (True, False)]
            runs += [(f"p4_{'spread' if sp else 'packed'}", dict(pipelines=4, server=32, spread=sp)) for sp in (True, False)]
        if args.pool_sweep:
            runs = [(f"p{p}_pool{m}{'' if prof else '_noprof'}", dict(pipelines=p, server=32, pool=m, profile=prof))
                    for p in (1, 4, 16) for m in (10000, 65536) for prof in (True, False)]
        if args.extra:
            top = max(int(p) for p in args.pipelines.split(","))
            S = SERVER_BLOCKS
            runs += [(f"p{top}_any_cpus", dict(pipelines=top, server=S, local_cpus=False)),
                     (f"p{top}_packed_cpus", dict(pipelines=top, server=S, spread=False)),
                     (f"p{top}_pool65536", dict(pipelines=top, server=S, pool=65536)),
                     (f"p{top}_noprof", dict(pipelines=top, server=S, profile=False)),
                     (f"p{top}_server32", dict(pipelines=top, server=32)),
                     (f"p{top}_depth4", dict(pipelines=top, server=S, depth=4)),
                     ("p1_depth4", dict(pipelines=1, server=S, depth=4)),
                     (f"p{top}_win48", dict(pipelines=top, server=S, env={"NBG_HOST_WIN48": "1"})),
                     ("p1_win48", dict(pipelines=1, server=S, env={"NBG_HOST_WIN48": "1"})),
                     (f"p{top}_server_zero_copy", dict(pipelines=top, server=S, zero_copy=True)),
                     ("p1_server_zero_copy", dict(pipelines=1, server=S, zero_copy=True)),
                     (f"p{top}_server_drop_on_full", dict(pipelines=top, server=S, drop_on_full=True)),
                     (f"p{top}_server_4k_pages", dict(pipelines=top, server=S, huge=False)),
                     (f"p{top}_launch", dict(pipelines=top)),
                     ("p4_launch", dict(pipelines=4)),
                     ("p1_launch", dict(pipelines=1)),
                     (f"p{top}_launch_zero_copy", dict(pipelines=top, zero_copy=True)),
                     ("p1_launch_zero_copy", dict(pipelines=1, zero_copy=True)),
                     (f"p{top}_launch_hwq4", dict(pipelines=top, hw_queues=4)),
                     (f"p{top}_launch_zero_copy_4k_pages", dict(pipelines=top, zero_copy=True, huge=False)),
                     (f"p{top}_launch_b496", dict(pipelines=top, batch=496)),
                     ("p1_launch_depth1", dict(pipelines=1, depth=1))]
        for name, kw in runs:
            r = run(pcap, total=args.total, **kw)
            out[name] = r
            print(f"{name}: {r.get('aggregate_mpps', r.get('error'))}", file=sys.stderr, flush=True)
    rows = []
    for name, r in out.items():
        if name.startswith("p") and name[1:].isdigit() and "aggregate_mpps" in r:
            per = r["per_pipeline_mpps"]
            # the producer task alone (the GPU group_by: pull, submit, wait, enqueue), the part of the
            # pipeline bench.py's cpu_baseline restates (the reference's producer loop, no consumer)
            prod = sum(r["rx_per_pipeline"] / s for s in r["producer_seconds"] if s > 0)
            rows.append({"pipelines": r["pipelines"], "per_pipeline_mpps": round(sum(per) / len(per), 2),
                         "aggregate_mpps": r["aggregate_mpps"], "producer_only_mpps": round(prod / 1e6, 1)})
    print(json.dumps({"dropin": rows, "runs": out, "batch": 992, "queue_slots": 1024, "depth": 8,
                      "server_blocks": SERVER_BLOCKS, "capture": "10k 64-B UDP frames (C1 style), 65 backends / 65537, "
                                                      "LoopPort replay (a pool of 10,000 2-KiB mbufs in huge pages at a "
                                                      "2,368-B object stride, one per frame of the capture); threads on "
                                                      "the GPU's socket, idle cores first"}))


if __name__ == "__main__":
    main()
