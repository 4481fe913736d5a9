#!/usr/bin/env python3
"""Throughput of the secondary BASELINE configs on one GPU (bench.py measures C2).

  c3  Maglev 1000 backends / 655373-slot LUT (u16), IMIX 7:4:1 descriptors (u32 off + u16 len),
      MAC swap in place (owned 64-B windows), per-backend grouping.
      Algorithmic bytes/pkt: 64 window + 6 descriptor + 12 MAC + 2 backend + 4 perm = 88.
  c5  chained test/lpm -> test/maglev (65 backends / 65537), IMIX descriptors, DIR-24-8 table of the
      reference's 105 routes + the mixed route set (tests/golden/lpm_routes.json); the two MAC swaps
      cancel, so packets are only read.  Bytes/pkt: 64 + 6 + 2 gate + 2 backend + 4 perm + 4 LPM = 82.

Steps rotate over 8 distinct 1M-packet batches on --streams streams (one handle per stream), timed
with events like bench.py; a single-stream pass times the classify kernel alone per launch.
Prints one JSON line per config.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BATCH = 1 << 20
N_BATCHES = 8


def cpu_baseline(cfg, names, m, routes, cpu_s=4.0):
    """The reference's per-core loop restated in C (oracle/, kind "port"; for C5 test/lpm's stage and
    group rings first), over one BATCH-packet trace of this config: all allowed cores, one core,
    and without the memo map.  Test infrastructure used as the baseline only."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import orc
    from bench import cpu_inventory

    import netbricks_amd as nb

    affinity, quota, model = cpu_inventory()
    cores = max(1, min(affinity, int(quota))) if quota else affinity
    lut = orc.lut_build(names, m)
    buf, off, ln = nb.make_trace(BATCH, 1, seed=1000)
    chain = None
    if cfg == "c5":
        rc, t24, tl = orc.lpm_build(routes["reference"] + routes["mixed"])
        chain = (t24, tl)

    def measure(threads, cache, budget):
        t, _ = orc.cpu_baseline(buf, BATCH, lut, len(names), offs=off, lens=ln, chain=chain, cache=cache,
                                threads=threads)
        reps = int(min(max(1, budget / max(t * threads, 1e-6)), 10000))
        t, _ = orc.cpu_baseline(buf, BATCH, lut, len(names), offs=off, lens=ln, chain=chain, cache=cache,
                                threads=threads, reps=reps)
        return round(BATCH * reps / t / 1e6, 1), reps

    allc, ra = measure(cores, True, cpu_s)
    single, r1 = measure(1, True, cpu_s / 4)
    nocache, rn = measure(cores, False, cpu_s / 2)
    return {"value": allc, "unit": "Mpps", "cores": cores, "kind": "port", "single_core_mpps": single,
            "no_cache_mpps": nocache, "cpu_model": model,
            "sample": f"one {BATCH:,}-packet IMIX trace of this config: {cores} pinned threads x {ra} passes, "
                      f"1 thread x {r1} passes, no memo map {rn} passes"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3,c5")
    ap.add_argument("--streams", type=int, default=3)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--stream-desc", action="store_true", help="NBG_STREAM_DESC: the streaming classify kernel")
    ap.add_argument("--lut-lds", action="store_true", help="NBG_LUT_LDS: stage the LUT in LDS (u8/u16 LUT <= 72 KiB)")
    ap.add_argument("--c3-variant", default="in_place", choices=["in_place", "records", "read_only"],
                    help="C3's MAC handling: in place (default), 12-B records, or none (parse + hash + lookup)")
    ap.add_argument("--cpu-baseline", action="store_true",
                    help="also time the C port of the reference loop (oracle/) on this host's cores, same traces")
    args = ap.parse_args()
    import torch

    import netbricks_amd as nb

    dev = torch.device("cuda:0")
    routes = json.load(open(os.path.join(ROOT, "tests", "golden", "lpm_routes.json")))
    for cfg in args.config.split(","):
        if cfg in ("c3", "c3t"):  # c3t: the LDS-tiled lookup (NBG_LUT_TILED) instead of the L2 gather
            names, m, nbk = [f"be{i}" for i in range(1000)], 655373, 1000
            bytes_pkt, classify_bytes = 88, 84
        elif cfg == "c5":
            names, m, nbk = [f"backend-{i}" for i in range(65)], 65537, 65
            bytes_pkt, classify_bytes = 82, 78
        else:
            raise SystemExit(f"unknown config {cfg}")
        t0 = time.time()
        bufs, offs, lens = [], [], []
        for b in range(N_BATCHES):
            buf, off, ln = nb.make_trace(BATCH, 1, seed=1000 + b)
            bufs.append(torch.from_numpy(buf).to(dev))
            offs.append(torch.from_numpy(off.view(np.int32)).to(dev).view(torch.uint32))
            lens.append(torch.from_numpy(ln.view(np.int16)).to(dev).view(torch.uint16))
        print(f"[{cfg}] traces in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
        S = args.streams
        mgs = [nb.Maglev(names, m) for _ in range(S)]
        lpm = nb.Lpm(routes["reference"] + routes["mixed"]) if cfg == "c5" else None
        sts = [torch.cuda.Stream(dev) for _ in range(S)]
        recs = [torch.empty(BATCH * 12, dtype=torch.uint8, device=dev) for _ in range(S)]
        c3v = args.c3_variant
        if cfg.startswith("c3") and c3v != "in_place":
            classify_bytes = 84 if c3v == "records" else 72  # 64 + 6 descriptor + 2 backend (+ 12 record)
            bytes_pkt = classify_bytes + 4
        outs = [dict(backend=torch.empty(BATCH, dtype=torch.uint16, device=dev),
                     perm=torch.empty(BATCH, dtype=torch.uint32, device=dev),
                     counts=torch.empty(nbk + 1, dtype=torch.uint32, device=dev)) for _ in range(S)]
        gates = [torch.empty(BATCH, dtype=torch.uint16, device=dev) for _ in range(S)]

        def step(i, j=None, defer=False):
            j = i % S if j is None else j
            k = i % N_BATCHES
            if cfg == "c5":
                nb.chain_lpm_maglev(mgs[j], lpm, bufs[k], BATCH, offsets=offs[k], lens=lens[k], owned_windows=True, bounds_check=False,
                                    defer_group=defer, gate=gates[j], stream=sts[j].cuda_stream,
                                    stream_desc=args.stream_desc, lut_lds=args.lut_lds, **outs[j])
            else:
                mgs[j].group_by(bufs[k], BATCH, offsets=offs[k], lens=lens[k], owned_windows=True, bounds_check=False,
                                swap_macs=c3v != "read_only", mac_out=recs[j] if c3v == "records" else None,
                                defer_group=defer, lut_tiled=cfg == "c3t", stream=sts[j].cuda_stream,
                                stream_desc=args.stream_desc, lut_lds=args.lut_lds, **outs[j])

        for i in range(args.warmup):
            step(i)
        torch.cuda.synchronize()
        ev0 = torch.cuda.Event(enable_timing=True)
        ev0.record(torch.cuda.current_stream(dev))
        for st in sts:
            st.wait_event(ev0)
        t_start = time.perf_counter()
        for i in range(args.steps):
            step(i)
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t_start
        # classify kernel alone (single stream, fence-free HIP events around each launch)
        from bench import KernelTimer

        st = sts[0]
        kt = KernelTimer(args.steps)
        for i in range(args.steps):
            kt.start(i, st.cuda_stream)
            step(i, 0, defer=True)
            kt.stop(i, st.cuda_stream)
            mgs[0].finish_group(st.cuda_stream)
        torch.cuda.synchronize()
        for mg in mgs:
            mg.check()
        kus = float(kt.ms().mean()) * 1e3
        kt.close()
        mpps = BATCH * args.steps / elapsed / 1e6
        line = {"config": cfg + ("" if cfg == "c5" or c3v == "in_place" else f"_{c3v}"), "mpps": round(mpps, 1), "us_per_batch": round(elapsed / args.steps * 1e6, 2),
                "streams": S, "batch_pkts": BATCH, "backends": nbk, "table_size": m,
                "path_bytes_per_pkt": bytes_pkt, "path_gbps": round(mpps * bytes_pkt / 1e3, 1),
                "classify_us": round(kus, 2), "classify_bytes_per_pkt": classify_bytes,
                "classify_gbps": round(BATCH * classify_bytes / kus / 1e3, 1),
                "classify_frac_of_8TBps": round(BATCH * classify_bytes / kus / 1e3 / 8000.0, 4)}
        if cfg == "c5":
            g = gates[0].view(torch.int16).cpu().numpy().view(np.uint16)
            line["gate_hist"] = {str(k): int(v) for k, v in zip(*np.unique(g, return_counts=True))}
        if args.cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(cfg, names, m, routes)
        print(json.dumps(line), flush=True)
        for mg in mgs:
            mg.close()
        if lpm is not None:
            lpm.close()
        del bufs, offs, lens
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
