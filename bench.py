#!/usr/bin/env python3
"""Benchmark: device-resident Maglev (parse + MAC swap + FNV + LUT + per-backend FIFO grouping).

Workload (BASELINE.json configs[1], "C2"): 65 backends, 65537-slot LUT, 1,048,576 synthetic
64-B UDP frames (60-B frames in 64-B slots) per batch, resident in HBM.  One step = one batch
through `nbg_maglev_classify_device` (classify kernel + group scatter kernel).  Steps rotate
over 8 distinct batches (512 MiB > the 256 MiB Infinity Cache) so repeats are not cache hits.

Multi-GPU (`torch.distributed.run --nproc-per-node N`): packet batches shard trivially; each
rank owns its own batches (weak scaling, no data-path collective).  The LUT is built on rank 0
and broadcast once over RCCL (setup, untimed).

Prints ONE JSON line on rank 0 (see DESIGN.md "Measurement").
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

N_BACKENDS = 65
TABLE = 65537
BATCH = 1 << 20
SLOT = 64
FRAME = 60
N_BATCHES = 8
SEED = 0x4E42474D41474C56
# algorithmic bytes per packet: classify kernel = 64 B read + 12 B MAC write
# + 2 B backend write; whole path adds the scatter's 4 B perm write (= 82 B, C2).
CLASSIFY_BYTES = 64 + 12 + 2
PATH_BYTES = 82
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(batches_host, lut, target_cpu_s=12.0):
    """Reference per-core loop restated in C (oracle/, kind "port"), timed on this host's cores."""
    import ctypes as C

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import orc  # test infrastructure: the oracle is only the baseline/checker here

    L = orc.lib()
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    threads = max(1, min(cores, 16))
    lut32 = np.ascontiguousarray(lut, dtype=np.uint32)
    bufs = [b.copy() for b in batches_host[:2]]
    # one timing pass to size the sample
    t = L.orc_cpu_baseline(bufs[0].ctypes.data, None, SLOT, None, FRAME, BATCH, lut32.ctypes.data, TABLE,
                           N_BACKENDS, 1, threads, None)
    passes = max(1, int(target_cpu_s / max(t * threads, 1e-6)))
    passes = min(passes, 400)
    total_s = 0.0
    for p in range(passes):
        b = bufs[p % len(bufs)]
        total_s += L.orc_cpu_baseline(b.ctypes.data, None, SLOT, None, FRAME, BATCH, lut32.ctypes.data, TABLE,
                                      N_BACKENDS, 1, threads, None)
    mpps = passes * BATCH / total_s / 1e6
    try:
        model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except Exception:
        model = "unknown"
    _ = C
    return {"value": round(mpps, 2), "unit": "Mpps", "cores": threads, "kind": "port",
            "sample": f"{passes} passes x 1,048,576 C2 packets (64-B UDP, 65 backends, FNV memo map as "
                      f"nf.rs:91,104, 32-pkt bursts, per-group rings), {threads} pinned threads, "
                      f"{total_s * threads:.1f} CPU-s; host CPU: {model}"}


def read_traffic():
    """HBM bytes per classify launch from the committed PMC profile (profiles/pmc_*.json), if any."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json")))
    if not files:
        return None
    try:
        d = json.load(open(files[-1]))
        return d.get("classify_hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--lut-global", action="store_true", help="L2-gather LUT instead of LDS-staged")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    import netbricks_amd as nb

    names = [f"backend-{i}" for i in range(N_BACKENDS)]
    if world > 1:
        lut_t = torch.empty(TABLE, dtype=torch.int32, device=dev)
        if rank == 0:
            lut_t.copy_(torch.from_numpy(nb.build_lut(names, TABLE).astype(np.int32)))
        dist.broadcast(lut_t, 0)  # RCCL over xGMI, once per backend set
        lut = lut_t.cpu().numpy().astype(np.uint16)
        mg = nb.Maglev(lut=lut, n_backends=N_BACKENDS, device=local)
    else:
        mg = nb.Maglev(names, TABLE, device=local)
        lut = mg.lut()
    mg.reserve(BATCH)

    t0 = time.time()
    host = []
    dbufs = []
    for b in range(N_BATCHES):
        buf, _, _ = nb.make_trace(BATCH, 0, seed=SEED + 1000003 * rank + b)
        host.append(buf)
        dbufs.append(torch.from_numpy(buf).to(dev))
    log(f"[rank {rank}] traces ready in {time.time() - t0:.1f}s")
    backend = torch.empty(BATCH, dtype=torch.uint16, device=dev)
    perm = torch.empty(BATCH, dtype=torch.uint32, device=dev)
    counts = torch.empty(N_BACKENDS + 1, dtype=torch.uint32, device=dev)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream

    def step(i, ev=None):
        if ev is not None:
            ev[0].record(stream)
        mg.group_by(dbufs[i % N_BATCHES], BATCH, stride=SLOT, frame_len=FRAME, swap_macs=True,
                    lut_global=args.lut_global, backend=backend, perm=perm, counts=counts, stream=sp)
        if ev is not None:
            ev[1].record(stream)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize(dev)
    mg.check()

    # ---- timed region: K steps, events around each step on the launch stream
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    for i in range(args.steps):
        step(i, evs[i])
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t_start
    if world > 1:
        dist.barrier()
    step_ms = np.array([a.elapsed_time(b) for a, b in evs])
    dev_elapsed = evs[0][0].elapsed_time(evs[-1][1]) / 1e3
    mg.check()

    t = torch.tensor([elapsed, dev_elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, dev_elapsed = float(t[0]), float(t[1])

    # ---- per-kernel roofline: split classify / scatter with events in a second pass
    kev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
            torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    for i in range(args.steps):
        kev[i][0].record(stream)
        mg.group_by(dbufs[i % N_BATCHES], BATCH, stride=SLOT, frame_len=FRAME, swap_macs=True,
                    lut_global=args.lut_global, backend=backend, counts=counts, scatter=False, stream=sp)
        kev[i][1].record(stream)
    torch.cuda.synchronize(dev)
    classify_only_ms = float(np.mean([a.elapsed_time(b) for a, b, _ in kev]))

    total_pkts = BATCH * args.steps * world
    mpps = total_pkts / elapsed / 1e6
    step_med = float(np.median(step_ms))
    step_avg = float(np.mean(step_ms))
    path_gbps = BATCH * PATH_BYTES / (step_avg / 1e3) / 1e9
    ach = BATCH * CLASSIFY_BYTES / (classify_only_ms / 1e3) / 1e9
    traffic = read_traffic()

    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            try:
                cpu = cpu_baseline(host, lut)
            except Exception as e:  # baseline is informational; never fail the bench on it
                log(f"cpu baseline failed: {e}")
        line = {
            "metric": "Mpps + HBM GB/s device-resident Maglev (64B pkts)",
            "value": round(mpps, 1),
            "unit": "Mpps",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": "C2: Maglev 65 backends / 65537-slot LUT, 64B synthetic UDP, "
                                   "1M-packet device-resident batch per GPU",
                       "backends": N_BACKENDS, "table_size": TABLE, "batch_pkts": BATCH, "slot_bytes": SLOT,
                       "frame_bytes": FRAME, "rotating_batches": N_BATCHES, "swap_macs": True, "group_by": True,
                       "lut": "global" if args.lut_global else "lds", "parallelism": f"shard{world}"},
            "hbm_gbps_path": round(path_gbps, 1),
            "step_ms_median": round(step_med, 4),
            "device_mpps_per_gpu": round(BATCH * args.steps / dev_elapsed / 1e6, 1),
            "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(ach / HBM_PEAK_GBPS, 4), "traffic": traffic,
                         "kernel": "classify_kernel (grouping variant, as in the step)", "bytes_per_pkt": CLASSIFY_BYTES,
                         "avg_launch_us": round(classify_only_ms * 1e3, 2)},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    mg.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
