#!/usr/bin/env python3
"""Benchmark: device-resident Maglev (parse + MAC swap + FNV + LUT + per-backend FIFO grouping).

Workload (BASELINE.json configs[1], "C2"): 65 backends, 65537-slot LUT, 1,048,576 synthetic
64-B UDP frames (60-B frames in 64-B slots) per batch, resident in HBM.  One step = one batch
through `nbg_maglev_classify_device` (classify kernel + grouping kernel), MAC swap in place.
Steps rotate over 8 distinct batches (512 MiB > the 256 MiB Infinity Cache) and are issued
round-robin on `--streams` (default 3) HIP streams (independent batches, one handle per stream: NetBricks
runs one pipeline per RX queue), so one batch's latency-bound grouping overlaps the next
batch's bandwidth-bound classify.  Three streams plus the default stream fill HIP's 4 hardware
queues (GPU_MAX_HW_QUEUES) one each; a fourth stream would share a queue and serialise behind
another (measured: 3 streams 34.0-35.3 Gpps, 4 streams 32.3-32.8 on one box).

Roofline: the classify kernel (dominant) is timed with HIP events around each launch in a
separate single-stream pass (NBG_DEFER_GROUP splits it from the grouping kernel).

Multi-GPU (`torch.distributed.run --nproc-per-node N`): packet batches shard trivially; each
rank owns its own batches (weak scaling, no data-path collective).  The LUT is built on rank 0
and broadcast once over RCCL (setup, untimed).

Prints ONE JSON line on rank 0 (see DESIGN.md "Measurement").
"""
from __future__ import annotations

import argparse
import glob
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
# + 2 B backend write; the whole path adds the grouping kernel's 4 B perm write (= 82 B, C2).
CLASSIFY_BYTES = 64 + 12 + 2
PATH_BYTES = 82
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(batch_host, lut, target_cpu_s=12.0):
    """Reference per-core loop restated in C (oracle/, kind "port"), timed on this host's cores."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import orc  # test infrastructure: the oracle is the baseline/checker only

    L = orc.lib()
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    threads = max(1, min(cores, 16))
    lut32 = np.ascontiguousarray(lut, dtype=np.uint32)
    buf = batch_host.copy()

    def one():
        return L.orc_cpu_baseline(buf.ctypes.data, None, SLOT, None, FRAME, BATCH, lut32.ctypes.data, TABLE,
                                  N_BACKENDS, 1, threads, None)

    one()  # cold pass: page faults, thread start-up
    t = one()  # a warm pass sizes the sample
    passes = int(min(max(1, target_cpu_s / max(t * threads, 1e-6)), 2000))
    total_s = sum(one() for _ in range(passes))
    mpps = passes * BATCH / total_s / 1e6
    try:
        model = [ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name")][0]
    except Exception:
        model = "unknown"
    return {"value": round(mpps, 2), "unit": "Mpps", "cores": threads, "kind": "port",
            "sample": f"{passes} passes over one 1,048,576-packet C2 batch (64-B UDP, 65 backends, M=65537; "
                      f"FNV-keyed memo map nf.rs:91,104, 32-pkt bursts, per-group 1024-slot rings), "
                      f"{threads} pinned threads, {total_s * threads:.1f} CPU-s; host CPU: {model}"}


def shard_seed(rank: int, batch: int) -> int:
    """Seed of rank `rank`'s batch `batch`: every rank owns distinct packets (weak scaling)."""
    return SEED + 1000003 * rank + batch


def shared_lut(names, table, rank, world, device):
    """Rank 0 builds the Maglev LUT (Maglev::new, nf.rs:70-76) and broadcasts it once (RCCL over
    xGMI on GPUs, gloo in the CPU tests); every rank returns the same u16 table."""
    import torch
    import torch.distributed as dist

    import netbricks_amd as nb

    lut_t = torch.empty(table, dtype=torch.int32, device=device)
    if rank == 0:
        lut_t.copy_(torch.from_numpy(nb.build_lut(names, table).astype(np.int32)))
    if world > 1:
        dist.broadcast(lut_t, 0)
    return lut_t.cpu().numpy().astype(np.uint16)


class KernelTimer:
    """HIP events created with hipEventDisableSystemFence (timing only): a default timing event's
    system-scope release writes back and invalidates L2 at every record, which lands inside the
    interval of a kernel that writes (the in-place MAC swap) and inflates its measured duration.
    Uses the HIP runtime torch already loaded (same soname, one runtime per process)."""

    FLAGS = 0x20000000  # hipEventDisableSystemFence

    def __init__(self, n: int):
        import ctypes as C

        self.C = C
        self.hip = C.CDLL("libamdhip64.so.7")
        self.ev = [(C.c_void_p(), C.c_void_p()) for _ in range(n)]
        for a, b in self.ev:
            for e in (a, b):
                rc = self.hip.hipEventCreateWithFlags(C.byref(e), C.c_uint(self.FLAGS))
                if rc != 0:
                    raise RuntimeError(f"hipEventCreateWithFlags failed ({rc})")

    def start(self, i: int, stream: int) -> None:
        self.hip.hipEventRecord(self.ev[i][0], self.C.c_void_p(stream))

    def stop(self, i: int, stream: int) -> None:
        self.hip.hipEventRecord(self.ev[i][1], self.C.c_void_p(stream))

    def ms(self):
        out = []
        for a, b in self.ev:
            self.hip.hipEventSynchronize(b)
            t = self.C.c_float()
            if self.hip.hipEventElapsedTime(self.C.byref(t), a, b) != 0:
                raise RuntimeError("hipEventElapsedTime failed")
            out.append(t.value)
        return np.array(out)

    def close(self) -> None:
        for a, b in self.ev:
            self.hip.hipEventDestroy(a)
            self.hip.hipEventDestroy(b)


def scatter_shard(global_buf, out, rank: int, world: int) -> None:
    """Config C4's data-path collective: rank 0 holds the whole batch (world contiguous shards)
    and scatters shard r to rank r (RCCL ncclScatter over xGMI on GPUs; gloo in the CPU tests).
    Shard-major order == global packet order, so per-shard grouping composes."""
    import torch.distributed as dist

    if rank == 0:
        dist.scatter(out, list(global_buf.chunk(world)), src=0)
    else:
        dist.scatter(out, None, src=0)


def gather_results(backend, counts, gbuf, gcounts, rank: int, world: int) -> None:
    """Config C4's return leg: rank 0 collects every shard's backend[] (u16, sent as bytes: RCCL has
    no 16-bit integer type) and per-group counts (RCCL gather over xGMI on GPUs; gloo in the CPU
    tests).  Shard-major order == global packet order."""
    import torch
    import torch.distributed as dist

    b = backend.view(torch.uint8)
    c = counts.view(torch.int32)
    if rank == 0:
        dist.gather(b, list(gbuf.chunk(world)), dst=0)
        dist.gather(c, list(gcounts.chunk(world)), dst=0)
    else:
        dist.gather(b, None, dst=0)
        dist.gather(c, None, dst=0)


def read_traffic():
    """HBM bytes per classify launch from the committed PMC profile (profiles/pmc_*.json), if any."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json")))
    if not files:
        return None
    try:
        return json.load(open(files[-1])).get("classify_hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--streams", type=int, default=3)
    ap.add_argument("--mac-record", action="store_true",
                    help="write the swapped MACs as dense 12-B egress records instead of in place")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--scatter-steps", type=int, default=50,
                    help="N>1: steps of the scatter-inclusive pass (RCCL scatter from rank 0 + classify); 0 = skip")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    import netbricks_amd as nb

    names = [f"backend-{i}" for i in range(N_BACKENDS)]
    if world > 1:
        lut = shared_lut(names, TABLE, rank, world, dev)  # RCCL broadcast, once per backend set
        mgs = [nb.Maglev(lut=lut, n_backends=N_BACKENDS, device=local) for _ in range(args.streams)]
    else:
        mgs = [nb.Maglev(names, TABLE, device=local) for _ in range(args.streams)]
        lut = mgs[0].lut()

    t0 = time.time()
    host0 = None
    dbufs = []
    for b in range(N_BATCHES):
        buf, _, _ = nb.make_trace(BATCH, 0, seed=shard_seed(rank, b))
        if b == 0:
            host0 = buf.copy()
        dbufs.append(torch.from_numpy(buf).to(dev))
    log(f"[rank {rank}] traces ready in {time.time() - t0:.1f}s")
    streams = [torch.cuda.Stream(dev) for _ in range(args.streams)]
    outs = [dict(backend=torch.empty(BATCH, dtype=torch.uint16, device=dev),
                 perm=torch.empty(BATCH, dtype=torch.uint32, device=dev),
                 counts=torch.empty(N_BACKENDS + 1, dtype=torch.uint32, device=dev),
                 mac_out=torch.empty(BATCH * 12, dtype=torch.uint8, device=dev) if args.mac_record else None)
            for _ in range(args.streams)]

    def step(i):
        j = i % args.streams
        mgs[j].group_by(dbufs[i % N_BATCHES], BATCH, stride=SLOT, frame_len=FRAME, swap_macs=True,
                        stream=streams[j].cuda_stream, **outs[j])

    def sync_all():
        torch.cuda.synchronize(dev)

    for i in range(args.warmup):
        step(i)
    sync_all()
    for m in mgs:
        m.check()

    # ---- timed region: K steps over all streams, bracketed by barrier + synchronize
    if world > 1:
        dist.barrier()
    sync_all()
    start_ev = torch.cuda.Event(enable_timing=True)
    start_ev.record(torch.cuda.current_stream(dev))
    for st in streams:
        st.wait_event(start_ev)
    t_start = time.perf_counter()
    for i in range(args.steps):
        step(i)
    sync_all()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        dist.barrier()
    for m in mgs:
        m.check()
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t[0])

    # ---- C4 scatter-inclusive pass (N > 1): every step rank 0 scatters world x 1M packets over
    #      xGMI and each rank classifies its shard; reported beside the device-resident value
    scatter = None
    if world > 1 and args.scatter_steps > 0:
        try:
            recv = torch.empty(BATCH * SLOT, dtype=torch.uint8, device=dev)
            glob = torch.cat([dbufs[0]] + [torch.empty_like(dbufs[0]) for _ in range(world - 1)]) if rank == 0 else None
            if rank == 0:
                for r in range(1, world):  # rank 0 holds every rank's first shard (same seeds as the ranks own)
                    buf_r, _, _ = nb.make_trace(BATCH, 0, seed=shard_seed(r, 0))
                    glob[r * BATCH * SLOT:(r + 1) * BATCH * SLOT].copy_(torch.from_numpy(buf_r))
            cur = torch.cuda.current_stream(dev).cuda_stream
            gb = torch.empty(world * BATCH * 2, dtype=torch.uint8, device=dev) if rank == 0 else None
            gc = torch.empty(world * (N_BACKENDS + 1), dtype=torch.int32, device=dev) if rank == 0 else None

            def sstep():
                scatter_shard(glob, recv, rank, world)
                mgs[0].group_by(recv, BATCH, stride=SLOT, frame_len=FRAME, swap_macs=True, stream=cur, **outs[0])
                gather_results(outs[0]["backend"], outs[0]["counts"], gb, gc, rank, world)

            for _ in range(3):
                sstep()
            sync_all()
            dist.barrier()
            sync_all()
            t1 = time.perf_counter()
            for _ in range(args.scatter_steps):
                sstep()
            sync_all()
            st_el = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device=dev)
            dist.all_reduce(st_el, op=dist.ReduceOp.MAX)
            st_s = float(st_el[0])
            if rank == 0 and int(gc.sum()) != world * BATCH:
                raise RuntimeError(f"gathered counts sum {int(gc.sum())} != {world * BATCH}")
            scatter = {"value": round(BATCH * world * args.scatter_steps / st_s / 1e6, 1), "unit": "Mpps",
                       "ms_per_step": round(st_s / args.scatter_steps * 1e3, 4), "steps": args.scatter_steps,
                       "root_egress_GBps": round(BATCH * SLOT * (world - 1) * args.scatter_steps / st_s / 1e9, 1),
                       "what": "rank 0 scatters world x 1M 64-B packets (ncclScatter over xGMI), each rank classifies "
                               "its shard (MAC swap + grouping), rank 0 gathers every shard's backend[] and counts "
                               "(ncclGather); single stream per rank"}
            del recv, glob, gb, gc
        except Exception as e:  # informational; the device-resident value above stands on its own
            log(f"[rank {rank}] scatter-inclusive pass failed: {e}")
            scatter = {"error": str(e)[:200]}

    # ---- roofline pass: classify kernel timed alone (single stream, HIP events around each launch
    #      on the stream it runs on; grouping deferred and launched after the stop event)
    st = streams[0]
    kt, gt = KernelTimer(args.steps), KernelTimer(args.steps)
    t_single = time.perf_counter()
    for i in range(args.steps):
        kt.start(i, st.cuda_stream)
        mgs[0].group_by(dbufs[i % N_BATCHES], BATCH, stride=SLOT, frame_len=FRAME, swap_macs=True,
                        defer_group=True, stream=st.cuda_stream, **outs[0])
        kt.stop(i, st.cuda_stream)
        gt.start(i, st.cuda_stream)
        mgs[0].finish_group(st.cuda_stream)
        gt.stop(i, st.cuda_stream)
    sync_all()
    single_ms = (time.perf_counter() - t_single) / args.steps * 1e3
    classify_ms = kt.ms()
    group_ms = gt.ms()
    kt.close()
    gt.close()

    total_pkts = BATCH * args.steps * world
    mpps = total_pkts / elapsed / 1e6
    ms_step = elapsed / args.steps * 1e3
    path_gbps = BATCH * PATH_BYTES * args.steps / elapsed / 1e9  # per GPU
    ach = BATCH * CLASSIFY_BYTES / (classify_ms.mean() / 1e3) / 1e9
    traffic = read_traffic()

    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            try:
                cpu = cpu_baseline(host0, lut)
            except Exception as e:  # the baseline is informational; never fail the bench on it
                log(f"cpu baseline failed: {e}")
        line = {
            "metric": "Mpps + HBM GB/s device-resident Maglev (64B pkts)",
            "value": round(mpps, 1),
            "unit": "Mpps",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": "C2: Maglev 65 backends / 65537-slot LUT, 64B synthetic UDP, "
                                   "1M-packet device-resident batch per GPU",
                       "backends": N_BACKENDS, "table_size": TABLE, "batch_pkts": BATCH, "slot_bytes": SLOT,
                       "frame_bytes": FRAME, "rotating_batches": N_BATCHES,
                       "mac_swap": "12-B egress records" if args.mac_record else "in place",
                       "group_by": "perm + counts", "streams": args.streams, "parallelism": f"shard{world}"},
            "hbm_gbps_per_gpu": round(path_gbps, 1),
            "hbm_bytes_per_pkt": PATH_BYTES,
            "single_stream_ms_per_step": round(single_ms, 5),
            "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(ach / HBM_PEAK_GBPS, 4), "traffic": traffic,
                         "kernel": "classify_kernel<GlobalU8,F4,HIST,1>", "bytes_per_pkt": CLASSIFY_BYTES,
                         "pkts_per_launch": BATCH, "avg_launch_us": round(classify_ms.mean() * 1e3, 2),
                         "group_kernel_avg_us": round(group_ms.mean() * 1e3, 2)},
            "cpu_baseline": cpu,
        }
        if scatter is not None:
            line["scatter_inclusive"] = scatter
        print(json.dumps(line), flush=True)
    for m in mgs:
        m.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
