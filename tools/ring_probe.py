#!/usr/bin/env python3
"""Measurement (round 3): the persistent RX ring (nbg_ring_*) against one launch per batch, C2 1M
batches (8 rotating inputs), read only and in place.  The ring is fed as an RX ring is: the host
posts whenever a slot is free and records when the completed count moves, so the steady-state time
per batch is the slope of completions over the middle of the run (no launch, LUT staging or ramp
per batch).  The per-launch figure is the same batches through nbg_maglev_classify_device_ex (no
grouping), one stream, HIP events per launch.  Prints one JSON line.
--timeline (a -DNBG_SPROBE build through NBG_LIB_OVERRIDE): per-wave tile arrivals of unit steps
probe..probe+15 (two batch boundaries at 8 steps per block per 1M batch), showing whether a
batch boundary costs a ramp."""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=256)
    ap.add_argument("--timeline", action="store_true")
    ap.add_argument("--variants", default="read_only,in_place")
    args = ap.parse_args()
    import torch

    import netbricks_amd as nb
    from bench import KernelTimer
    from netbricks_amd._lib import lib

    n, K = 1 << 20, args.batches
    dev = torch.device("cuda:0")
    mg = nb.Maglev([f"backend-{i}" for i in range(65)], 65537)
    bufs = [torch.from_numpy(nb.make_trace(n, 0, seed=900 + b)[0]).to(dev) for b in range(8)]
    outs = [torch.empty(n, dtype=torch.uint16, device=dev) for _ in range(8)]
    st = torch.cuda.Stream(dev)
    res = {"n_pkts": n, "batches": K}
    for variant, swap in (("read_only", False), ("in_place", True)):
        if variant not in args.variants.split(","):
            continue
        # one launch per batch (the same kernel family), events per launch
        flags = 0x1 if swap else 0
        kt = KernelTimer(K)
        for rnd in range(2):
            for i in range(K):
                if rnd:
                    kt.start(i, st.cuda_stream)
                rc = lib.nbg_maglev_classify_device_ex(mg._h, bufs[i % 8].data_ptr(), None, None, 64, 60, n, flags,
                                                       outs[i % 8].data_ptr(), None, None, None, st.cuda_stream)
                assert rc == 0, nb._lib.last_error()
                if rnd:
                    kt.stop(i, st.cuda_stream)
            torch.cuda.synchronize()
        launch_us = float(kt.ms()[1:].mean()) * 1e3
        kt.close()
        # the ring
        ring = mg.ring(swap_macs=swap, stream=st)
        for i in range(16):  # warm: the kernel is resident and polling
            ring.post(bufs[i % 8], n, outs[i % 8])
        ring.wait(15)
        # the feed loop on bare ctypes with prebuilt arguments (Ring.post's checks cost ~5 us a call,
        # about half a batch): the producer must stay ahead of the kernel
        post, poll, rr = lib.nbg_ring_post, lib.nbg_ring_poll, ring._r
        pk = [C.c_void_p(bufs[i].data_ptr()) for i in range(8)]
        ob = [C.c_void_p(outs[i].data_ptr()) for i in range(8)]
        tk, cc = C.c_uint64(), C.c_uint64()
        base = 16
        stamps = []
        posted, done = 0, 0
        slots = nb._lib.NBG_RING_SLOTS
        t0 = time.perf_counter()
        while done < K:
            while posted < K and posted - done < slots:
                assert post(rr, pk[posted % 8], n, ob[posted % 8], C.byref(tk)) == 0
                posted += 1
            assert poll(rr, C.byref(cc)) == 0
            c = cc.value - base
            if c != done:
                stamps.append((time.perf_counter(), c))
                done = c
        t1 = time.perf_counter()
        ring.stop()
        ts = np.array([s[0] for s in stamps])
        cs = np.array([s[1] for s in stamps])
        lo, hi = K // 8, K - K // 8
        i0, i1 = np.searchsorted(cs, lo), np.searchsorted(cs, hi)
        slope = (ts[i1] - ts[i0]) / (cs[i1] - cs[i0]) * 1e6
        res[variant] = {"launch_us": round(launch_us, 2), "ring_us_per_batch": round(float(slope), 2),
                        "ring_wall_us_per_batch": round((t1 - t0) / K * 1e6, 2),
                        "ring_gpps": round(n / slope / 1e3, 1), "launch_gpps": round(n / launch_us / 1e3, 1)}
        print(json.dumps({variant: res[variant]}), flush=True)
    if args.timeline:
        fn = lib.nbg_debug_sprobe
        fn.restype = C.c_int
        fn.argtypes = [C.c_void_p, C.c_uint64]
        probe = int(os.environ.get("NBG_RING_PROBE_STEP", "24"))
        ring = mg.ring(stream=st)
        tk = C.c_uint64()
        for i in range(probe // 8 + 8):  # enough 1M batches to cover the probed steps, posted ahead
            assert lib.nbg_ring_post(ring._r, bufs[i % 8].data_ptr(), n, outs[i % 8].data_ptr(), C.byref(tk)) == 0
        ring.wait(probe // 8 + 7)
        ring.stop()
        raw = np.zeros(4096 * 20, dtype=np.uint64)
        assert fn(raw.ctypes.data, raw.size) == 0
        t = raw.reshape(4096, 20)[:256 * 8].astype(np.float64)
        us = (t[:, 2:18] - t[:, 2:18].min()) / 100.0
        iv = np.diff(us, axis=1)  # per wave: step k -> k+1
        dbg = np.zeros(1024 * 20, dtype=np.uint32)
        fd = lib.nbg_debug_ringdbg
        fd.restype = C.c_int
        fd.argtypes = [C.c_void_p, C.c_uint64]
        assert fd(dbg.ctypes.data, dbg.size) == 0
        d = dbg.reshape(1024, 20)[:256]
        res["ring_debug"] = {"prefetches": int(d[:, 0].sum()), "taken": int(d[:, 1].sum()),
                             "empty_prefetches": int(d[:, 2].sum()), "idle_entries": int(d[:, 3].sum()),
                             "block0_failed_stage": [hex(int(x)) for x in dbg[4:20]]}
        print(json.dumps({"ring_debug": res["ring_debug"]}), flush=True)
        res["timeline"] = {"probe_step": probe,
                           "median_step_interval_us": [round(float(x), 3) for x in np.median(iv, axis=0)],
                           "p90_step_interval_us": [round(float(x), 3) for x in np.percentile(iv, 90, axis=0)]}
        print(json.dumps({"timeline": res["timeline"]}), flush=True)
    mg.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
