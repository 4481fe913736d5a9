#!/usr/bin/env python3
"""C2 (fixed 64-B slots, 65 backends, in place) through nbg_maglev_classify_device_multi with K batches
per launch: the classify launch alone (HIP events, grouping deferred) and the whole job on 2 streams,
over `--rotate` distinct 1M batches (each stream its own K inputs per call; no buffer in two calls in
flight).  Measurement tool: is K = 8 worth a larger rotation in the headline?  Prints one JSON line."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", default="4,8")
    ap.add_argument("--calls", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--nohist", action="store_true",
                    help="also time the launch without grouping (no per-unit histogram in the classify kernel)")
    args = ap.parse_args()
    import torch

    import netbricks_amd as nb
    from bench import KernelTimer
    from netbricks_amd._lib import NBG_DEFER_GROUP, NBG_SWAP_MACS, NbgBatch, lib

    dev = torch.device("cuda:0")
    n = 1 << 20
    ks = [int(k) for k in args.k.split(",")]
    ms = 2
    bufs = []
    for b in range(max(ks) * ms):
        buf, _, _ = nb.make_trace(n, 0, seed=2000 + b)
        bufs.append(torch.from_numpy(buf).to(dev))
    lut = nb.build_lut([f"backend-{i}" for i in range(65)], 65537)
    hs = [nb.Maglev(lut=lut, n_backends=65) for _ in range(ms)]
    sts = [torch.cuda.Stream(dev) for _ in range(ms)]
    keep = []
    out = {}
    for rnd in range(args.rounds):
        for k in ks:
            arrs = []
            for j in range(ms):
                arr = (NbgBatch * k)()
                for q in range(k):
                    o = (torch.empty(n, dtype=torch.uint16, device=dev), torch.empty(n, dtype=torch.uint32, device=dev),
                         torch.empty(66, dtype=torch.uint32, device=dev))
                    keep.append(o)
                    arr[q] = NbgBatch(bufs[j * k + q].data_ptr(), n, o[0].data_ptr(), o[1].data_ptr(), o[2].data_ptr(),
                                      None)
                arrs.append(arr)

            def call(j, st, defer=False):
                rc = lib.nbg_maglev_classify_device_multi(hs[j]._h, arrs[j], k, 64, 60,
                                                          NBG_SWAP_MACS | (NBG_DEFER_GROUP if defer else 0), st)
                assert rc == 0, nb._lib.last_error()

            for i in range(6):
                call(i % ms, sts[i % ms].cuda_stream)
            torch.cuda.synchronize()
            calls = args.calls * 8 // k
            t1 = time.perf_counter()
            for i in range(calls):
                call(i % ms, sts[i % ms].cuda_stream)
            torch.cuda.synchronize()
            el = time.perf_counter() - t1
            kt = KernelTimer(calls)
            st = sts[0].cuda_stream
            for i in range(calls):
                kt.start(i, st)
                call(0, st, defer=True)
                kt.stop(i, st)
                hs[0].finish_group(st)
            torch.cuda.synchronize()
            kus = float(kt.ms().mean()) * 1e3
            kt.close()
            for h in hs:
                h.check()
            if args.nohist:
                na = (NbgBatch * k)()
                for q in range(k):
                    o = keep[-(ms * k) + q]
                    na[q] = NbgBatch(bufs[q].data_ptr(), n, o[0].data_ptr(), None, None, None)
                kt2 = KernelTimer(calls)
                for i in range(calls):
                    kt2.start(i, st)
                    assert lib.nbg_maglev_classify_device_multi(hs[0]._h, na, k, 64, 60, NBG_SWAP_MACS, st) == 0
                    kt2.stop(i, st)
                torch.cuda.synchronize()
                out[f"k{k}_r{rnd}_nohist_classify_us_per_batch"] = round(float(kt2.ms().mean()) * 1e3 / k, 2)
                kt2.close()
            out[f"k{k}_r{rnd}"] = {"path_us_per_batch": round(el / (calls * k) * 1e6, 2),
                                   "classify_us_per_batch": round(kus / k, 2), "frac": round(n * 78 / (kus / k) / 8e6, 4)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
