#!/usr/bin/env python3
"""Classify-kernel time of configs C5 (lpm -> maglev, IMIX) and C3 (1000 backends / 655373, IMIX, in
place) on one stream (HIP events around each launch, grouping deferred past the stop event), for
A/B builds loaded with NBG_LIB_OVERRIDE (tools/build_ab.sh).  Prints one JSON line."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=60)
    ap.add_argument("--which", default="c5,c3")
    ap.add_argument("--stream-desc", action="store_true")
    ap.add_argument("--tpw", default="1", help="comma-separated NBG_TPW values (tiles per wave), one handle each")
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--lut-lds", action="store_true", help="stage the LUT in LDS (NBG_LUT_LDS)")
    ap.add_argument("--wb-partial", default="0", help="C3: comma-separated 0/1: NBG_WB_PARTIAL (rewrite only the "
                                                    "16 B holding the MACs of each owned window)")
    ap.add_argument("--n", default=str(1 << 20), help="comma-separated batch sizes (packets); times are also per 1M")
    ap.add_argument("--max-plen", type=int, default=32,
                    help="C5: drop routes longer than this (24: no tbl_long lookups; measures their cost)")
    ap.add_argument("--multi", default="", help="comma-separated batches per launch (descriptor multi path, 1M "
                                               "IMIX batches); also times the grouping launches")
    args = ap.parse_args()
    import torch

    import netbricks_amd as nb
    from bench import KernelTimer

    dev = torch.device("cuda:0")
    sizes = [int(x) for x in args.n.split(",")]
    n = max(sizes)
    bufs, offs, lens = [], [], []
    for b in range(2):
        buf, off, ln = nb.make_trace(n, 1, seed=1000 + b)
        bufs.append(torch.from_numpy(buf).to(dev))
        offs.append(torch.from_numpy(off.view(np.int32)).to(dev).view(torch.uint32))
        lens.append(torch.from_numpy(ln.view(np.int16)).to(dev).view(torch.uint16))
    routes = json.load(open(os.path.join(ROOT, "tests", "golden", "lpm_routes.json")))
    for k in ("reference", "mixed"):
        routes[k] = [r for r in routes[k] if int(r[1]) <= args.max_plen]
    out = {"lib": os.environ.get("NBG_LIB_OVERRIDE", "in-tree")}
    if args.multi:
        multi(args, torch, nb, KernelTimer, routes, out)
        print(json.dumps(out), flush=True)
        return
    st = torch.cuda.Stream(dev)
    backend = torch.empty(n, dtype=torch.uint16, device=dev)
    perm = torch.empty(n, dtype=torch.uint32, device=dev)
    gate = torch.empty(n, dtype=torch.uint16, device=dev)
    for which, tpw, rnd, n in [(w, t, r, z) for r in range(args.rounds) for w in args.which.split(",")
                               for t in args.tpw.split(",") for z in sizes]:
        os.environ["NBG_TPW"] = tpw
        if which == "c5":
            mg = nb.Maglev([f"backend-{i}" for i in range(65)], 65537)
            lpm = nb.Lpm(routes["reference"] + routes["mixed"])
            counts = torch.empty(66, dtype=torch.uint32, device=dev)

            def call(i):
                nb.chain_lpm_maglev(mg, lpm, bufs[i % 2], n, offsets=offs[i % 2], lens=lens[i % 2], owned_windows=True, bounds_check=False,
                                    defer_group=True, gate=gate, stream=st.cuda_stream, backend=backend, perm=perm,
                                    counts=counts, stream_desc=args.stream_desc, lut_lds=args.lut_lds)
        else:
            mg = nb.Maglev([f"be{i}" for i in range(1000)], 655373)
            counts = torch.empty(1001, dtype=torch.uint32, device=dev)

            def call(i):
                mg.group_by(bufs[i % 2], n, offsets=offs[i % 2], lens=lens[i % 2], owned_windows=True, bounds_check=False, defer_group=True,
                            stream=st.cuda_stream, backend=backend, perm=perm, counts=counts,
                            stream_desc=args.stream_desc, lut_lds=args.lut_lds)
        for i in range(6):
            call(i)
            mg.finish_group(st.cuda_stream)
        torch.cuda.synchronize()
        kt = KernelTimer(args.iters)
        for i in range(args.iters):
            kt.start(i, st.cuda_stream)
            call(i)
            kt.stop(i, st.cuda_stream)
            mg.finish_group(st.cuda_stream)
        torch.cuda.synchronize()
        ms = kt.ms()
        kt.close()
        key = f"{which}_tpw{tpw}_r{rnd}" + (f"_n{n}" if len(sizes) > 1 else "")
        out[key] = {"classify_us_mean": round(float(ms.mean()) * 1e3, 2),
                    "classify_us_median": round(float(np.median(ms)) * 1e3, 2),
                    "us_per_1m": round(float(ms.mean()) * 1e3 * (1 << 20) / n, 2)}
        mg.close()
        if which == "c5":
            lpm.close()
    print(json.dumps(out), flush=True)


def multi(args, torch, nb, KernelTimer, routes, out):
    """nbg_maglev_classify_desc_multi / nbg_chain_lpm_maglev_multi over K distinct 1M IMIX batches:
    the classify launch and the deferred grouping launches (finish_group) timed separately, one stream."""
    dev = torch.device("cuda:0")
    n = 1 << 20
    ks = [int(k) for k in args.multi.split(",")]
    dbs = []
    for b in range(max(ks)):
        buf, off, ln = nb.make_trace(n, 1, seed=1000 + b)
        dbs.append((torch.from_numpy(buf).to(dev), torch.from_numpy(off.view(np.int32)).to(dev).view(torch.uint32),
                    torch.from_numpy(ln.view(np.int16)).to(dev).view(torch.uint16), n))
    st = torch.cuda.Stream(dev)
    for rnd in range(args.rounds):
        for which in args.which.split(","):
            for k, wbp in [(k, int(w)) for k in ks for w in args.wb_partial.split(",")]:
                if which == "c5":
                    mg = nb.Maglev([f"backend-{i}" for i in range(65)], 65537)
                    lpm = nb.Lpm(routes["reference"] + routes["mixed"])

                    def call():
                        nb.chain_lpm_maglev_multi(mg, lpm, dbs[:k], owned_windows=True, bounds_check=False,
                                                  defer_group=True, stream=st.cuda_stream)
                else:
                    mg = nb.Maglev([f"be{i}" for i in range(1000)], 655373)

                    def call():
                        mg.group_by_desc_multi(dbs[:k], owned_windows=True, bounds_check=False, wb_partial=bool(wbp),
                                               defer_group=True, stream=st.cuda_stream)
                for _ in range(4):
                    call()
                    mg.finish_group(st.cuda_stream)
                torch.cuda.synchronize()
                kt, gt = KernelTimer(args.iters), KernelTimer(args.iters)
                for i in range(args.iters):
                    kt.start(i, st.cuda_stream)
                    call()
                    kt.stop(i, st.cuda_stream)
                    gt.start(i, st.cuda_stream)
                    mg.finish_group(st.cuda_stream)
                    gt.stop(i, st.cuda_stream)
                torch.cuda.synchronize()
                mg.check()
                c, g = float(kt.ms().mean()) * 1e3, float(gt.ms().mean()) * 1e3
                kt.close()
                gt.close()
                out[f"{which}_multi{k}_r{rnd}" + (f"_wbp{wbp}" if which == "c3" else "")] = {"classify_us": round(c, 2), "classify_us_per_batch": round(c / k, 2),
                                                   "group_us": round(g, 2), "group_us_per_batch": round(g / k, 2)}
                mg.close()
                if which == "c5":
                    lpm.close()


if __name__ == "__main__":
    main()
