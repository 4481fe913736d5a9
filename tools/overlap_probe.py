"""How much of the multi-stream C2 per-batch time is the classify kernel itself: per-batch time of
each variant with and without the grouping launch, on 1, 2 and 3 streams (bench.py's setup: 8
resident 1M-packet batches, one handle per stream).

    python tools/overlap_probe.py --steps 300
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--passes", type=int, default=2)
    ap.add_argument("--only", default=None, help="variant,group(0/1),streams: one configuration")
    args = ap.parse_args()
    import torch

    import netbricks_amd as nb

    dev = torch.device("cuda:0")
    names = [f"backend-{i}" for i in range(65)]
    lut = nb.build_lut(names, 65537)
    n = 1 << 20
    bufs = [torch.from_numpy(nb.make_trace(n, 0, seed=b)[0]).to(dev) for b in range(8)]
    S = 3
    mgs = [nb.Maglev(lut=lut, n_backends=65, device=0) for _ in range(S)]
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    outs = [dict(backend=torch.empty(n, dtype=torch.uint16, device=dev),
                 perm=torch.empty(n, dtype=torch.uint32, device=dev),
                 counts=torch.empty(66, dtype=torch.uint32, device=dev)) for _ in range(S)]
    recs = [torch.empty(n * 12, dtype=torch.uint8, device=dev) for _ in range(S)]

    def kw(variant, j, group):
        o = dict(outs[j]) if group else dict(backend=outs[j]["backend"])
        if variant == "records":
            o.update(swap_macs=True, mac_out=recs[j])
        else:
            o.update(swap_macs=variant == "in_place")
        return o

    def run(variant, group, ns):
        def step(i):
            j = i % ns
            mgs[j].group_by(bufs[i % 8], n, stride=64, frame_len=60, group=group, stream=streams[j].cuda_stream,
                            **kw(variant, j, group))
        for i in range(args.warmup):
            step(i)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for i in range(args.steps):
            step(i)
        torch.cuda.synchronize()
        for m in mgs:
            m.check()
        return (time.perf_counter() - t) / args.steps * 1e6

    rows = []
    if args.only:
        v, g, ns = args.only.split(",")
        us = run(v, g == "1", int(ns))
        print(json.dumps(dict(variant=v, group=g == "1", streams=int(ns), us_per_batch=round(us, 2))), flush=True)
        return
    for p in range(args.passes):
        for variant in ("read_only", "records", "in_place"):
            for group in (True, False):
                for ns in (1, 2, 3):
                    us = run(variant, group, ns)
                    r = dict(variant=variant, group=group, streams=ns, us_per_batch=round(us, 2),
                             gpps=round(n / us / 1e3, 1), pass_=p)
                    rows.append(r)
                    print(json.dumps(r), flush=True)
    for m in mgs:
        m.close()


if __name__ == "__main__":
    main()
