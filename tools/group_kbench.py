#!/usr/bin/env python3
"""The grouping launches alone (hipEvent medians): classify with NBG_DEFER_GROUP, then time the
handle's finish_group on the same stream.

  [NBG_LIB_OVERRIDE=tools/ab/lib_X.so] python tools/group_kbench.py [--iters 40] [--label X]

C2: 65 backends, 1M fixed 64-B slots (group_kernel, rows from the classify kernel).
C3: 1000 backends / 655373, 1M IMIX descriptors (hist_kernel + scan_kernel + group_kernel), one batch
and 8 batches per launch (nbg_maglev_classify_desc_multi).  Eight rotating input batches."""
import argparse
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--label", default=os.path.basename(os.environ.get("NBG_LIB_OVERRIDE", "") or "tree"))
    args = ap.parse_args()
    import torch

    import netbricks_amd as nb

    dev = torch.device("cuda:0")
    n = 1 << 20
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def timed(classify, finish):
        ts = []
        for i in range(args.iters + 5):
            classify(i)
            ev[0].record()
            finish()
            ev[1].record()
            torch.cuda.synchronize()
            if i >= 5:
                ts.append(ev[0].elapsed_time(ev[1]) * 1e3)
        return statistics.median(ts)

    out = {}
    mg = nb.Maglev([f"backend-{i}" for i in range(65)], 65537)
    mg.reserve(n)
    bufs = [torch.from_numpy(nb.make_trace(n, 0, seed=11 + b)[0]).to(dev) for b in range(8)]
    be = torch.empty(n, dtype=torch.uint16, device=dev)
    perm = torch.empty(n, dtype=torch.uint32, device=dev)
    cnt = torch.empty(66, dtype=torch.uint32, device=dev)
    out["c2_group"] = timed(lambda i: mg.group_by(bufs[i % 8], n, swap_macs=False, defer_group=True, backend=be,
                                                  perm=perm, counts=cnt), mg.finish_group)
    mg.close()

    mg = nb.Maglev([f"backend-{i}" for i in range(1000)], 655373)
    mg.reserve(n)
    dbs = []
    for b in range(8):
        buf, off, ln = nb.make_trace(n, 1, seed=31 + b)
        dbs.append((torch.from_numpy(buf).to(dev), torch.from_numpy(off.view(np.int32)).to(dev).view(torch.uint32),
                    torch.from_numpy(ln.view(np.int16)).to(dev).view(torch.uint16), n))
    be = torch.empty(n, dtype=torch.uint16, device=dev)
    cnt = torch.empty(1001, dtype=torch.uint32, device=dev)

    def c3_one(i):
        p, o, l, _ = dbs[i % 8]
        mg.group_by(p, n, offsets=o, lens=l, owned_windows=True, bounds_check=False, swap_macs=False,
                    defer_group=True, backend=be, perm=perm, counts=cnt)

    out["c3_group_hist_scan"] = timed(c3_one, mg.finish_group)
    out["c3_multi8_group_per_batch"] = timed(lambda i: mg.group_by_desc_multi(dbs, swap_macs=False, defer_group=True),
                                             mg.finish_group) / 8
    mg.close()
    print(args.label, " ".join(f"{k} {v:.2f}" for k, v in out.items()))


if __name__ == "__main__":
    main()
