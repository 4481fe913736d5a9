#!/usr/bin/env python3
"""Multi-batch classify launch (4 x 1M C2 batches) timed alone with HIP events: read-only with the
partition histograms (grouping deferred, as the bench's kernel pass) and without them (no
grouping: no per-unit barrier, no flush), to price the histogram work inside the launch."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import netbricks_amd as nb

    dev = torch.device("cuda:0")
    mg = nb.Maglev([f"backend-{i}" for i in range(65)], 65537)
    n, K = 1 << 20, 4
    bufs = [torch.from_numpy(nb.make_trace(n, 0, seed=b + 3)[0]).to(dev) for b in range(8)]
    from netbricks_amd._lib import NbgBatch, lib

    outs = [(torch.empty(n, dtype=torch.uint16, device=dev), torch.empty(n, dtype=torch.uint32, device=dev),
             torch.empty(66, dtype=torch.uint32, device=dev)) for _ in range(8)]

    def arr(g0, group):
        a = (NbgBatch * K)()
        for j in range(K):
            be, pm, ct = outs[g0 + j]
            a[j] = NbgBatch(bufs[g0 + j].data_ptr(), n, be.data_ptr(), pm.data_ptr() if group else None,
                            ct.data_ptr() if group else None, None)
        return a

    arrs = {(g, grp): arr(g, grp) for g in (0, 4) for grp in (False, True)}
    st = torch.cuda.current_stream(dev).cuda_stream
    for name, swap, group in (("read-only, histograms (deferred group)", 0, True), ("read-only, no grouping", 0, False),
                              ("in place, histograms (deferred group)", 1, True), ("in place, no grouping", 1, False)):
        ts = []
        for rnd in range(120):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a = arrs[(4 * (rnd % 2), group)]
            e0.record()
            rc = lib.nbg_maglev_classify_device_multi(mg._h, a, K, 64, 60, swap | (0x10 if group else 0), st)
            e1.record()
            assert rc == 0, rc
            if group:
                mg.finish_group()
            if rnd >= 20:
                ts.append((e0, e1))
        torch.cuda.synchronize()
        v = np.median([x.elapsed_time(y) * 1e3 for x, y in ts])
        print(f"{name:42s} median {v:8.2f} us per {K} x 1M launch", flush=True)


if __name__ == "__main__":
    main()
