#!/usr/bin/env python3
"""Per-wave timeline of one streaming-classify launch (diagnostic build with -DNBG_SPROBE, loaded
through NBG_LIB_OVERRIDE): entry, LUT visible, each tile's arrival, exit (100 MHz wall clock).
Prints, relative to the earliest wave entry: block start spread (dispatch ramp), LUT-ready times,
arrival of tile k (percentiles over waves), and exits, for the read-only / in-place / records
variants at 1M packets."""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pct(x, qs=(0, 10, 50, 90, 100)):
    return " ".join(f"{np.percentile(x, q):6.2f}" for q in qs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--group", action="store_true", help="with grouping (the kernel's per-unit histogram barriers)")
    ap.add_argument("--lag", action="store_true", help="NBG_GROUP_LAG: each launch also groups the previous batch")
    args = ap.parse_args()
    import torch

    import netbricks_amd as nb
    from netbricks_amd import _lib

    fn = _lib.lib.nbg_debug_sprobe
    fn.restype = C.c_int
    fn.argtypes = [C.c_void_p, C.c_uint64]
    dev = torch.device("cuda:0")
    mg = nb.Maglev([f"backend-{i}" for i in range(65)], 65537)
    n = args.n
    bufs = [torch.from_numpy(nb.make_trace(n, 0, seed=b + 5)[0]).to(dev) for b in range(8)]
    be = [torch.empty(n, dtype=torch.uint16, device=dev) for _ in range(2)]
    pm = [torch.empty(n, dtype=torch.uint32, device=dev) for _ in range(2)]
    rec = torch.empty(n * 12, dtype=torch.uint8, device=dev)
    for variant in ("read_only", "in_place", "records"):
        kw = dict(swap_macs=variant != "read_only")
        if variant == "records":
            kw["mac_out"] = rec
        for i in range(20):
            if args.lag:
                mg.group_by(bufs[i % 8], n, group_lag=True, backend=be[i & 1], perm=pm[i & 1], **kw)
            else:
                mg.group_by(bufs[i % 8], n, group=args.group, backend=be[0], **kw)
        torch.cuda.synchronize()  # the last launch's timeline (the finish_group launch is not probed)
        if args.lag:
            mg.finish_group()
        waves = 256 * 8
        raw = np.zeros(4096 * 20, dtype=np.uint64)
        assert fn(raw.ctypes.data, raw.size) == 0
        t = raw.reshape(4096, 20)[:waves].astype(np.float64)
        t0 = t[:, 0].min()
        us = (t - t0) / 100.0  # 100 MHz -> us
        print(f"== {variant}: launch span {us[:, 11].max():.2f} us (first entry to last exit)")
        print(f"   entry        {pct(us[:, 0])}")
        if args.lag:
            print(f"   prologue done {pct(us[:, 10])}")
        print(f"   LUT visible  {pct(us[:, 1])}")
        for k in range(8):
            print(f"   tile {k} in    {pct(us[:, 2 + k])}")
        print(f"   exit         {pct(us[:, 11])}")
        # inside step 4 (per wave, relative to its tile-4 arrival): classify + next issue, rank,
        # barrier, flush, lagged-group sync work
        d = us[:, 12:17] - us[:, 6:7]
        for nm, c in zip(("classified", "ranked", "barrier", "flushed", "synced"), range(5)):
            print(f"   step4 {nm:10s} {pct(d[:, c])}")
        steady = np.diff(us[:, 2:10], axis=1)
        print(f"   tile interval (k -> k+1) median {np.median(steady):.2f} us, p90 {np.percentile(steady, 90):.2f}")
        # where the exit spread comes from: per block (max over its waves), grouped by XCD (blocks
        # are dealt round-robin to the 8 XCDs), and against the block's first-tile arrival
        blk_exit = us[:, 11].reshape(256, 8).max(axis=1)
        blk_t0 = us[:, 2].reshape(256, 8).max(axis=1)
        xcd = np.arange(256) % 8
        per_x = [blk_exit[xcd == x] for x in range(8)]
        print("   exit by XCD (median / max):", " ".join(f"{np.median(e):.2f}/{e.max():.2f}" for e in per_x))
        within = np.mean([e.max() - e.min() for e in per_x])
        print(f"   block exit spread {blk_exit.max() - blk_exit.min():.2f} us; mean within-XCD spread {within:.2f} us; "
              f"XCD median range {max(np.median(e) for e in per_x) - min(np.median(e) for e in per_x):.2f} us; "
              f"corr(first tile, exit) {np.corrcoef(blk_t0, blk_exit)[0, 1]:.2f}")
    mg.close()


if __name__ == "__main__":
    main()
