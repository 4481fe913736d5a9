#!/usr/bin/env python3
"""Per-wave timeline of one classify launch (diagnostic build with -DNBG_CPROBE, loaded through
NBG_LIB_OVERRIDE): entry, first tile transposed (its data arrived), last store retired, exit.
Prints the launch span and how the waves' phases are spread over it (ramp, load wait, classify
tail), to locate the per-launch overhead above the streaming rate."""
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
    ap.add_argument("--variant", default="noswap", choices=["noswap", "inplace", "macout", "hist", "c5"])
    ap.add_argument("--lut-lds", action="store_true")
    ap.add_argument("--n", type=int, default=1 << 20)
    args = ap.parse_args()
    import torch

    import netbricks_amd as nb
    from netbricks_amd import _lib

    fn = _lib.lib.nbg_debug_cprobe
    fn.restype = C.c_int
    fn.argtypes = [C.c_void_p, C.c_uint64]
    dev = torch.device("cuda:0")
    mg = nb.Maglev([f"backend-{i}" for i in range(65)], 65537)
    n = args.n
    mode = 1 if args.variant == "c5" else 0  # C5: IMIX descriptors through the lpm -> maglev chain
    traces = [nb.make_trace(n, mode, seed=b + 5) for b in range(8)]
    bufs = [torch.from_numpy(t[0]).to(dev) for t in traces]
    offs = [torch.from_numpy(t[1].view(np.int32)).to(dev).view(torch.uint32) for t in traces] if mode else None
    lens = [torch.from_numpy(t[2].view(np.int16)).to(dev).view(torch.uint16) for t in traces] if mode else None
    if mode:
        import json
        routes = json.load(open(os.path.join(ROOT, "tests", "golden", "lpm_routes.json")))
        lpm = nb.Lpm(routes["reference"] + routes["mixed"])
        gate = torch.empty(n, dtype=torch.uint16, device=dev)
    be = torch.empty(n, dtype=torch.uint16, device=dev)
    perm = torch.empty(n, dtype=torch.uint32, device=dev)
    cnt = torch.empty(66, dtype=torch.uint32, device=dev)
    mac = torch.empty(n * 12, dtype=torch.uint8, device=dev)

    def launch(i):
        kw = dict(backend=be, lut_lds=args.lut_lds)
        if args.variant == "noswap":
            mg.group_by(bufs[i % 8], n, group=False, swap_macs=False, **kw)
        elif args.variant == "inplace":
            mg.group_by(bufs[i % 8], n, group=False, **kw)
        elif args.variant == "c5":
            nb.chain_lpm_maglev(mg, lpm, bufs[i % 8], n, offsets=offs[i % 8], lens=lens[i % 8], owned_windows=True, bounds_check=False,
                                defer_group=True, gate=gate, perm=perm, counts=cnt, **kw)
            mg.finish_group()
        elif args.variant == "macout":
            mg.group_by(bufs[i % 8], n, group=False, mac_out=mac, **kw)
        else:
            mg.group_by(bufs[i % 8], n, defer_group=True, perm=perm, counts=cnt, **kw)
            mg.finish_group()

    for i in range(20):
        launch(i)
    torch.cuda.synchronize()
    waves = n // 64
    out = np.zeros(waves * 4, dtype=np.uint64)
    launch(21)
    torch.cuda.synchronize()
    _lib.check(fn(out.ctypes.data, out.size), "nbg_debug_cprobe")
    t = out.reshape(waves, 4).astype(np.int64)
    t = t[(t > 0).all(axis=1)]
    t0 = t[:, 0].min()
    us = (t - t0) / 100.0  # 100 MHz wall clock -> us
    span = us[:, 3].max()
    print(f"variant={args.variant} lut_lds={args.lut_lds} n={n} waves={len(t)} span={span:.2f} us")
    print("             p0     p10    p50    p90   p100")
    print("entry      ", pct(us[:, 0]))
    print("data in    ", pct(us[:, 1]))
    print("stores done", pct(us[:, 2]))
    print("exit       ", pct(us[:, 3]))
    print("load wait  ", pct(us[:, 1] - us[:, 0]))
    print("classify   ", pct(us[:, 2] - us[:, 1]))
    print("flush      ", pct(us[:, 3] - us[:, 2]))
    bins = np.arange(0, span + 0.5, 0.5)
    load = [((us[:, 0] <= b) & (us[:, 1] > b)).sum() for b in bins]
    work = [((us[:, 1] <= b) & (us[:, 3] > b)).sum() for b in bins]
    print("t(us)   waiting-for-data  after-data")
    for b, l, w in zip(bins, load, work):
        print(f"{b:5.1f}  {l:8d}  {w:8d}")


if __name__ == "__main__":
    main()
