#!/usr/bin/env python3
"""Variant micro-benchmark (interleaved rounds in one process, hipEvent timing).

Times the classify kernel with/without grouping, LDS vs L2 LUT, the full path, and a
plain device copy of the same bytes as the achievable-bandwidth reference.
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--nb", type=int, default=65)
    ap.add_argument("--m", type=int, default=65537)
    ap.add_argument("--only", default="", help="comma-separated substrings of variant names to run")
    ap.add_argument("--no-multistream", action="store_true")
    ap.add_argument("--lut-lds", action="store_true", help="stage the LUT in LDS for every variant")
    ap.add_argument("--streams", default="2,3,4", help="stream counts of the multi-stream variants")
    args = ap.parse_args()
    import torch

    import netbricks_amd as nb

    dev = torch.device("cuda:0")
    names = [f"backend-{i}" for i in range(args.nb)]
    mg = nb.Maglev(names, args.m)
    n = args.n
    mg.reserve(n)
    bufs, offs, lens = [], [], []
    for b in range(8):
        buf, off, ln = nb.make_trace(n, args.mode, seed=b + 17)
        bufs.append(torch.from_numpy(buf).to(dev))
        offs.append(torch.from_numpy(off.view(np.int32)).to(dev).view(torch.uint32))
        lens.append(torch.from_numpy(ln.view(np.int16)).to(dev).view(torch.uint16))
    stride = 64
    backend = torch.empty(n, dtype=torch.uint16, device=dev)
    perm = torch.empty(n, dtype=torch.uint32, device=dev)
    counts = torch.empty(args.nb + 1, dtype=torch.uint32, device=dev)
    dst = torch.empty(max(int(b.numel()) for b in bufs), dtype=torch.uint8, device=dev)
    mac = torch.empty(n * 12, dtype=torch.uint8, device=dev)
    desc = args.mode != 0

    def kw(i):
        extra = dict(lut_lds=True) if args.lut_lds else {}
        if desc:
            return dict(offsets=offs[i % 8], lens=lens[i % 8], owned_windows=True, bounds_check=False, **extra)
        return dict(stride=stride, frame_len=60, **extra)

    variants = {
        "copy(read+write all bytes)": lambda i: dst[:bufs[i % 8].numel()].copy_(bufs[i % 8]),
        "classify noswap nogroup": lambda i: mg.group_by(bufs[i % 8], n, group=False, swap_macs=False,
                                                         backend=backend, **kw(i)),
        "classify inplace nogroup": lambda i: mg.group_by(bufs[i % 8], n, group=False, backend=backend, **kw(i)),
        "classify inplace-wb16 nogroup": lambda i: mg.group_by(bufs[i % 8], n, group=False, wb_partial=True,
                                                               backend=backend, **kw(i)),
        "classify mac_out nogroup": lambda i: mg.group_by(bufs[i % 8], n, group=False, backend=backend,
                                                          mac_out=mac, **kw(i)),
        "classify inplace hist (deferred)": lambda i: (mg.group_by(bufs[i % 8], n, defer_group=True,
                                                                   backend=backend, perm=perm, counts=counts,
                                                                   **kw(i)), mg.finish_group()),
        "classify inplace counts": lambda i: mg.group_by(bufs[i % 8], n, scatter=False, backend=backend,
                                                         counts=counts, **kw(i)),
        "full path inplace": lambda i: mg.group_by(bufs[i % 8], n, backend=backend, perm=perm, counts=counts,
                                                   **kw(i)),
        "full path mac_out": lambda i: mg.group_by(bufs[i % 8], n, backend=backend, perm=perm, counts=counts,
                                                   mac_out=mac, **kw(i)),
    }
    # several batches per launch (nbg_maglev_classify_device_multi): per-call time covers K batches
    from netbricks_amd._lib import NbgBatch, lib as _clib
    m_outs = [(torch.empty(n, dtype=torch.uint16, device=dev), torch.empty(n, dtype=torch.uint32, device=dev),
               torch.empty(args.nb + 1, dtype=torch.uint32, device=dev), torch.empty(n * 12, dtype=torch.uint8, device=dev))
              for _ in range(8)]
    m_arrs = {}
    for K in (2, 4):
        for rec in (False, True):
            for g0 in range(0, 8, K):
                arr = (NbgBatch * K)()
                for j in range(K):
                    be, pm, ct, mo = m_outs[g0 + j]
                    arr[j] = NbgBatch(bufs[g0 + j].data_ptr(), n, be.data_ptr(), pm.data_ptr(), ct.data_ptr(),
                                      mo.data_ptr() if rec else None)
                m_arrs[(K, rec, g0 // K)] = arr

    def multi(i, K, rec, swap):
        st = torch.cuda.current_stream(dev).cuda_stream
        rc = _clib.nbg_maglev_classify_device_multi(mg._h, m_arrs[(K, rec, i % (8 // K))], K, 64, 60,
                                                    1 if swap else 0, st)
        assert rc == 0, rc

    for K in (2, 4):
        for mode, rec, swap in (("noswap", False, False), ("inplace", False, True), ("mac_out", True, True)):
            variants[f"multi{K} {mode} (per call of {K} batches)"] = (
                lambda i, K=K, rec=rec, swap=swap: multi(i, K, rec, swap))
    # multi-stream: independent batches in flight on S streams, one handle (scratch) per stream
    extra = {}
    for S in (() if args.no_multistream else tuple(int(x) for x in args.streams.split(","))):
        mgs = [nb.Maglev(names, args.m) for _ in range(S)]
        sts = [torch.cuda.Stream(dev) for _ in range(S)]
        outs = [(torch.empty(n, dtype=torch.uint16, device=dev), torch.empty(n, dtype=torch.uint32, device=dev),
                 torch.empty(args.nb + 1, dtype=torch.uint32, device=dev),
                 torch.empty(n * 12, dtype=torch.uint8, device=dev)) for _ in range(S)]

        def ms(i, S=S, mgs=mgs, sts=sts, outs=outs, mac=True, group=True, scatter=True, swap=True):
            j = i % S
            be, pm, ct, mo = outs[j]
            mgs[j].group_by(bufs[i % 8], n, backend=be, perm=pm if scatter else None, counts=ct, group=group,
                            scatter=scatter, swap_macs=swap,
                            mac_out=mo if mac else None, stream=sts[j].cuda_stream, **kw(i))

        extra[f"full path l2 mac_out x{S} streams"] = ms
        extra[f"full path l2 inplace x{S} streams"] = (lambda i, f=ms: f(i, mac=False))
        extra[f"classify only inplace x{S} streams"] = (lambda i, f=ms: f(i, mac=False, group=False))
        extra[f"full path l2 noswap x{S} streams"] = (lambda i, f=ms: f(i, mac=False, swap=False))
        extra[f"classify only mac_out x{S} streams"] = (lambda i, f=ms: f(i, group=False))
        extra[f"counts only inplace x{S} streams"] = (lambda i, f=ms: f(i, mac=False, scatter=False))
        extra[f"_keep{S}"] = (mgs, sts, outs)
        if S % 2 == 0:
            # S handles; classify on streams 0..S/2-1, the deferred group kernel on streams S/2..S-1
            H = S // 2
            gdone = [None] * S

            def split(i, S=S, H=H, mgs=mgs, sts=sts, outs=outs, gdone=gdone, mac=False):
                j = i % S
                cs, gs = sts[j % H], sts[H + j % H]
                be, pm, ct, mo = outs[j]
                if gdone[j] is not None:
                    cs.wait_event(gdone[j])
                mgs[j].group_by(bufs[i % 8], n, backend=be, perm=pm, counts=ct, defer_group=True,
                                mac_out=mo if mac else None, stream=cs.cuda_stream, **kw(i))
                ev = torch.cuda.Event()
                ev.record(cs)
                gs.wait_event(ev)
                mgs[j].finish_group(gs.cuda_stream)
                g = torch.cuda.Event()
                g.record(gs)
                gdone[j] = g

            extra[f"split path inplace x{S} streams"] = split
            extra[f"split path mac_out x{S} streams"] = (lambda i, f=split: f(i, mac=True))
    variants.update({k: v for k, v in extra.items() if not k.startswith("_keep")})
    if args.only:
        keys = [k.strip() for k in args.only.split(",")]
        variants = {k: v for k, v in variants.items() if any(q in k for q in keys)}
    res = {k: [] for k in variants}
    all_streams = [st for k, v in extra.items() if k.startswith("_keep") for st in v[1]]
    for r in range(args.rounds):
        for name, fn in variants.items():
            for i in range(3):
                fn(i)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            cur = torch.cuda.current_stream(dev)
            for st in all_streams:
                st.wait_event(e0)
            for i in range(args.iters):
                fn(i)
            for st in all_streams:
                ev = torch.cuda.Event()
                ev.record(st)
                cur.wait_event(ev)
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) / args.iters * 1e3)
    mg.check()
    data_bytes = sum(int(b.numel()) for b in bufs) / 8
    for name, v in res.items():
        v = np.array(v)
        med = np.median(v)
        print(f"{name:32s} median {med:8.2f} us  min {v.min():8.2f}  -> {n / med / 1e3:8.1f} Gpps "
              f" read-GB/s {data_bytes / med / 1e3:8.1f}")


if __name__ == "__main__":
    main()
