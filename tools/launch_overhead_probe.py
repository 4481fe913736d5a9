#!/usr/bin/env python3
"""Host cost of issuing one C2 batch from Python (Maglev.group_by: argument checks + one C-ABI call
that launches classify + group) against the GPU time per batch, with the bench's 3 streams: if the
issue loop were slower than the GPU, the bench value would measure the host, not the kernels."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import netbricks_amd as nb
from netbricks_amd import _lib


def main():
    n, S, steps = 1 << 20, 3, 400
    dev = torch.device("cuda:0")
    names = [f"backend-{i}" for i in range(65)]
    bufs = [torch.from_numpy(nb.make_trace(n, 0, seed=b)[0]).to(dev) for b in range(8)]
    mgs = [nb.Maglev(names, 65537) for _ in range(S)]
    sts = [torch.cuda.Stream(dev) for _ in range(S)]
    outs = [dict(backend=torch.empty(n, dtype=torch.uint16, device=dev), perm=torch.empty(n, dtype=torch.uint32, device=dev),
                 counts=torch.empty(66, dtype=torch.uint32, device=dev)) for _ in range(S)]
    res = {}

    def wrapper(i):
        j = i % S
        mgs[j].group_by(bufs[i % 8], n, stream=sts[j].cuda_stream, **outs[j])

    ptrs = [(b.data_ptr(), ) for b in bufs]
    raw_args = [(mgs[j]._h, outs[j]["backend"].data_ptr(), outs[j]["perm"].data_ptr(), outs[j]["counts"].data_ptr(),
                 sts[j].cuda_stream) for j in range(S)]

    def raw(i):
        h, be, pm, ct, st = raw_args[i % S]
        _lib.lib.nbg_maglev_classify_device_ex(h, ptrs[i % 8][0], None, None, 64, 60, n, _lib.NBG_SWAP_MACS, be, pm, ct,
                                               None, st)

    for name, fn in [("wrapper", wrapper), ("raw_ctypes", raw)]:
        for i in range(30):
            fn(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            fn(i)
        t_issue = time.perf_counter() - t0
        torch.cuda.synchronize()
        t_all = time.perf_counter() - t0
        res[name] = {"issue_us_per_step": round(t_issue / steps * 1e6, 2), "total_us_per_step": round(t_all / steps * 1e6, 2)}
        print(name, res[name], file=sys.stderr, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
