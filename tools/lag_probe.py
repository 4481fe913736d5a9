#!/usr/bin/env python3
"""Diagnostic (round 3): what a lagged-grouping launch (NBG_GROUP_LAG) costs against the classify
launch alone, one stream, HIP events around each launch, 1M-packet C2 batches rotating over 8.
Run once per library build (NBG_LIB_OVERRIDE, e.g. the NBG_LAG_ABL ablations) and compare.
Prints one JSON line: mean launch us per variant, and the 3-stream whole-job rate of each."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import netbricks_amd as nb
    from bench import KernelTimer
    from netbricks_amd._lib import lib

    n, nb_ = 1 << 20, 65
    launches = int(os.environ.get("LAG_PROBE_LAUNCHES", "64"))
    dev = torch.device("cuda:0")
    lut = nb.build_lut([f"backend-{i}" for i in range(nb_)], 65537)
    bufs = [torch.from_numpy(nb.make_trace(n, 0, seed=300 + b)[0]).to(dev) for b in range(8)]
    S = 3
    mgs = [nb.Maglev(lut=lut, n_backends=nb_) for _ in range(S)]
    sts = [torch.cuda.Stream(dev) for _ in range(S)]
    outs = [[(torch.empty(n, dtype=torch.uint16, device=dev), torch.empty(n, dtype=torch.uint32, device=dev),
              torch.empty(nb_ + 1, dtype=torch.uint32, device=dev)) for _ in range(2)] for _ in range(S)]

    def call(j, i, flags, stream=None, par=None):
        be, pm, ct = outs[j][(i if par is None else par) & 1]
        rc = lib.nbg_maglev_classify_device_ex(mgs[j]._h, bufs[i % 8].data_ptr(), None, None, 64, 60, n, flags,
                                               be.data_ptr(), pm.data_ptr(), ct.data_ptr(), None,
                                               sts[j].cuda_stream if stream is None else stream)
        assert rc == 0, nb._lib.last_error()

    res = {"lib": os.path.basename(os.environ.get("NBG_LIB_OVERRIDE", "libnbgpu.so"))}
    st = sts[0].cuda_stream
    for name, flags in (("in_place_sep", 0x1 | 0x10), ("in_place_lag", 0x1 | 0x80), ("read_only_sep", 0x10),
                        ("read_only_lag", 0x80)):
        kt = KernelTimer(launches)
        for rnd in range(2):  # round 0 warms up
            for i in range(launches):
                if rnd:
                    kt.start(i, st)
                call(0, i, flags, st)
                if rnd:
                    kt.stop(i, st)
                if flags & 0x10:
                    lib.nbg_maglev_finish_group(mgs[0]._h, st)
            lib.nbg_maglev_finish_group(mgs[0]._h, st)
            torch.cuda.synchronize()
        ms = kt.ms()[1:]
        kt.close()
        res[name] = round(float(ms.mean()) * 1e3, 2)
    for name, flags in (("in_place_sep_3s", 0x1), ("in_place_lag_3s", 0x1 | 0x80), ("read_only_sep_3s", 0x0),
                        ("read_only_lag_3s", 0x80)):
        for rnd in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(launches * 3):
                call(i % S, i, flags, par=i // S)
            for m in mgs:
                lib.nbg_maglev_finish_group(m._h, sts[0].cuda_stream)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
        res[name] = round(el / (launches * 3) * 1e6, 2)
    for m in mgs:
        m.check()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
