#!/usr/bin/env python3
"""Follow-up to nullstream_probe.py: after a handle was created, used and destroyed (hipFree), do
hipMalloc / hipStreamCreate / Maglev create wait for a gated null stream?"""
import ctypes as C
import json
import sys
import time

import torch

sys.path.insert(0, ".")
import netbricks_amd as nb  # noqa: E402

hip = C.CDLL("libamdhip64.so.7")
torch.cuda.set_device(0)
names = [f"backend-{i}" for i in range(65)]
buf, _, _ = nb.make_trace(100000, 0, seed=1)
d = torch.from_numpy(buf).cuda()
m0 = nb.Maglev(names, 65537)
m0.group_by(d, 100000)
torch.cuda.synchronize()
m0.close()
out = {}
for rnd in range(2):
    x = torch.randn(4096, 4096, device="cuda:0")
    torch.cuda.synchronize()
    g = torch.cuda.Stream()
    with torch.cuda.stream(g):
        for _ in range(3000):
            x = x @ x
            x = x / x.norm()
        gate = torch.cuda.Event()
        gate.record(g)
    torch.cuda.current_stream().wait_event(gate)
    t0 = time.perf_counter()
    res = []

    def step(name, fn):
        r = fn()
        res.append((name, round((time.perf_counter() - t0) * 1e3, 2), not gate.query()))
        return r

    p = C.c_void_p()
    step("hipMalloc 64KB", lambda: hip.hipMalloc(C.byref(p), C.c_size_t(65552)))
    step("hipMalloc 135KB", lambda: hip.hipMalloc(C.byref(p), C.c_size_t(135168)))
    st = C.c_void_p()
    step("hipStreamCreateWithFlags", lambda: hip.hipStreamCreateWithFlags(C.byref(st), C.c_uint(1)))
    step("hipStreamDestroy", lambda: hip.hipStreamDestroy(st))
    step("hipGetDeviceCount", lambda: hip.hipGetDeviceCount(C.byref(C.c_int())))
    m = step("Maglev create", lambda: nb.Maglev(names, 65537))
    torch.cuda.synchronize()
    out[f"round{rnd}"] = res
    m.close()
print(json.dumps(out, indent=1))
