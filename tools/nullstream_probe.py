#!/usr/bin/env python3
"""Which calls wait for the legacy null stream?  With the null stream gated on a ~1 s kernel chain
of another stream, time each step and report whether the gate was still closed after it."""
import ctypes as C
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import netbricks_amd as nb  # noqa: E402
from netbricks_amd.lpm import Lpm  # noqa: E402

hip = C.CDLL("libamdhip64.so.7")
torch.cuda.set_device(0)
x = torch.randn(4096, 4096, device="cuda:0")
torch.cuda.synchronize()
g = torch.cuda.Stream()
with torch.cuda.stream(g):
    for _ in range(1500):
        x = x @ x
        x = x / x.norm()
    gate = torch.cuda.Event()
    gate.record(g)
torch.cuda.current_stream().wait_event(gate)
t0 = time.perf_counter()
res = []


def step(name, fn):
    t = time.perf_counter()
    out = fn()
    res.append({"step": name, "ms": round((time.perf_counter() - t) * 1e3, 2), "gate_closed": not gate.query()})
    return out


p = C.c_void_p()
step("hipMalloc 1MB", lambda: hip.hipMalloc(C.byref(p), C.c_size_t(1 << 20)))
hp = C.c_void_p()
step("hipHostMalloc 1MB", lambda: hip.hipHostMalloc(C.byref(hp), C.c_size_t(1 << 20), C.c_uint(0)))
st = C.c_void_p()
step("hipStreamCreateWithFlags nb", lambda: hip.hipStreamCreateWithFlags(C.byref(st), C.c_uint(1)))
step("hipMemsetAsync on nb stream + sync", lambda: (hip.hipMemsetAsync(p, 0, C.c_size_t(1 << 20), st), hip.hipStreamSynchronize(st)))
ev = C.c_void_p()
step("hipEventCreateWithFlags", lambda: hip.hipEventCreateWithFlags(C.byref(ev), C.c_uint(2)))
mg = step("Maglev create", lambda: nb.Maglev([f"backend-{i}" for i in range(65)], 65537))
lpm = step("Lpm create", lambda: Lpm([("10.0.0.0", 8, 1)]))
s = torch.cuda.Stream()
n = 100000
buf, _, _ = nb.make_trace(n, 0, seed=77)
pin = torch.from_numpy(buf.copy()).pin_memory()
d = torch.empty(n * 64, dtype=torch.uint8, device="cuda:0")
step("pinned H2D on stream s + sync", lambda: (d.copy_(pin, non_blocking=True) if False else None))
with torch.cuda.stream(s):
    step("torch copy_ pinned non_blocking on s", lambda: d.copy_(pin, non_blocking=True))
step("s.synchronize", lambda: s.synchronize())
step("group_by on s + sync", lambda: (mg.group_by(d, n, stream=s.cuda_stream), s.synchronize()))
frames = [bytearray(buf[i * 64:i * 64 + 60].tobytes()) for i in range(2000)]
step("group_by_host (first: slot alloc)", lambda: mg.group_by_host(frames))
step("group_by_host (again)", lambda: mg.group_by_host(frames))
step("hipFree", lambda: hip.hipFree(p))
step("Maglev close", lambda: mg.close())
torch.cuda.synchronize()
print(json.dumps({"total_ms": round((time.perf_counter() - t0) * 1e3, 1), "steps": res}, indent=1))
