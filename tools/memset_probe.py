#!/usr/bin/env python3
"""Probe: is a synchronous hipMemset (null stream) ordered before work on a hipStreamNonBlocking
stream?  The round-1 host path zeroed each fresh staging buffer with hipMemset and then copied the
header windows H2D on a non-blocking stream; kernels sporadically read zero windows.

Per trial: keep the null stream busy (a long torch kernel chain on the legacy default stream),
hipMemset a device buffer to 0, then on a non-blocking stream hipMemcpyAsync a 0xAB pattern into it
and synchronise that stream only.  If hipMemset returned before running, it runs after the busy
chain — possibly after the copy — and the pattern is lost.  Prints the host time of the hipMemset
call and whether the pattern survived (after a device-wide synchronise)."""
import ctypes as C
import json
import time

import numpy as np
import torch

hip = C.CDLL("libamdhip64.so.7")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
NB = 1  # hipStreamNonBlocking
s = C.c_void_p()
assert hip.hipStreamCreateWithFlags(C.byref(s), C.c_uint(NB)) == 0
size = 64 << 20
buf = C.c_void_p()
assert hip.hipMalloc(C.byref(buf), C.c_size_t(size)) == 0
pat = np.full(size, 0xAB, dtype=np.uint8)
hpin = C.c_void_p()
assert hip.hipHostMalloc(C.byref(hpin), C.c_size_t(size), C.c_uint(0)) == 0
C.memmove(hpin, pat.ctypes.data, size)
out = np.empty(size, dtype=np.uint8)
x = torch.randn(4096, 4096, device=dev)
res = []
for trial in range(6):
    busy = 20 * (trial + 1)
    hip.hipDeviceSynchronize()
    # the null stream: torch's default stream on this device is the legacy default stream
    assert torch.cuda.current_stream(dev).cuda_stream == 0
    for _ in range(busy):
        x = x @ x
        x = x / x.norm()
    t0 = time.perf_counter()
    rc = hip.hipMemset(buf, C.c_int(0), C.c_size_t(size))
    t_memset = time.perf_counter() - t0
    assert rc == 0
    assert hip.hipMemcpyAsync(buf, hpin, C.c_size_t(size), C.c_int(1), s) == 0  # H2D
    assert hip.hipStreamSynchronize(s) == 0
    t_copy = time.perf_counter() - t0
    hip.hipDeviceSynchronize()
    t_all = time.perf_counter() - t0
    assert hip.hipMemcpy(out.ctypes.data_as(C.c_void_p), buf, C.c_size_t(size), C.c_int(2)) == 0
    res.append({"busy_matmuls": busy, "memset_call_ms": round(t_memset * 1e3, 3),
                "copy_done_ms": round(t_copy * 1e3, 3), "device_idle_ms": round(t_all * 1e3, 3),
                "pattern_survived": bool((out == 0xAB).all()), "zero_bytes": int((out == 0).sum())})
print(json.dumps(res, indent=1))
