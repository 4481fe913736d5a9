#!/usr/bin/env python3
"""Diagnostics (round 3): start a ring, post one batch, and print the relay's state words from the
host control line (an NBG_RING_DEBUG build through NBG_LIB_OVERRIDE) every 20 ms for 0.3 s."""
import ctypes as C
import time

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import netbricks_amd as nb  # noqa: E402
from netbricks_amd._lib import lib  # noqa: E402

fn = lib.nbg_debug_ring_ctl
fn.restype = C.c_int
fn.argtypes = [C.c_void_p, C.c_void_p]
n = 4096
mg = nb.Maglev([f"backend-{i}" for i in range(65)], 65537)
d = torch.from_numpy(nb.make_trace(n, 0, seed=1)[0]).cuda()
out = torch.empty(n, dtype=torch.uint16, device="cuda")
torch.cuda.synchronize()
ring = mg.ring(idle_ms=400)
w = (C.c_uint32 * 16)()
for i in range(16):
    if i == 3:
        t = ring.post(d, n, out)
        print("posted", t, flush=True)
    fn(ring._r, C.byref(w))
    print(i, "stop err completed", w[0], w[1], w[2], "| known iters lag prog0 dstop behind first grid", list(w[3:11]), flush=True)
    time.sleep(0.02)
try:
    ring.stop()
except Exception as e:
    print("stop:", e)
