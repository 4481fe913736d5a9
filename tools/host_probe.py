#!/usr/bin/env python3
"""Where the pipelined host path's time goes: nbg_maglev_host_submit/_wait over 1M mbufs with parts
of the work switched off (MAC write-back, perm, counts), and with the mbufs at a 2-KiB stride
against a dense 64-B stride (memory-access cost of the gather and write-back)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401  (the HIP runtime first, as the package does)

import netbricks_amd as nb


def run(mg, ptrs, lens, n, batches, swap, perm, counts):
    outs = [(np.empty(n, np.uint16), np.empty(n, np.uint32) if perm else None,
             np.empty(66, np.uint32) if counts else None) for _ in range(2)]
    prev = None
    for it in range(batches + 2):
        if it == 2:
            t0 = time.perf_counter()
        be, pm, ct = outs[it % 2]
        tk = mg.host_submit(ptrs, lens, be, pm, ct, swap_macs=swap)
        if prev is not None:
            mg.host_wait(prev)
        prev = tk
    mg.host_wait(prev)
    dt = (time.perf_counter() - t0) / batches
    return round(dt * 1e3, 3), round(n / dt / 1e6, 1)


def main():
    n, batches = 1 << 20, 10
    buf, _, _ = nb.make_trace(n, 0, seed=3)
    mg = nb.Maglev([f"backend-{i}" for i in range(65)], 65537)
    lens = np.full(n, 60, dtype=np.uint16)
    res = {}
    for room in (2048, 64):
        pool = np.zeros(n * room, dtype=np.uint8)
        pool.reshape(n, room)[:, :64] = buf.reshape(n, 64)
        ptrs = (np.arange(n, dtype=np.uint64) * room + np.uint64(pool.ctypes.data)).astype(np.uint64)
        for name, kw in [("full", (True, True, True)), ("no_perm", (True, False, True)),
                         ("no_swap", (False, True, True)), ("backend_only", (False, False, False))]:
            ms, mpps = run(mg, ptrs, lens, n, batches, *kw)
            res[f"room{room}_{name}"] = {"ms_per_batch": ms, "mpps": mpps}
            print(f"room {room} {name}: {ms} ms, {mpps} Mpps", file=sys.stderr, flush=True)
        del pool
    res["cpus"] = os.cpu_count()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
