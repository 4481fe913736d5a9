#!/usr/bin/env python3
"""Feasibility probe: the GPU reads the header windows straight out of host mbufs and writes the MAC
swap back into them (the mbuf pool registered once with hipHostRegister, as a DPDK hugepage pool
would be), instead of a host gather into staging, H2D, D2H and a host write-back.  Per batch only
the u32 offsets and u16 lengths go H2D and backend/perm/counts come back.  Checks bit-exactness
against the oracle and times the batch rate against the pipelined host path."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch

import netbricks_amd as nb
from netbricks_amd import _lib

import orc  # checker only


def alloc_pool(nbytes, thp):
    import mmap

    m = mmap.mmap(-1, nbytes, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    if thp:
        m.madvise(mmap.MADV_HUGEPAGE)
    return m, np.frombuffer(m, dtype=np.uint8)


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--room", type=int, default=2048)
    ap.add_argument("--thp", action="store_true")
    ap.add_argument("--streams", type=int, default=1)
    args = ap.parse_args()
    n, room, batches = 1 << 20, args.room, 12
    hip = C.CDLL("libamdhip64.so.7")
    buf, _, _ = nb.make_trace(n, 0, seed=3)
    names = [f"backend-{i}" for i in range(65)]
    mg = nb.Maglev(names, 65537)
    _m, pool = alloc_pool(n * room, args.thp)
    pool.reshape(n, room)[:, :64] = buf.reshape(n, 64)
    t0 = time.perf_counter()
    rc = hip.hipHostRegister(C.c_void_p(pool.ctypes.data), C.c_size_t(pool.nbytes), C.c_uint(0x2))  # Mapped
    t_reg = time.perf_counter() - t0
    assert rc == 0, f"hipHostRegister {rc}"
    dptr = C.c_void_p()
    rc = hip.hipHostGetDevicePointer(C.byref(dptr), C.c_void_p(pool.ctypes.data), C.c_uint(0))
    assert rc == 0, f"hipHostGetDevicePointer {rc}"
    res = {"room": room, "thp": args.thp, "streams": args.streams, "register_ms": round(t_reg * 1e3, 1),
           "pool_bytes": pool.nbytes,
           "device_ptr_equals_host": dptr.value == pool.ctypes.data}
    offs = (np.arange(n, dtype=np.uint64) * room).astype(np.uint32)
    lens = np.full(n, 60, dtype=np.uint16)
    dev = torch.device("cuda:0")
    h_off = torch.from_numpy(offs.view(np.int32)).pin_memory()
    h_len = torch.from_numpy(lens.view(np.int16)).pin_memory()
    S = args.streams
    mgs = [mg] + [nb.Maglev(names, 65537) for _ in range(S - 1)]
    bufs = [dict(d_off=torch.empty(n, dtype=torch.int32, device=dev), d_len=torch.empty(n, dtype=torch.int16, device=dev),
                 be=torch.empty(n, dtype=torch.int16, device=dev), pm=torch.empty(n, dtype=torch.int32, device=dev),
                 ct=torch.empty(66, dtype=torch.int32, device=dev), h_be=torch.empty(n, dtype=torch.int16).pin_memory(),
                 h_pm=torch.empty(n, dtype=torch.int32).pin_memory(), h_ct=torch.empty(66, dtype=torch.int32).pin_memory())
            for _ in range(S)]
    sts = [torch.cuda.Stream(dev) for _ in range(S)]
    h_be, h_pm = bufs[0]["h_be"], bufs[0]["h_pm"]
    st = sts[0]
    cnt = [0]

    def batch(flags):
        j = cnt[0] % S
        cnt[0] += 1
        b, s_ = bufs[j], sts[j]
        with torch.cuda.stream(s_):
            b["d_off"].copy_(h_off, non_blocking=True)
            b["d_len"].copy_(h_len, non_blocking=True)
            rc = _lib.lib.nbg_maglev_classify_device_ex(mgs[j]._h, dptr, b["d_off"].data_ptr(), b["d_len"].data_ptr(),
                                                        0, 0, n, flags, b["be"].data_ptr(), b["pm"].data_ptr(),
                                                        b["ct"].data_ptr(), None, s_.cuda_stream)
            _lib.check(rc, "classify_device_ex")
            b["h_be"].copy_(b["be"], non_blocking=True)
            b["h_pm"].copy_(b["pm"], non_blocking=True)
            b["h_ct"].copy_(b["ct"], non_blocking=True)

    flags = _lib.NBG_SWAP_MACS | _lib.NBG_OWNED_WINDOWS | _lib.NBG_WB_PARTIAL
    # correctness: one batch against the oracle (the swap lands in the host mbufs)
    ref = pool.reshape(n, room)[:, :64].copy().reshape(-1)
    exp_be = orc.classify(ref, n, orc.lut_build(names, 65537), stride=64, fixed_len=60)
    cnt[0] = 0
    batch(flags)
    torch.cuda.synchronize()
    got = pool.reshape(n, room)[:, :64].reshape(-1)
    res["backend_ok"] = bool(np.array_equal(h_be.numpy().view(np.uint16), exp_be))
    res["mac_swap_ok"] = bool(np.array_equal(got, ref))
    exp_perm, exp_cnt = orc.group(exp_be, 65)
    res["perm_ok"] = bool(np.array_equal(h_pm.numpy().view(np.uint32), exp_perm))
    for name, f in [("swap_wb16", flags), ("swap_wb64", flags & ~_lib.NBG_WB_PARTIAL),
                    ("no_swap", _lib.NBG_OWNED_WINDOWS)]:
        for _ in range(2 * S):
            batch(f)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(batches):
            batch(f)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / batches
        res[name] = {"ms_per_batch": round(dt * 1e3, 3), "mpps": round(n / dt / 1e6, 1)}
        print(name, res[name], file=sys.stderr, flush=True)
    hip.hipHostUnregister(C.c_void_p(pool.ctypes.data))
    del pool
    print(json.dumps(res))


if __name__ == "__main__":
    main()
