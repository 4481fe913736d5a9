"""Python surface of the chained test/lpm -> test/maglev path (BASELINE config C5).

`Lpm(routes)` mirrors test/lpm's IPLookup (test/lpm/src/nf.rs:12-99): insert every
(prefix, len, gate) route, construct the DIR-24-8 tables (nf.rs:49-86), upload them.
`chain_lpm_maglev(maglev, lpm, pkts, n)` runs, in one kernel pass over a device-resident
batch, test/lpm's pipeline (parse -> swap -> parse::<IpHeader> -> group_by(3, lookup(src)),
nf.rs:212-228) followed by test/maglev's (test/maglev/src/nf.rs:92-106).
"""
from __future__ import annotations

import ctypes as C
import ipaddress
from typing import Iterable, Tuple, Union

import numpy as np

from . import _lib
from ._lib import NBG_DEFER_GROUP, NBG_LUT_LDS, NBG_OWNED_WINDOWS, NBG_STREAM_DESC, check, lib
from .maglev import GroupedBatch, Maglev, _check_owned, _ptr

__all__ = ["Lpm", "build_lpm", "chain_lpm_maglev", "chain_lpm_maglev_multi", "LpmResult"]

Route = Tuple[Union[str, int], int, int]


def _routes(routes: Iterable[Route]):
    pf, ln, gt = [], [], []
    for ip, plen, gate in routes:
        pf.append(int(ipaddress.IPv4Address(ip)) if isinstance(ip, str) else int(ip))  # u32::from(Ipv4Addr)
        ln.append(int(plen))
        gt.append(int(gate))
    return (np.asarray(pf, dtype=np.uint32), np.asarray(ln, dtype=np.uint8), np.asarray(gt, dtype=np.uint16))


def build_lpm(routes: Iterable[Route]):
    """The product's host DIR-24-8 builder (what Lpm uploads): (tbl24 u16[2^24+1], tbl_long u16[used])."""
    pf, ln, gt = _routes(routes)
    tbl24 = np.empty(_lib.NBG_LPM_TBL24_SIZE, dtype=np.uint16)
    cap = _lib.NBG_LPM_TBL24_SIZE
    tbl_long = np.empty(cap, dtype=np.uint16)
    used = C.c_uint64()
    check(lib.nbg_lpm_build_host(pf.ctypes.data, ln.ctypes.data, gt.ctypes.data, pf.size, tbl24.ctypes.data,
                                 tbl_long.ctypes.data, cap, C.byref(used)), "nbg_lpm_build_host")
    return tbl24, tbl_long[:used.value].copy()


class LpmResult(GroupedBatch):
    """GroupedBatch plus the per-packet lpm gate (NBG_SENTINEL: lpm cannot parse the packet)."""

    def __init__(self, gate, backend, perm, counts):
        super().__init__(backend, perm, counts)
        self.gate = gate


class Lpm:
    """Device-resident DIR-24-8 table of test/lpm (IPLookup, test/lpm/src/nf.rs:12-99)."""

    def __init__(self, routes: Iterable[Route], device: int = 0):
        pf, ln, gt = _routes(routes)
        self._h = C.c_void_p()
        self.device = device
        check(lib.nbg_lpm_create(pf.ctypes.data, ln.ctypes.data, gt.ctypes.data, pf.size, device,
                                 C.byref(self._h)), "nbg_lpm_create")

    def close(self) -> None:
        if self._h:
            lib.nbg_lpm_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def lookup(self, ips, gate=None, stream=None):
        """lookup_entry (nf.rs:88-98) over a device u32 tensor of host-order addresses."""
        import torch

        n = ips.numel()
        if gate is None:
            gate = torch.empty(n, dtype=torch.uint16, device=ips.device)
        if stream is None:
            stream = torch.cuda.current_stream(ips.device).cuda_stream
        check(lib.nbg_lpm_lookup_device(self._h, _ptr(ips), n, _ptr(gate), stream), "nbg_lpm_lookup_device")
        return gate


def chain_lpm_maglev(mg: Maglev, lpm: Lpm, pkts, n_pkts: int, *, lpm_groups: int = 3, stride: int = 64,
                     frame_len: int = 60, offsets=None, lens=None, owned_windows: bool = False,
                     defer_group: bool = False, group: bool = True, lut_lds: bool = False,
                     stream_desc: bool = False, gate=None, bounds_check: bool = True,
                     backend=None, perm=None,
                     counts=None, stream=None) -> LpmResult:
    """lpm(...) -> maglev(...) over a device-resident batch (packet layout as Maglev.group_by)."""
    import torch

    dev = pkts.device
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    if owned_windows and bounds_check:
        _check_owned("offsets", pkts, offsets, n_pkts, stream)
    if gate is None:
        gate = torch.empty(max(n_pkts, 1), dtype=torch.uint16, device=dev)
    if backend is None:
        backend = torch.empty(max(n_pkts, 1), dtype=torch.uint16, device=dev)
    if group and perm is None:
        perm = torch.empty(max(n_pkts, 1), dtype=torch.uint32, device=dev)
    if group and counts is None:
        counts = torch.empty(mg.n_backends + 1, dtype=torch.uint32, device=dev)
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    flags = ((NBG_OWNED_WINDOWS if owned_windows else 0) | (NBG_DEFER_GROUP if defer_group else 0)
             | (NBG_LUT_LDS if lut_lds else 0) | (NBG_STREAM_DESC if stream_desc else 0))
    rc = lib.nbg_chain_lpm_maglev_device(mg._h, lpm._h, lpm_groups, _ptr(pkts), _ptr(offsets), _ptr(lens), stride,
                                         frame_len, n_pkts, flags, _ptr(gate), _ptr(backend),
                                         _ptr(perm) if group else None, _ptr(counts) if group else None, stream)
    check(rc, "nbg_chain_lpm_maglev_device")
    return LpmResult(gate, backend, perm if group else None, counts if group else None)


def chain_lpm_maglev_multi(mg: Maglev, lpm: Lpm, batches, *, lpm_groups: int = 3, owned_windows: bool = False,
                           group: bool = True, defer_group: bool = False, bounds_check: bool = True,
                           stream=None) -> list:
    """lpm(...) -> maglev(...) over several descriptor batches ((pkts, offsets, lens, n_pkts) each) in
    one launch of each kernel (nbg_chain_lpm_maglev_multi).  Returns one LpmResult per batch, as
    chain_lpm_maglev would give it for that batch alone."""
    import torch

    if stream is None:
        stream = torch.cuda.current_stream(torch.device("cuda", mg.device)).cuda_stream
    arr, out = mg._desc_batches(batches, group, True, True, owned_windows and bounds_check, stream)
    flags = (NBG_OWNED_WINDOWS if owned_windows else 0) | (NBG_DEFER_GROUP if defer_group else 0)
    check(lib.nbg_chain_lpm_maglev_multi(mg._h, lpm._h, lpm_groups, arr, len(batches), flags, stream),
          "nbg_chain_lpm_maglev_multi")
    mg._multi_keep = arr
    return [LpmResult(g, b, p, c) for b, p, c, g in out]
