"""TEST INFRASTRUCTURE: ctypes view of the C oracle (oracle/liborc.so).

Used only as the checker in tests/, __graft_entry__.smoke() and bench.py's cpu_baseline.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORC_PATH = os.path.join(ROOT, "oracle", "liborc.so")
SENTINEL = 0xFFFF

_P = C.c_void_p
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORC_PATH):
            raise FileNotFoundError(f"{ORC_PATH} missing: run `make -C oracle`")
        L = C.CDLL(ORC_PATH)
        L.orc_lut_build.restype = C.c_int
        L.orc_lut_build.argtypes = [C.POINTER(C.c_char_p), C.POINTER(C.c_uint32), C.c_uint32, C.c_uint64, _P]
        L.orc_classify.restype = None
        L.orc_classify.argtypes = [_P, _P, C.c_uint64, _P, C.c_uint32, C.c_uint64, _P, C.c_uint64, C.c_int, _P]
        L.orc_group.restype = None
        L.orc_group.argtypes = [_P, C.c_uint64, C.c_uint32, _P, _P]
        L.orc_flow_hash.restype = C.c_uint64
        L.orc_flow_hash.argtypes = [_P, C.c_uint32, C.POINTER(C.c_int)]
        L.orc_fnv1a64.restype = C.c_uint64
        L.orc_fnv1a64.argtypes = [_P, C.c_uint64]
        L.orc_xxh64.restype = C.c_uint64
        L.orc_xxh64.argtypes = [_P, C.c_uint64, C.c_uint64]
        L.orc_offset_skip.restype = None
        L.orc_offset_skip.argtypes = [C.c_char_p, C.c_uint32, C.c_uint64, C.POINTER(C.c_uint64),
                                      C.POINTER(C.c_uint64)]
        L.orc_cpu_baseline.restype = C.c_double
        L.orc_cpu_baseline.argtypes = [_P, _P, C.c_uint64, _P, C.c_uint32, C.c_uint64, _P, C.c_uint64, C.c_uint32,
                                       C.c_int, C.c_int, _P]
        L.orc_cpu_baseline_reps.restype = C.c_double
        L.orc_cpu_baseline_reps.argtypes = [_P, _P, C.c_uint64, _P, C.c_uint32, C.c_uint64, _P, C.c_uint64,
                                            C.c_uint32, C.c_int, C.c_int, C.c_uint32, _P]
        L.orc_set_cpu_order.restype = None
        L.orc_set_cpu_order.argtypes = [_P, C.c_int]
        L.orc_cpu_baseline_chain_reps.restype = C.c_double
        L.orc_cpu_baseline_chain_reps.argtypes = [_P, _P, C.c_uint64, _P, C.c_uint32, C.c_uint64, _P, _P, C.c_uint32,
                                                  _P, C.c_uint64, C.c_uint32, C.c_int, C.c_int, C.c_uint32, _P]
        L.orc_lpm_build.restype = C.c_int
        L.orc_lpm_build.argtypes = [_P, _P, _P, C.c_uint64, _P, _P, C.POINTER(C.c_uint64)]
        L.orc_lpm_lookup.restype = None
        L.orc_lpm_lookup.argtypes = [_P, _P, _P, C.c_uint64, _P]
        L.orc_chain_classify.restype = None
        L.orc_chain_classify.argtypes = [_P, _P, C.c_uint64, _P, C.c_uint32, C.c_uint64, _P, _P, C.c_uint32, _P,
                                         C.c_uint64, _P, _P]
        _lib = L
    return _lib


def lut_build(names, m):
    enc = [n.encode() for n in names]
    arr = (C.c_char_p * len(enc))(*enc)
    lens = (C.c_uint32 * len(enc))(*[len(e) for e in enc])
    out = np.empty(m, dtype=np.uint32)
    rc = lib().orc_lut_build(arr, lens, len(enc), m, out.ctypes.data)
    assert rc == 0
    return out


def classify(buf, n, lut, *, offs=None, stride=64, lens=None, fixed_len=60, swap=True):
    """Mutates `buf` (numpy u8) like the product; returns backend u16[n]."""
    lut = np.ascontiguousarray(lut, dtype=np.uint32)
    offs64 = None if offs is None else np.ascontiguousarray(offs, dtype=np.uint64)
    lens16 = None if lens is None else np.ascontiguousarray(lens, dtype=np.uint16)
    out = np.empty(max(n, 1), dtype=np.uint16)
    lib().orc_classify(buf.ctypes.data, None if offs64 is None else offs64.ctypes.data, stride,
                       None if lens16 is None else lens16.ctypes.data, fixed_len, n, lut.ctypes.data,
                       lut.size, 1 if swap else 0, out.ctypes.data)
    return out[:n]


def group(backend, nb):
    backend = np.ascontiguousarray(backend, dtype=np.uint16)
    perm = np.empty(max(backend.size, 1), dtype=np.uint32)
    counts = np.empty(nb + 1, dtype=np.uint32)
    lib().orc_group(backend.ctypes.data, backend.size, nb, perm.ctypes.data, counts.ctypes.data)
    return perm[:backend.size], counts


def flow_hash(frame: bytes):
    b = (C.c_uint8 * max(len(frame), 1)).from_buffer_copy(frame if frame else b"\0")
    ok = C.c_int(0)
    h = lib().orc_flow_hash(b, len(frame), C.byref(ok))
    return h if ok.value else None


TBL24 = (1 << 24) + 1


def routes_arrays(routes):
    """[(dotted-quad | int, len, gate)] -> (u32 prefixes, u8 lens, u16 gates)."""
    pf, ln, gt = [], [], []
    for ip, plen, gate in routes:
        if isinstance(ip, str):
            a = [int(x) for x in ip.split(".")]
            ip = (a[0] << 24) | (a[1] << 16) | (a[2] << 8) | a[3]
        pf.append(ip)
        ln.append(plen)
        gt.append(gate)
    return (np.asarray(pf, dtype=np.uint32), np.asarray(ln, dtype=np.uint8), np.asarray(gt, dtype=np.uint16))


def lpm_build(routes):
    """-> (rc, tbl24 u16[2^24+1], tbl_long u16[used])"""
    pf, ln, gt = routes_arrays(routes)
    t24 = np.empty(TBL24, dtype=np.uint16)
    tl = np.empty(TBL24, dtype=np.uint16)
    used = C.c_uint64(0)
    rc = lib().orc_lpm_build(pf.ctypes.data, ln.ctypes.data, gt.ctypes.data, pf.size, t24.ctypes.data,
                             tl.ctypes.data, C.byref(used))
    return rc, t24, tl[:used.value].copy()


def lpm_lookup(t24, tl, ips):
    ips = np.ascontiguousarray(ips, dtype=np.uint32)
    tl = tl if tl.size else np.zeros(1, dtype=np.uint16)
    out = np.empty(max(ips.size, 1), dtype=np.uint16)
    lib().orc_lpm_lookup(t24.ctypes.data, tl.ctypes.data, ips.ctypes.data, ips.size, out.ctypes.data)
    return out[:ips.size]


def chain_classify(buf, n, t24, tl, lut, *, offs=None, stride=64, lens=None, fixed_len=60, lpm_groups=3):
    """lpm() -> maglev(): (gate u16[n], backend u16[n]); `buf` is not modified."""
    lut = np.ascontiguousarray(lut, dtype=np.uint32)
    tl = tl if tl.size else np.zeros(1, dtype=np.uint16)
    offs64 = None if offs is None else np.ascontiguousarray(offs, dtype=np.uint64)
    lens16 = None if lens is None else np.ascontiguousarray(lens, dtype=np.uint16)
    gate = np.empty(max(n, 1), dtype=np.uint16)
    be = np.empty(max(n, 1), dtype=np.uint16)
    lib().orc_chain_classify(buf.ctypes.data, None if offs64 is None else offs64.ctypes.data, stride,
                             None if lens16 is None else lens16.ctypes.data, fixed_len, n, t24.ctypes.data,
                             tl.ctypes.data, lpm_groups, lut.ctypes.data, lut.size, gate.ctypes.data, be.ctypes.data)
    return gate[:n], be[:n]


def cpu_baseline(buf, n, lut, nb, *, offs=None, stride=64, lens=None, fixed_len=60, chain=None, lpm_groups=3,
                 cache=True, threads=1, reps=1):
    """The reference's producer loop restated in C (the CPU baseline).  `chain` = (tbl24, tbl_long)
    runs test/lpm's stage first (config C5).  Modifies `buf` (MAC swaps).  -> (wall seconds, backend)."""
    lut = np.ascontiguousarray(lut, dtype=np.uint32)
    offs64 = None if offs is None else np.ascontiguousarray(offs, dtype=np.uint64)
    lens16 = None if lens is None else np.ascontiguousarray(lens, dtype=np.uint16)
    be = np.empty(max(n, 1), dtype=np.uint16)
    o = None if offs64 is None else offs64.ctypes.data
    ln = None if lens16 is None else lens16.ctypes.data
    if chain is None:
        t = lib().orc_cpu_baseline_reps(buf.ctypes.data, o, stride, ln, fixed_len, n, lut.ctypes.data, lut.size, nb,
                                        1 if cache else 0, threads, reps, be.ctypes.data)
    else:
        t24, tl = chain
        tl = tl if tl.size else np.zeros(1, dtype=np.uint16)
        t = lib().orc_cpu_baseline_chain_reps(buf.ctypes.data, o, stride, ln, fixed_len, n, t24.ctypes.data,
                                              tl.ctypes.data, lpm_groups, lut.ctypes.data, lut.size, nb,
                                              1 if cache else 0, threads, reps, be.ctypes.data)
    return t, be[:n]
