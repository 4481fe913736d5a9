"""ctypes binding of the in-tree C-ABI library `netbricks_amd/libnbgpu.so` (include/nbgpu.h).

The product path has no CPU fallback: if the HIP library is missing this module
raises at import time, and every device entry point returns -ENODEV without a GPU.
"""
from __future__ import annotations

import ctypes as C
import os

try:
    # torch ships its own libamdhip64 / libhsa-runtime64.  Load them before libnbgpu.so so that the
    # library binds to that runtime (same SONAME): loaded first, libnbgpu.so would pull in the
    # system runtime and torch a second one, and a second HSA runtime in the process sees no GPU
    # ("no ROCm-capable device is detected").  Importing torch does not initialise the GPU.
    import torch  # noqa: F401
except ImportError:  # the C-ABI needs no torch; only the device-memory plumbing does
    pass

_HERE = os.path.dirname(os.path.abspath(__file__))
# NBG_LIB_OVERRIDE: diagnostic builds of the same library (tools/); never set by the product
LIB_PATH = os.environ.get("NBG_LIB_OVERRIDE") or os.path.join(_HERE, "libnbgpu.so")

NBG_OK = 0
NBG_SENTINEL = 0xFFFF
NBG_SWAP_MACS = 0x1
NBG_LUT_LDS = 0x2
NBG_OWNED_WINDOWS = 0x4
NBG_WB_PARTIAL = 0x8
NBG_DEFER_GROUP = 0x10
NBG_LUT_TILED = 0x20
NBG_STREAM_DESC = 0x40
NBG_GROUP_LAG = 0x80
NBG_HOST_SLOTS = 8
NBG_MAX_MULTI = 16
NBG_RING_SLOTS = 64
NBG_RING_MAX_QUEUES = 16
NBG_EBUSY = -16
NBG_EINVAL = -22
NBG_EIO = -5
NBG_TRACE_UNIQUE = 0x1
NBG_LPM_TBL24_SIZE = (1 << 24) + 1

# every symbol include/nbgpu.h declares: name -> (restype, argtypes)
_P = C.c_void_p


class NbgBatch(C.Structure):
    """struct nbg_batch (include/nbgpu.h): one batch of nbg_maglev_classify_device_multi."""
    _fields_ = [("d_pkts", C.c_void_p), ("n_pkts", C.c_uint64), ("d_backend", C.c_void_p),
                ("d_perm", C.c_void_p), ("d_counts", C.c_void_p), ("d_mac_out", C.c_void_p)]


class NbgDescBatch(C.Structure):
    """struct nbg_desc_batch (include/nbgpu.h): one batch of nbg_maglev_classify_desc_multi /
    nbg_chain_lpm_maglev_multi."""
    _fields_ = [("d_pkts", C.c_void_p), ("d_off", C.c_void_p), ("d_len", C.c_void_p), ("n_pkts", C.c_uint64),
                ("d_backend", C.c_void_p), ("d_perm", C.c_void_p), ("d_counts", C.c_void_p), ("d_gate", C.c_void_p)]


class NbgRingBatch(C.Structure):
    """struct nbg_ring_batch (include/nbgpu.h): one batch of nbg_ring_post_burst."""
    _fields_ = [("d_pkts", C.c_void_p), ("n_pkts", C.c_uint64), ("d_backend", C.c_void_p)]


SIGNATURES = {
    "nbg_maglev_create": (C.c_int, [C.POINTER(C.c_char_p), C.POINTER(C.c_uint32), C.c_uint32, C.c_uint64,
                                    C.c_int, C.POINTER(_P)]),
    "nbg_maglev_create_from_lut": (C.c_int, [_P, C.c_uint64, C.c_uint32, C.c_int, C.POINTER(_P)]),
    "nbg_maglev_destroy": (None, [_P]),
    "nbg_maglev_backends": (C.c_uint32, [_P]),
    "nbg_maglev_table_size": (C.c_uint64, [_P]),
    "nbg_maglev_lut": (C.c_int, [_P, _P, C.c_uint64]),
    "nbg_maglev_reserve": (C.c_int, [_P, C.c_uint64]),
    "nbg_maglev_classify_device": (C.c_int, [_P, _P, _P, _P, C.c_uint32, C.c_uint16, C.c_uint64, C.c_uint32,
                                             _P, _P, _P, _P]),
    "nbg_maglev_classify_device_ex": (C.c_int, [_P, _P, _P, _P, C.c_uint32, C.c_uint16, C.c_uint64, C.c_uint32,
                                                _P, _P, _P, _P, _P]),
    "nbg_maglev_classify_device_multi": (C.c_int, [_P, _P, C.c_uint32, C.c_uint32, C.c_uint16, C.c_uint32, _P]),
    "nbg_maglev_classify_desc_multi": (C.c_int, [_P, _P, C.c_uint32, C.c_uint32, _P]),
    "nbg_chain_lpm_maglev_multi": (C.c_int, [_P, _P, C.c_uint32, _P, C.c_uint32, C.c_uint32, _P]),
    "nbg_maglev_finish_group": (C.c_int, [_P, _P]),
    "nbg_ring_start": (C.c_int, [_P, C.c_uint32, C.c_uint16, C.c_uint32, C.c_uint32, _P, C.POINTER(_P)]),
    "nbg_ring_post": (C.c_int, [_P, _P, C.c_uint64, _P, C.POINTER(C.c_uint64)]),
    "nbg_ring_post_burst": (C.c_int, [_P, _P, C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)]),
    "nbg_ring_group": (C.c_int, [_P, C.c_uint64, _P, _P, _P]),
    "nbg_ring_group_burst": (C.c_int, [_P, C.c_uint64, C.c_uint32, _P, _P, _P]),
    "nbg_ring_poll": (C.c_int, [_P, C.POINTER(C.c_uint64)]),
    "nbg_ring_wait": (C.c_int, [_P, C.c_uint64, C.c_uint32]),
    "nbg_ring_stop": (C.c_int, [_P]),
    "nbg_ring_kernel_ms": (C.c_int, [_P, C.POINTER(C.c_float)]),
    "nbg_ring_queue_open": (C.c_int, [_P, C.POINTER(_P)]),
    "nbg_ring_queue_post": (C.c_int, [_P, _P, C.c_uint64, _P, C.POINTER(C.c_uint64)]),
    "nbg_ring_queue_poll": (C.c_int, [_P, C.POINTER(C.c_uint64)]),
    "nbg_ring_queue_wait": (C.c_int, [_P, C.c_uint64, C.c_uint32]),
    "nbg_ring_queue_group": (C.c_int, [_P, C.c_uint64, _P, _P, _P]),
    "nbg_ring_queue_close": (C.c_int, [_P]),
    "nbg_maglev_check": (C.c_int, [_P]),
    "nbg_maglev_classify_host": (C.c_int, [_P, _P, _P, C.c_uint64, C.c_uint32, _P, _P, _P]),
    "nbg_maglev_host_submit": (C.c_int, [_P, _P, _P, C.c_uint64, C.c_uint32, _P, _P, _P, C.POINTER(C.c_uint64)]),
    "nbg_maglev_host_wait": (C.c_int, [_P, C.c_uint64]),
    "nbg_maglev_host_query": (C.c_int, [_P, C.c_uint64, C.POINTER(C.c_int)]),
    "nbg_host_register": (C.c_int, [_P, C.c_uint64, C.c_int, C.POINTER(_P)]),
    "nbg_host_unregister": (C.c_int, [_P, C.c_int]),
    "nbg_device_local_cpus": (C.c_int, [C.c_int, C.POINTER(C.c_int32), C.c_uint32, C.POINTER(C.c_uint32)]),
    "nbg_host_ring_start": (C.c_int, [C.c_int, C.c_uint32, C.c_uint32, C.POINTER(_P)]),
    "nbg_host_ring_stop": (C.c_int, [_P]),
    "nbg_maglev_set_host_ring": (C.c_int, [_P, _P]),
    "nbg_lpm_create": (C.c_int, [_P, _P, _P, C.c_uint64, C.c_int, C.POINTER(_P)]),
    "nbg_lpm_destroy": (None, [_P]),
    "nbg_lpm_lookup_device": (C.c_int, [_P, _P, C.c_uint64, _P, _P]),
    "nbg_chain_lpm_maglev_device": (C.c_int, [_P, _P, C.c_uint32, _P, _P, _P, C.c_uint32, C.c_uint16, C.c_uint64,
                                              C.c_uint32, _P, _P, _P, _P, _P]),
    "nbg_last_error": (C.c_char_p, []),
    "nbg_lpm_build_host": (C.c_int, [_P, _P, _P, C.c_uint64, _P, _P, C.c_uint64, C.POINTER(C.c_uint64)]),
    "nbg_lut_build_host": (C.c_int, [C.POINTER(C.c_char_p), C.POINTER(C.c_uint32), C.c_uint32, C.c_uint64, _P]),
    "nbg_trace_layout": (C.c_uint64, [C.c_uint64, C.c_int, C.c_uint64, _P, _P]),
    "nbg_trace_fill": (C.c_int, [_P, _P, _P, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32]),
}


# diagnostics the library exports beside include/nbgpu.h (tests only; not part of the C-ABI)
DEBUG_SIGNATURES = {
    "nbg_debug_set_group_compact": (C.c_int, [C.c_int]),
    "nbg_debug_group_lds": (C.c_uint64, [C.c_uint32, C.c_int]),
    "nbg_debug_lds_beside_ring": (C.c_uint64, []),
    "nbg_debug_hold_cus": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, _P]),
    "nbg_debug_host_win": (C.c_int, [_P, C.c_uint64]),
}


class NbgError(RuntimeError):
    def __init__(self, code: int, where: str):
        self.code = code
        super().__init__(f"{where} failed ({code}): {last_error()}")


def _load() -> C.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(there is no CPU fallback for the Maglev path)")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            if os.environ.get("NBG_LIB_OVERRIDE"):  # an older diagnostic build (A/B timing)
                continue
            raise ImportError(f"{LIB_PATH}: missing {name}")
        fn.restype = res
        fn.argtypes = args
    for name, (res, args) in DEBUG_SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is not None:
            fn.restype = res
            fn.argtypes = args
    return lib


lib = _load()


def last_error() -> str:
    msg = lib.nbg_last_error()
    return msg.decode(errors="replace") if msg else ""


def check(rc: int, where: str) -> None:
    if rc != NBG_OK:
        raise NbgError(rc, where)


def names_args(names):
    enc = [n.encode("utf-8") for n in names]
    arr = (C.c_char_p * len(enc))(*enc)
    lens = (C.c_uint32 * len(enc))(*[len(e) for e in enc])
    return arr, lens, enc
