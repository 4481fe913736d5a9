"""Python surface of the MI355X Maglev path (thin wrapper over include/nbgpu.h).

Mirrors the reference's Maglev NF (test/maglev/src/nf.rs): `Maglev(backends, 65537)`
builds the consistent-hash LUT (nf.rs:70-76) and `Maglev.group_by(...)` performs, for a
whole device-resident batch, what `parse::<MacHeader>().transform(swap).group_by(ct,
group_fn)` does per packet (nf.rs:92-108): MAC swap, 5-tuple FNV-1a, `lut[hash % M]`,
and the per-group FIFO order of the group_by MPSC queues (operators/group_by.rs:43-55).
PyTorch is only used for device memory and streams.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import (NBG_DEFER_GROUP, NBG_GROUP_LAG, NBG_HOST_SLOTS, NBG_LUT_LDS, NBG_LUT_TILED, NBG_MAX_MULTI, NBG_OWNED_WINDOWS,
                   NBG_SENTINEL, NBG_STREAM_DESC, NbgBatch, NbgDescBatch, NbgRingBatch,
                   NBG_SWAP_MACS, NBG_WB_PARTIAL, check, lib)

__all__ = ["Maglev", "GroupedBatch", "Ring", "RingQueue", "HostRing", "build_lut", "make_trace", "NBG_SENTINEL"]


def _ptr(t) -> Optional[int]:
    if t is None:
        return None
    return t.data_ptr()


def _check_np(name: str, a, dtype, min_size: int) -> None:
    """The library writes min_size elements of `dtype` through a raw pointer: refuse anything else."""
    if not isinstance(a, np.ndarray):
        raise ValueError(f"{name}: expected a numpy array, got {type(a).__name__}")
    if a.dtype != np.dtype(dtype):
        raise ValueError(f"{name}: dtype {a.dtype}, expected {np.dtype(dtype)}")
    if not a.flags.c_contiguous or not a.flags.writeable:
        raise ValueError(f"{name}: must be C-contiguous and writeable")
    if a.size < min_size:
        raise ValueError(f"{name}: {a.size} elements, needs >= {min_size}")


def _check_dev(name: str, t, dtype, min_size: int, device) -> None:
    """Device outputs/inputs handed to the library as raw pointers: dtype, contiguity, size, device."""
    if t is None:
        return
    if t.dtype != dtype:
        raise ValueError(f"{name}: dtype {t.dtype}, expected {dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if t.numel() < min_size:
        raise ValueError(f"{name}: {t.numel()} elements, needs >= {min_size}")
    if t.device != device:
        raise ValueError(f"{name}: on {t.device}, expected {device}")


def _slot_tail(stride: int, frame_len: int) -> int:
    """Bytes the library may touch in the last fixed slot: slots of >= 64 B own their 64-B window
    (read whole, and rewritten whole by the in-place swap: include/nbgpu.h), narrower slots only
    their frame."""
    return max(64, frame_len) if stride >= 64 else frame_len


def _check_owned(name: str, pkts, offsets, n_pkts: int, stream=None) -> None:
    """NBG_OWNED_WINDOWS: the kernels read, and in place rewrite, the whole 64-B window at every offset,
    so each window must lie inside pkts.  One device reduction, run on `stream` (the raw stream the
    kernels are launched on; None = torch's current stream), so that offsets the caller wrote there
    are read in order; its .item() synchronises the host with that stream once per call, which a
    multi-stream pipeline avoids with bounds_check=False after checking its descriptors once."""
    import contextlib

    import torch

    if not n_pkts or offsets is None:
        return
    ctx = (torch.cuda.stream(torch.cuda.ExternalStream(stream, device=pkts.device)) if stream
           else contextlib.nullcontext())
    with ctx:
        if torch.cuda.is_current_stream_capturing():
            return  # no reduction inside a graph capture: the caller's descriptors are taken as they are
        top = int((offsets[:n_pkts].view(torch.int32).to(torch.int64) & 0xFFFFFFFF).max().item())
    if top + 64 > pkts.numel():
        raise ValueError(f"{name}: the 64-B owned window at offset {top} runs past the end of pkts "
                         f"({pkts.numel()} B); pass owned_windows=False for frames without a 64-B data room")


def build_lut(backends: Sequence[str], lut_size: int = 65537) -> np.ndarray:
    """The product's host LUT builder (Maglev::new, nf.rs:70-76) -> u16 entries."""
    arr, lens, _keep = _lib.names_args(backends)
    out = np.empty(lut_size, dtype=np.uint16)
    check(lib.nbg_lut_build_host(arr, lens, len(backends), lut_size, out.ctypes.data), "nbg_lut_build_host")
    return out


def make_trace(n: int, mode: int = 0, seed: int = 0x4E42474D41474C56, n_flows: int = 65536,
               unique: bool = False):
    """Synthetic trace on the host: (bytes u8[size], offsets u32[n], lens u16[n])."""
    off = np.empty(n, dtype=np.uint32)
    ln = np.empty(n, dtype=np.uint16)
    size = lib.nbg_trace_layout(n, mode, seed, off.ctypes.data, ln.ctypes.data)
    buf = np.zeros(max(size, 1), dtype=np.uint8)
    flags = _lib.NBG_TRACE_UNIQUE if unique else 0
    check(lib.nbg_trace_fill(buf.ctypes.data, off.ctypes.data, ln.ctypes.data, n, seed, n_flows, flags),
          "nbg_trace_fill")
    return buf, off, ln


@dataclass
class GroupedBatch:
    """Result of one batch: per-packet backend (NBG_SENTINEL = would-panic packet), and
    the per-group FIFO order: perm[group_start[g]:group_start[g]+counts[g]] are the
    packets of group g in arrival order (groups 0..n-1, then the sentinel group)."""
    backend: "object"
    perm: "object"
    counts: "object"

    def group_start(self):
        c = self.counts.cpu().numpy().view(np.uint32).astype(np.int64)
        return np.concatenate([[0], np.cumsum(c)[:-1]])


class Maglev:
    """Device-resident Maglev consistent-hash steering (test/maglev/src/nf.rs:14-111)."""

    def __init__(self, backends: Optional[Sequence[str]] = None, lut_size: int = 65537, device: int = 0,
                 lut: Optional[np.ndarray] = None, n_backends: Optional[int] = None):
        self._h = C.c_void_p()
        self.device = device
        if lut is not None:
            lut = np.ascontiguousarray(lut, dtype=np.uint16)
            nb = int(n_backends if n_backends is not None else int(lut.max()) + 1)
            check(lib.nbg_maglev_create_from_lut(lut.ctypes.data, lut.size, nb, device, C.byref(self._h)),
                  "nbg_maglev_create_from_lut")
        else:
            if not backends:
                raise ValueError("backends must be non-empty")
            arr, lens, _keep = _lib.names_args(backends)
            check(lib.nbg_maglev_create(arr, lens, len(backends), lut_size, device, C.byref(self._h)),
                  "nbg_maglev_create")
        self.n_backends = lib.nbg_maglev_backends(self._h)
        self.lut_size = lib.nbg_maglev_table_size(self._h)

    def close(self) -> None:
        ring = self.__dict__.get("_ring")
        if ring is not None:
            ring.stop()
        if self._h:
            lib.nbg_maglev_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def lut(self) -> np.ndarray:
        out = np.empty(self.lut_size, dtype=np.uint16)
        check(lib.nbg_maglev_lut(self._h, out.ctypes.data, out.size), "nbg_maglev_lut")
        return out

    def reserve(self, max_pkts: int) -> None:
        check(lib.nbg_maglev_reserve(self._h, max_pkts), "nbg_maglev_reserve")

    def check(self) -> None:
        check(lib.nbg_maglev_check(self._h), "nbg_maglev_check")

    def group_by_region(self, region: "HostRegion", n_pkts: int, offsets, lens, *, swap_macs: bool = True,
                        group: bool = True, backend=None, perm=None, counts=None, stream=None) -> GroupedBatch:
        """Zero-copy host path: classify n_pkts frames that live in a registered host region
        (frame i at region offset offsets[i], lens[i] bytes; both u32/u16 tensors on this device).
        The GPU reads the header windows over PCIe and writes the swapped MACs back into the
        frames (16 B per frame); mbuf-style owned 64-B windows are assumed."""
        import torch

        if region.device != self.device or region.dev_ptr is None:
            raise ValueError("region: not registered on this handle's device")
        dev = torch.device("cuda", self.device)
        _check_dev("offsets", offsets, torch.uint32, n_pkts, dev)
        _check_dev("lens", lens, torch.uint16, n_pkts, dev)
        if offsets is None or lens is None:
            raise ValueError("offsets and lens are required")
        # the kernel reads (and may rewrite) the 64-B owned window at every offset, over PCIe: an
        # offset past the registered region would touch host memory outside it (the C host_submit
        # zero-copy path checks the same bound, nbgpu_api.hip)
        if n_pkts and int((offsets[:n_pkts].view(torch.int32).to(torch.int64) & 0xFFFFFFFF).max().item()) + 64 \
                > region.array.nbytes:
            raise ValueError("offsets: a 64-B window past the end of the registered region")
        if backend is None:
            backend = torch.empty(max(n_pkts, 1), dtype=torch.uint16, device=dev)
        if group and perm is None:
            perm = torch.empty(max(n_pkts, 1), dtype=torch.uint32, device=dev)
        if group and counts is None:
            counts = torch.empty(self.n_backends + 1, dtype=torch.uint32, device=dev)
        _check_dev("backend", backend, torch.uint16, n_pkts, dev)
        _check_dev("perm", perm, torch.uint32, n_pkts, dev)
        _check_dev("counts", counts, torch.uint32, self.n_backends + 1, dev)
        if stream is None:
            stream = torch.cuda.current_stream(dev).cuda_stream
        flags = (NBG_SWAP_MACS if swap_macs else 0) | NBG_OWNED_WINDOWS | NBG_WB_PARTIAL
        rc = lib.nbg_maglev_classify_device_ex(self._h, region.dev_ptr, _ptr(offsets), _ptr(lens), 0, 0, n_pkts,
                                               flags, _ptr(backend), _ptr(perm) if group else None,
                                               _ptr(counts) if group else None, None, stream)
        check(rc, "nbg_maglev_classify_device_ex")
        return GroupedBatch(backend, perm if group else None, counts if group else None)

    def group_by(self, pkts, n_pkts: int, *, stride: int = 64, frame_len: int = 60, offsets=None, lens=None,
                 swap_macs: bool = True, group: bool = True, scatter: bool = True, lut_lds: bool = False,
                 owned_windows: bool = False, wb_partial: bool = False,
                 defer_group: bool = False, lut_tiled: bool = False, stream_desc: bool = False,
                 group_lag: bool = False, bounds_check: bool = True,
                 backend=None, perm=None, counts=None, mac_out=None, stream=None) -> GroupedBatch:
        """Classify a device-resident batch (torch uint8 tensor on this device).

        Packet i starts at pkts[offsets[i]] (u32 tensor) or pkts[i*stride]; its length is
        lens[i] (u16 tensor) or frame_len.  Asynchronous on `stream` (default: torch's
        current stream).  group_lag=True (NBG_GROUP_LAG): perm / counts of this batch are
        completed by the handle's next call (inside its classify launch) or by finish_group()."""
        import torch

        dev = pkts.device
        if pkts.dtype != torch.uint8 or not pkts.is_contiguous():
            raise ValueError("pkts: expected a contiguous uint8 tensor")
        if dev.type != "cuda" or dev.index != self.device:
            raise ValueError(f"pkts: on {dev}, expected cuda:{self.device}")
        if offsets is None and n_pkts and (n_pkts - 1) * stride + _slot_tail(stride, frame_len) > pkts.numel():
            raise ValueError("pkts: smaller than n_pkts fixed slots")
        _check_dev("offsets", offsets, torch.uint32, n_pkts, dev)
        _check_dev("lens", lens, torch.uint16, n_pkts, dev)
        if owned_windows and bounds_check:
            _check_owned("offsets", pkts, offsets, n_pkts, stream)
        _check_dev("backend", backend, torch.uint16, n_pkts, dev)
        _check_dev("perm", perm, torch.uint32, n_pkts, dev)
        _check_dev("counts", counts, torch.uint32, self.n_backends + 1, dev)
        _check_dev("mac_out", mac_out, torch.uint8, 12 * n_pkts, dev)
        if backend is None:
            backend = torch.empty(n_pkts, dtype=torch.uint16, device=dev)
        scatter = group and scatter
        if scatter and perm is None:
            perm = torch.empty(max(n_pkts, 1), dtype=torch.uint32, device=dev)
        if group and counts is None:
            counts = torch.empty(self.n_backends + 1, dtype=torch.uint32, device=dev)
        if stream is None:
            stream = torch.cuda.current_stream(dev).cuda_stream
        flags = ((NBG_SWAP_MACS if swap_macs else 0) | (NBG_LUT_LDS if lut_lds else 0)
                 | (NBG_OWNED_WINDOWS if owned_windows else 0) | (NBG_WB_PARTIAL if wb_partial else 0)
                 | (NBG_DEFER_GROUP if defer_group else 0) | (NBG_LUT_TILED if lut_tiled else 0)
                 | (NBG_STREAM_DESC if stream_desc else 0) | (NBG_GROUP_LAG if group_lag else 0))
        rc = lib.nbg_maglev_classify_device_ex(self._h, _ptr(pkts), _ptr(offsets), _ptr(lens), stride, frame_len,
                                               n_pkts, flags, _ptr(backend), _ptr(perm) if scatter else None,
                                               _ptr(counts) if group else None, _ptr(mac_out), stream)
        check(rc, "nbg_maglev_classify_device_ex")
        return GroupedBatch(backend, perm if scatter else None, counts if group else None)

    def group_by_multi(self, batches, *, stride: int = 64, frame_len: int = 60, swap_macs: bool = True,
                       group: bool = True, scatter: bool = True, records: bool = False,
                       defer_group: bool = False, stream=None) -> list:
        """Classify several device-resident fixed-slot batches in one launch of each kernel
        (nbg_maglev_classify_device_multi): `batches` is a list of (pkts, n_pkts) with pkts a
        contiguous uint8 tensor on this device.  Every batch gets its own backend / perm / counts
        (and 12-B MAC records with records=True), as group_by would give it alone.  Returns one
        GroupedBatch per batch, or (GroupedBatch, records tensor) pairs with records=True."""
        import torch

        if not 1 <= len(batches) <= NBG_MAX_MULTI:
            raise ValueError(f"batches: 1..{NBG_MAX_MULTI}")
        arr = (NbgBatch * len(batches))()
        out = []
        for j, (pkts, n_pkts) in enumerate(batches):
            dev = pkts.device
            if pkts.dtype != torch.uint8 or not pkts.is_contiguous():
                raise ValueError(f"batch {j}: expected a contiguous uint8 tensor")
            if dev.type != "cuda" or dev.index != self.device:
                raise ValueError(f"batch {j}: on {dev}, expected cuda:{self.device}")
            if n_pkts and (n_pkts - 1) * stride + _slot_tail(stride, frame_len) > pkts.numel():
                raise ValueError(f"batch {j}: smaller than n_pkts fixed slots")
            backend = torch.empty(max(n_pkts, 1), dtype=torch.uint16, device=dev)
            perm = torch.empty(max(n_pkts, 1), dtype=torch.uint32, device=dev) if group and scatter else None
            counts = torch.empty(self.n_backends + 1, dtype=torch.uint32, device=dev) if group else None
            mac = torch.empty(max(12 * n_pkts, 1), dtype=torch.uint8, device=dev) if records else None
            arr[j] = NbgBatch(_ptr(pkts), n_pkts, _ptr(backend), _ptr(perm), _ptr(counts), _ptr(mac))
            out.append((GroupedBatch(backend, perm, counts), mac))
        if stream is None:
            stream = torch.cuda.current_stream(torch.device("cuda", self.device)).cuda_stream
        flags = (NBG_SWAP_MACS if swap_macs else 0) | (NBG_DEFER_GROUP if defer_group else 0)
        check(lib.nbg_maglev_classify_device_multi(self._h, arr, len(batches), stride, frame_len, flags, stream),
              "nbg_maglev_classify_device_multi")
        self._multi_keep = arr
        return [g for g, _ in out] if not records else out

    def _desc_batches(self, batches, group: bool, scatter: bool, gates: bool, owned: bool = False, stream=None):
        """ctypes array of nbg_desc_batch for group_by_desc_multi / chain_lpm_maglev_multi: `batches`
        is a list of (pkts, offsets, lens, n_pkts) device tensors (u8, u32, u16) on this device."""
        import torch

        if not 1 <= len(batches) <= NBG_MAX_MULTI:
            raise ValueError(f"batches: 1..{NBG_MAX_MULTI}")
        arr = (NbgDescBatch * len(batches))()
        out = []
        for j, (pkts, offsets, lens, n_pkts) in enumerate(batches):
            dev = pkts.device
            if pkts.dtype != torch.uint8 or not pkts.is_contiguous():
                raise ValueError(f"batch {j}: expected a contiguous uint8 tensor")
            if dev.type != "cuda" or dev.index != self.device:
                raise ValueError(f"batch {j}: on {dev}, expected cuda:{self.device}")
            _check_dev(f"batch {j} offsets", offsets, torch.uint32, n_pkts, dev)
            _check_dev(f"batch {j} lens", lens, torch.uint16, n_pkts, dev)
            if n_pkts and (offsets is None or lens is None):
                raise ValueError(f"batch {j}: offsets and lens are required")
            if owned:
                _check_owned(f"batch {j} offsets", pkts, offsets, n_pkts, stream)
            backend = torch.empty(max(n_pkts, 1), dtype=torch.uint16, device=dev)
            perm = torch.empty(max(n_pkts, 1), dtype=torch.uint32, device=dev) if group and scatter else None
            counts = torch.empty(self.n_backends + 1, dtype=torch.uint32, device=dev) if group else None
            gate = torch.empty(max(n_pkts, 1), dtype=torch.uint16, device=dev) if gates else None
            arr[j] = NbgDescBatch(_ptr(pkts), _ptr(offsets), _ptr(lens), n_pkts, _ptr(backend), _ptr(perm),
                                  _ptr(counts), _ptr(gate))
            out.append((backend, perm, counts, gate))
        return arr, out

    def group_by_desc_multi(self, batches, *, swap_macs: bool = True, owned_windows: bool = False,
                            group: bool = True, scatter: bool = True, defer_group: bool = False,
                            wb_partial: bool = False, bounds_check: bool = True, stream=None) -> list:
        """Classify several device-resident descriptor batches (IMIX: (pkts, offsets, lens, n_pkts)
        per batch) in one launch of each kernel (nbg_maglev_classify_desc_multi).  Every batch gets
        its own backend / perm / counts, as group_by(..., offsets=, lens=) would give it alone.
        owned_windows=True (mbuf data rooms: the 64 B at every offset belong to that frame) lets the
        MAC swap write whole windows back; every window is then checked to lie inside its pkts.
        Returns one GroupedBatch per batch."""
        import torch

        if stream is None:
            stream = torch.cuda.current_stream(torch.device("cuda", self.device)).cuda_stream
        arr, out = self._desc_batches(batches, group, scatter, False, owned_windows and bounds_check, stream)
        flags = ((NBG_SWAP_MACS if swap_macs else 0) | (NBG_OWNED_WINDOWS if owned_windows else 0)
                 | (NBG_DEFER_GROUP if defer_group else 0) | (NBG_WB_PARTIAL if wb_partial else 0))
        check(lib.nbg_maglev_classify_desc_multi(self._h, arr, len(batches), flags, stream),
              "nbg_maglev_classify_desc_multi")
        self._multi_keep = arr
        return [GroupedBatch(b, p, c) for b, p, c, _ in out]

    def finish_group(self, stream=None) -> None:
        """Launch the grouping deferred by group_by(..., defer_group=True) or left pending by
        group_by(..., group_lag=True)."""
        import torch

        if stream is None:
            stream = torch.cuda.current_stream(torch.device("cuda", self.device)).cuda_stream
        check(lib.nbg_maglev_finish_group(self._h, stream), "nbg_maglev_finish_group")

    def host_submit(self, ptrs: np.ndarray, lens: np.ndarray, backend: np.ndarray, perm: Optional[np.ndarray] = None,
                    counts: Optional[np.ndarray] = None, swap_macs: bool = True) -> int:
        """Pipelined host path (nbg_maglev_host_submit): frame i is `lens[i]` bytes at address
        `ptrs[i]` (u64 numpy arrays of host mbuf data pointers).  Returns a ticket; backend / perm /
        counts (numpy) and the frames' MAC swap are complete when host_wait(ticket) returns.  The
        caller keeps the frames alive until then; this wrapper holds the pointer, length and output
        arrays it passes to the library (converted copies included) until the batch completes."""
        ptrs = np.ascontiguousarray(ptrs, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint16)
        n = ptrs.size
        if lens.size != n:
            raise ValueError(f"lens: {lens.size} entries for {n} frames")
        _check_np("backend", backend, np.uint16, n)
        if perm is not None:
            _check_np("perm", perm, np.uint32, n)
        if counts is not None:
            _check_np("counts", counts, np.uint32, self.n_backends + 1)
        ticket = C.c_uint64(0)
        rc = lib.nbg_maglev_host_submit(self._h, ptrs.ctypes.data, lens.ctypes.data, n,
                                        NBG_SWAP_MACS if swap_macs else 0, backend.ctypes.data,
                                        None if perm is None else perm.ctypes.data,
                                        None if counts is None else counts.ctypes.data, C.byref(ticket))
        check(rc, "nbg_maglev_host_submit")
        t = ticket.value
        # the library reads ptrs/lens and writes the outputs until the batch completes: at its wait,
        # or when a later submit reuses its staging slot (NBG_HOST_SLOTS submits later)
        inflight = self.__dict__.setdefault("_inflight", {})
        for k in [k for k in inflight if k <= t - NBG_HOST_SLOTS]:
            del inflight[k]
        inflight[t] = (ptrs, lens, backend, perm, counts)
        return t

    def ring(self, *, stride: int = 64, frame_len: int = 60, swap_macs: bool = False, idle_ms: int = 2000,
             stream=None) -> "Ring":
        """Start this handle's persistent RX ring (nbg_ring_start): one classify kernel on `stream`
        (default: a new torch stream) that takes batches as they are posted until stop()."""
        return Ring(self, stride=stride, frame_len=frame_len, swap_macs=swap_macs, idle_ms=idle_ms, stream=stream)

    def use_host_ring(self, ring: Optional["HostRing"]) -> None:
        """nbg_maglev_set_host_ring: this handle's direct host batches (<= 2,048 packets) go to the
        device's host-batch server instead of a kernel launch each (None detaches)."""
        check(lib.nbg_maglev_set_host_ring(self._h, None if ring is None else ring._r), "nbg_maglev_set_host_ring")

    def host_query(self, ticket: int) -> bool:
        """nbg_maglev_host_query: True once batch `ticket` has finished on the GPU (non-blocking)."""
        done = C.c_int(0)
        check(lib.nbg_maglev_host_query(self._h, ticket, C.byref(done)), "nbg_maglev_host_query")
        return bool(done.value)

    def host_wait(self, ticket: int) -> None:
        check(lib.nbg_maglev_host_wait(self._h, ticket), "nbg_maglev_host_wait")
        self.__dict__.get("_inflight", {}).pop(ticket, None)

    def group_by_host(self, frames: Sequence[bytearray], swap_macs: bool = True, group: bool = True):
        """Host mbuf path: frames are mutable byte buffers (their MACs are swapped in place).
        Returns numpy (backend u16[n], perm u32[n] | None, counts u32[nb+1] | None)."""
        n = len(frames)
        keep = [(C.c_char * len(f)).from_buffer(f) if len(f) else (C.c_char * 1)() for f in frames]
        ptrs = (C.c_void_p * max(n, 1))(*[C.addressof(k) for k in keep])
        lens = np.array([len(f) for f in frames], dtype=np.uint16)
        backend = np.empty(max(n, 1), dtype=np.uint16)
        perm = np.empty(max(n, 1), dtype=np.uint32) if group else None
        counts = np.empty(self.n_backends + 1, dtype=np.uint32) if group else None
        flags = NBG_SWAP_MACS if swap_macs else 0
        rc = lib.nbg_maglev_classify_host(self._h, ptrs, lens.ctypes.data, n, flags, backend.ctypes.data,
                                          perm.ctypes.data if group else None,
                                          counts.ctypes.data if group else None)
        check(rc, "nbg_maglev_classify_host")
        return backend[:n], (perm[:n] if group else None), counts


class Ring:
    """A persistent RX ring (include/nbgpu.h, nbg_ring_*): one streaming-classify kernel that stays
    resident and classifies device-resident fixed-slot batches as they are posted (the RX queue that
    never stops, framework/src/operators/receive_batch.rs:26,52-61).  post() returns a ticket;
    wait(ticket) / poll() report completion, after which the batch's backend[] (and in-place swap)
    are in HBM.  The kernel runs on a private high-priority stream, ordered after `stream`'s earlier
    work, until stop() (or idle_ms without a post)."""

    def __init__(self, mg: "Maglev", *, stride: int, frame_len: int, swap_macs: bool, idle_ms: int, stream=None):
        import torch

        self._mg = mg
        self.stride, self.frame_len = stride, frame_len
        self._stream = stream if stream is not None else torch.cuda.Stream(torch.device("cuda", mg.device))
        st = self._stream.cuda_stream if hasattr(self._stream, "cuda_stream") else self._stream
        h = C.c_void_p()
        check(lib.nbg_ring_start(mg._h, stride, frame_len, NBG_SWAP_MACS if swap_macs else 0, idle_ms, st,
                                 C.byref(h)), "nbg_ring_start")
        self._r = h
        self._held = {}  # ticket -> tensors the kernel reads or writes until the batch is complete
        self._sizes = {}  # ticket -> n_pkts, for the last NBG_RING_SLOTS posts (group() checks perm)
        self._groups = []  # (event, tensors) of enqueued groupings, until their stream ran them
        self._queues = []
        mg._ring = self  # Maglev.close() stops the ring first (the handle frees it otherwise)

    def post(self, pkts, n_pkts: int, backend) -> int:
        import torch

        if self._r is None:
            raise RuntimeError("ring: stopped")
        dev = torch.device("cuda", self._mg.device)
        if pkts.dtype != torch.uint8 or not pkts.is_contiguous() or pkts.device != dev:
            raise ValueError(f"pkts: expected a contiguous uint8 tensor on {dev}")
        if n_pkts and pkts.numel() < (n_pkts - 1) * self.stride + _slot_tail(self.stride, self.frame_len):
            raise ValueError("pkts: too small for n_pkts slots")
        _check_dev("backend", backend, torch.uint16, n_pkts, dev)
        t = C.c_uint64()
        check(lib.nbg_ring_post(self._r, _ptr(pkts), n_pkts, _ptr(backend), C.byref(t)), "nbg_ring_post")
        self._held[t.value] = (pkts, backend)
        self._remember(t.value, n_pkts)
        return t.value

    def _remember(self, ticket: int, n_pkts: int) -> None:
        self._sizes[ticket] = n_pkts
        self._sizes.pop(ticket - _lib.NBG_RING_SLOTS, None)

    def post_burst(self, batches) -> tuple:
        """Post the first batches of `batches` ((pkts, n_pkts, backend) triples, an RX burst) without
        waiting for slots (nbg_ring_post_burst): returns (number posted, first ticket); the rest is
        for a later call."""
        import torch

        if self._r is None:
            raise RuntimeError("ring: stopped")
        dev = torch.device("cuda", self._mg.device)
        arr = (NbgRingBatch * max(len(batches), 1))()
        for i, (pkts, n_pkts, backend) in enumerate(batches):
            if pkts.dtype != torch.uint8 or not pkts.is_contiguous() or pkts.device != dev:
                raise ValueError(f"pkts: expected a contiguous uint8 tensor on {dev}")
            if n_pkts and pkts.numel() < (n_pkts - 1) * self.stride + _slot_tail(self.stride, self.frame_len):
                raise ValueError("pkts: too small for n_pkts slots")
            _check_dev("backend", backend, torch.uint16, n_pkts, dev)
            arr[i] = NbgRingBatch(_ptr(pkts), n_pkts, _ptr(backend))
        k, t = C.c_uint32(), C.c_uint64()
        check(lib.nbg_ring_post_burst(self._r, arr, len(batches), C.byref(k), C.byref(t)), "nbg_ring_post_burst")
        for i in range(k.value):
            self._held[t.value + i] = (batches[i][0], batches[i][2])
            self._remember(t.value + i, batches[i][1])
        return k.value, t.value

    def group(self, ticket: int, perm, counts, stream=None) -> None:
        """perm / counts of batch `ticket` (nbg_ring_group) on `stream` (default: torch's current
        stream).  The batch need not be complete: a gate kernel on the stream waits for it, so the
        grouping can be enqueued right after the post.  The tensors are held until the stream has run
        the grouping."""
        import torch

        if self._r is None:
            raise RuntimeError("ring: stopped")
        dev = torch.device("cuda", self._mg.device)
        _check_dev("perm", perm, torch.uint32, self._sizes.get(ticket, 0), dev)
        _check_dev("counts", counts, torch.uint32, self._mg.n_backends + 1, dev)
        st = stream if stream is not None else torch.cuda.current_stream(dev)
        check(lib.nbg_ring_group(self._r, ticket, _ptr(perm), _ptr(counts), _stream_ptr(st)), "nbg_ring_group")
        _hold_until_run(self._groups, st, dev, (self._held.get(ticket), perm, counts))

    def poll(self) -> int:
        c = C.c_uint64()
        check(lib.nbg_ring_poll(self._r, C.byref(c)), "nbg_ring_poll")
        for k in [k for k in self._held if k < c.value]:
            del self._held[k]
        return c.value

    def wait(self, ticket: int, timeout_ms: int = 10000) -> None:
        check(lib.nbg_ring_wait(self._r, ticket, timeout_ms), "nbg_ring_wait")
        for k in [k for k in self._held if k <= ticket]:
            del self._held[k]

    def group_burst(self, first: int, perms, counts, stream=None) -> None:
        """perm / counts of the len(perms) consecutive batches first.. (nbg_ring_group_burst: one gate,
        one hist and one group launch for all of them)."""
        import torch

        if self._r is None:
            raise RuntimeError("ring: stopped")
        n = len(perms)
        if n != len(counts) or not 1 <= n <= NBG_MAX_MULTI:
            raise ValueError(f"perms / counts: 1..{NBG_MAX_MULTI} batches each")
        dev = torch.device("cuda", self._mg.device)
        for j in range(n):
            _check_dev("perm", perms[j], torch.uint32, self._sizes.get(first + j, 0), dev)
            _check_dev("counts", counts[j], torch.uint32, self._mg.n_backends + 1, dev)
        pa = (C.c_void_p * n)(*[_ptr(p) for p in perms])
        ca = (C.c_void_p * n)(*[_ptr(c) for c in counts])
        st = stream if stream is not None else torch.cuda.current_stream(dev)
        check(lib.nbg_ring_group_burst(self._r, first, n, pa, ca, _stream_ptr(st)), "nbg_ring_group_burst")
        _hold_until_run(self._groups, st, dev, ([self._held.get(first + j) for j in range(n)], list(perms),
                                                list(counts)))

    def queue(self) -> "RingQueue":
        """Open an RX queue on this ring (nbg_ring_queue_open): its own tickets, completion and grouping
        over the shared ring (one pipeline per RSS queue, scheduler/context.rs:241-255)."""
        if self._r is None:
            raise RuntimeError("ring: stopped")
        q = RingQueue(self)
        self._queues.append(q)
        return q

    def stop(self) -> None:
        """nbg_ring_stop: every posted batch completes, the kernel ends, the ring's queues close.  The
        tensors the kernel reads or writes are released only once it has ended; if the stop times out
        (the kernel may still run) they are parked for the life of the process."""
        if self._r is not None:
            r, self._r = self._r, None
            self._mg.__dict__.pop("_ring", None)
            rc = lib.nbg_ring_stop(r)
            keep = (self._held, self._groups, [q._held for q in self._queues])
            for q in self._queues:
                q._q = None
            if rc == _lib.NBG_EBUSY:
                _LEAKED.append(keep)  # the kernel did not end: never hand its memory back to torch
            else:
                self._held = {}
                self._groups = []
            check(rc, "nbg_ring_stop")

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.stop()

    def __del__(self):
        try:
            self.stop()
        except Exception:  # noqa: BLE001 (interpreter teardown)
            pass


_LEAKED = []  # tensors of rings whose kernel did not end at stop (never returned to torch's allocator)


def _stream_ptr(st):
    return st.cuda_stream if hasattr(st, "cuda_stream") else st


def _hold_until_run(groups: list, st, dev, refs) -> None:
    """Keep `refs` alive until the work just enqueued on stream `st` has run (an event behind it),
    pruning entries whose event has passed."""
    import torch

    while groups and groups[0][0].query():
        groups.pop(0)
    ev = torch.cuda.Event()
    if hasattr(st, "cuda_stream"):
        ev.record(st)
    else:
        ev.record(torch.cuda.ExternalStream(st, device=dev))
    groups.append((ev, refs))


class RingQueue:
    """One RX queue on a device's ring (nbg_ring_queue_*): its own tickets 0, 1, 2, ..., completion and
    grouping; the batches of every queue of the ring share its slots in post order.  One thread per
    queue; queues of one ring may post from different threads."""

    def __init__(self, ring: "Ring"):
        self._ring = ring
        h = C.c_void_p()
        check(lib.nbg_ring_queue_open(ring._r, C.byref(h)), "nbg_ring_queue_open")
        self._q = h
        self._held = {}
        self._sizes = {}
        self._groups = []

    def post(self, pkts, n_pkts: int, backend) -> int:
        import torch

        if self._q is None:
            raise RuntimeError("ring queue: closed")
        r = self._ring
        dev = torch.device("cuda", r._mg.device)
        if pkts.dtype != torch.uint8 or not pkts.is_contiguous() or pkts.device != dev:
            raise ValueError(f"pkts: expected a contiguous uint8 tensor on {dev}")
        if n_pkts and pkts.numel() < (n_pkts - 1) * r.stride + _slot_tail(r.stride, r.frame_len):
            raise ValueError("pkts: too small for n_pkts slots")
        _check_dev("backend", backend, torch.uint16, n_pkts, dev)
        t = C.c_uint64()
        check(lib.nbg_ring_queue_post(self._q, _ptr(pkts), n_pkts, _ptr(backend), C.byref(t)), "nbg_ring_queue_post")
        self._held[t.value] = (pkts, backend)
        self._sizes[t.value] = n_pkts
        self._sizes.pop(t.value - _lib.NBG_RING_SLOTS, None)
        return t.value

    def poll(self) -> int:
        c = C.c_uint64()
        check(lib.nbg_ring_queue_poll(self._q, C.byref(c)), "nbg_ring_queue_poll")
        for k in [k for k in self._held if k < c.value]:
            del self._held[k]
        return c.value

    def wait(self, ticket: int, timeout_ms: int = 10000) -> None:
        check(lib.nbg_ring_queue_wait(self._q, ticket, timeout_ms), "nbg_ring_queue_wait")
        for k in [k for k in self._held if k <= ticket]:
            del self._held[k]

    def group(self, ticket: int, perm, counts, stream=None) -> None:
        import torch

        if self._q is None:
            raise RuntimeError("ring queue: closed")
        dev = torch.device("cuda", self._ring._mg.device)
        _check_dev("perm", perm, torch.uint32, self._sizes.get(ticket, 0), dev)
        _check_dev("counts", counts, torch.uint32, self._ring._mg.n_backends + 1, dev)
        st = stream if stream is not None else torch.cuda.current_stream(dev)
        check(lib.nbg_ring_queue_group(self._q, ticket, _ptr(perm), _ptr(counts), _stream_ptr(st)),
              "nbg_ring_queue_group")
        _hold_until_run(self._groups, st, dev, (self._held.get(ticket), perm, counts))

    def close(self) -> None:
        if self._q is not None:
            q, self._q = self._q, None
            check(lib.nbg_ring_queue_close(q), "nbg_ring_queue_close")


class HostRing:
    """The device's host-batch server (nbg_host_ring_*): one persistent kernel whose blocks classify and
    group the direct host batches of every attached handle (Maglev.use_host_ring) without a kernel
    launch per batch.  stop() ends it once every posted batch is done (handles detached first)."""

    def __init__(self, device: int = 0, blocks: int = 0, idle_ms: int = 2000):
        h = C.c_void_p()
        check(lib.nbg_host_ring_start(device, blocks, idle_ms, C.byref(h)), "nbg_host_ring_start")
        self._r = h
        self.device = device

    def stop(self) -> None:
        if self._r is not None:
            r, self._r = self._r, None
            rc = lib.nbg_host_ring_stop(r)
            if rc == _lib.NBG_EBUSY and "still use it" in _lib.last_error():
                self._r = r  # handles attached: nothing was stopped
            check(rc, "nbg_host_ring_stop")

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.stop()


class HostRegion:
    """A host memory region registered for zero-copy GPU access (nbg_host_register): the GPU reads
    frames out of it and writes the MAC swap back over PCIe.  `array` is a writable, C-contiguous
    numpy uint8 array (e.g. an mbuf pool); keep it alive while registered.  Offsets into it are u32,
    so the region must stay below 4 GiB."""

    def __init__(self, array: np.ndarray, device: int = 0):
        if array.dtype != np.uint8 or not array.flags.c_contiguous or not array.flags.writeable:
            raise ValueError("array: expected a writable C-contiguous uint8 numpy array")
        if array.nbytes == 0 or array.nbytes > (1 << 32):
            raise ValueError("array: 1 B .. 4 GiB")
        self.array = array
        self.device = device
        d = C.c_void_p()
        check(lib.nbg_host_register(array.ctypes.data, array.nbytes, device, C.byref(d)), "nbg_host_register")
        self.dev_ptr = d.value

    def close(self) -> None:
        if self.dev_ptr is not None:
            self.dev_ptr = None
            check(lib.nbg_host_unregister(self.array.ctypes.data, self.device), "nbg_host_unregister")

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
