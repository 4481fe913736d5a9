"""Ordering of a handle's work across streams, and the library's independence from the legacy
null stream.

A handle's kernels share its scratch (ping-pong partition histograms), so consecutive calls on
different streams must still run in call order (nbg_maglev_finish_group on another stream than
its classify, NBG_DEFER_GROUP; a handle moved between streams).  Setup work (LUT upload,
histogram zeroing, staging-buffer zeroing) must never go through the null stream: a hipMemset
there returns before it runs and is not ordered with non-blocking streams — the cause of the
round-1 host-path reads of zeroed staging windows (tools/memset_probe.py).
Reference semantics of every output: test/maglev/src/nf.rs:92-108, operators/group_by.rs:43-55.
"""
import ctypes as C

import numpy as np
import pytest

import orc

pytestmark = pytest.mark.gpu

NAMES65 = [f"backend-{i}" for i in range(65)]


def _u16(t, torch):
    return t.view(torch.int16).cpu().numpy().view(np.uint16)


def _u32(t, torch):
    return t.view(torch.int32).cpu().numpy().view(np.uint32)


def _busy(torch, stream, iters):
    """Queue ~iters ms of matmuls on `stream`; returns the event recorded after them."""
    x = torch.randn(4096, 4096, device="cuda:0")
    with torch.cuda.stream(stream):
        for _ in range(iters):
            x = x @ x
            x = x / x.norm()
        ev = torch.cuda.Event()
        ev.record(stream)
    return ev, x


def test_defer_group_on_other_stream(torch_cuda):
    """classify (NBG_DEFER_GROUP) on stream A, finish_group on stream B, back to back over many
    batches with no host synchronisation: every batch's grouping sees its own histograms."""
    torch = torch_cuda
    import netbricks_amd as nb

    lut = orc.lut_build(NAMES65, 65537)
    mg = nb.Maglev(NAMES65, 65537)
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    sizes = [70000, 1, 4096, 300000, 5000, 65536 + 13, 200000, 64, 123457, 9999] * 2
    bufs = [nb.make_trace(n, 0, seed=900 + k)[0] for k, n in enumerate(sizes)]
    ins = [torch.from_numpy(x.copy()).cuda() for x in bufs]
    torch.cuda.synchronize()
    outs = []
    for k, n in enumerate(sizes):
        r = mg.group_by(ins[k], n, defer_group=True, stream=a.cuda_stream)
        mg.finish_group(b.cuda_stream)
        outs.append(r)
    torch.cuda.synchronize()
    mg.check()
    for k, n in enumerate(sizes):
        ref = bufs[k].copy()
        be = orc.classify(ref, n, lut, stride=64, fixed_len=60)
        perm, counts = orc.group(be, 65)
        np.testing.assert_array_equal(_u16(outs[k].backend, torch), be)
        np.testing.assert_array_equal(_u32(outs[k].counts, torch), counts)
        np.testing.assert_array_equal(_u32(outs[k].perm, torch)[:n], perm)
        np.testing.assert_array_equal(ins[k].cpu().numpy(), ref)
    mg.close()


def test_handle_moves_between_streams(torch_cuda):
    """One handle used on a different stream every call (with a busy kernel chain on one of them,
    so a later call on another stream would overtake it if unordered)."""
    torch = torch_cuda
    import netbricks_amd as nb

    lut = orc.lut_build(NAMES65, 65537)
    mg = nb.Maglev(NAMES65, 65537)
    streams = [torch.cuda.Stream() for _ in range(3)]
    n = 150000
    bufs = [nb.make_trace(n, 0, seed=950 + k)[0] for k in range(9)]
    ins = [torch.from_numpy(x.copy()).cuda() for x in bufs]
    torch.cuda.synchronize()
    outs, keep = [], []
    for k in range(9):
        s = streams[k % 3]
        if k % 3 == 0:
            keep.append(_busy(torch, s, 10))  # this stream lags: the next call's stream must wait for it
        outs.append(mg.group_by(ins[k], n, stream=s.cuda_stream))
    torch.cuda.synchronize()
    mg.check()
    for k in range(9):
        ref = bufs[k].copy()
        be = orc.classify(ref, n, lut, stride=64, fixed_len=60)
        perm, counts = orc.group(be, 65)
        np.testing.assert_array_equal(_u16(outs[k].backend, torch), be)
        np.testing.assert_array_equal(_u32(outs[k].counts, torch), counts)
        np.testing.assert_array_equal(_u32(outs[k].perm, torch)[:n], perm)
    mg.close()


def test_hip_null_stream_memset_is_unordered(torch_cuda):
    """Characterises the HIP behaviour behind the round-1 stale staging windows: with the null
    stream busy, hipMemset returns at once and runs later, after (and over) a copy a non-blocking
    stream made in the meantime."""
    torch = torch_cuda
    hip = C.CDLL("libamdhip64.so.7")
    s = C.c_void_p()
    assert hip.hipStreamCreateWithFlags(C.byref(s), C.c_uint(1)) == 0
    size = 1 << 20
    buf = C.c_void_p()
    assert hip.hipMalloc(C.byref(buf), C.c_size_t(size)) == 0
    src = np.full(size, 0xAB, dtype=np.uint8)
    torch.cuda.synchronize()
    assert torch.cuda.current_stream().cuda_stream == 0
    ev, keep = _busy(torch, torch.cuda.current_stream(), 30)
    assert hip.hipMemset(buf, C.c_int(0), C.c_size_t(size)) == 0
    assert hip.hipMemcpyAsync(buf, src.ctypes.data_as(C.c_void_p), C.c_size_t(size), C.c_int(1), s) == 0
    assert hip.hipStreamSynchronize(s) == 0
    copy_before_memset = not ev.query()
    torch.cuda.synchronize()
    out = np.empty(size, dtype=np.uint8)
    assert hip.hipMemcpy(out.ctypes.data_as(C.c_void_p), buf, C.c_size_t(size), C.c_int(2)) == 0
    hip.hipFree(buf)
    hip.hipStreamDestroy(s)
    assert copy_before_memset  # the copy finished while the null stream was still busy
    assert (out == 0).all()    # ... and the memset ran after it, over the copied bytes


def test_results_with_gated_null_stream(torch_cuda):
    """With the legacy null stream blocked behind a kernel chain of another stream, a new Maglev
    handle, an LPM handle, device batches and pipelined host batches (first use of each staging
    slot allocates and zeroes it) all give the oracle's results: the library's setup work is done
    (or stream-ordered) before it is used, whatever the null stream is doing.  Progress is not
    asserted: a stream created after the process holds more streams than GPU_MAX_HW_QUEUES (4)
    shares a hardware queue with another stream and can wait behind that queue's barrier."""
    torch = torch_cuda
    import netbricks_amd as nb
    from netbricks_amd.lpm import Lpm

    lut = orc.lut_build(NAMES65, 65537)
    n = 100000
    buf, _, _ = nb.make_trace(n, 0, seed=77)
    pin = torch.from_numpy(buf.copy()).pin_memory()
    d = torch.empty(n * 64, dtype=torch.uint8, device="cuda:0")
    s = torch.cuda.Stream()
    sizes = [3000, 100, 40000, 1, 3000, 777]
    hbufs = [nb.make_trace(k, 1, seed=300 + j) for j, k in enumerate(sizes)]
    torch.cuda.synchronize()
    g = torch.cuda.Stream()
    gate, keep = _busy(torch, g, 400)
    torch.cuda.current_stream().wait_event(gate)  # the null stream waits for the chain
    mg = nb.Maglev(NAMES65, 65537)
    lpm = Lpm([("10.0.0.0", 8, 1)])
    with torch.cuda.stream(s):  # (a pageable torch copy would itself wait for the null stream)
        d.copy_(pin, non_blocking=True)
    r = mg.group_by(d, n, stream=s.cuda_stream)
    pending = []
    for j, (hb, off, ln) in enumerate(hbufs):
        frames = [bytearray(hb[o:o + l].tobytes()) for o, l in zip(off.tolist(), ln.tolist())]
        ptrs = np.array([C.addressof((C.c_char * len(f)).from_buffer(f)) for f in frames], dtype=np.uint64)
        lens = np.array([len(f) for f in frames], dtype=np.uint16)
        out = dict(backend=np.empty(len(frames), np.uint16), perm=np.empty(len(frames), np.uint32),
                   counts=np.empty(66, np.uint32))
        pending.append((mg.host_submit(ptrs, lens, **out), frames, out, hb, off, ln))
    for t, *_ in pending:
        mg.host_wait(t)
    torch.cuda.synchronize()
    ref = buf.copy()
    be = orc.classify(ref, n, lut, stride=64, fixed_len=60)
    perm, counts = orc.group(be, 65)
    np.testing.assert_array_equal(_u16(r.backend, torch), be)
    np.testing.assert_array_equal(_u32(r.perm, torch)[:n], perm)
    np.testing.assert_array_equal(_u32(r.counts, torch), counts)
    for t, frames, out, hb, off, ln in pending:
        ref = hb.copy()
        ebe = orc.classify(ref, len(frames), lut, offs=off, lens=ln)
        eperm, ecnt = orc.group(ebe, 65)
        np.testing.assert_array_equal(out["backend"], ebe)
        np.testing.assert_array_equal(out["perm"], eperm)
        np.testing.assert_array_equal(out["counts"], ecnt)
        for f, o, l in zip(frames, off.tolist(), ln.tolist()):
            assert bytes(f) == ref[o:o + l].tobytes()
    mg.close()
    lpm.close()
