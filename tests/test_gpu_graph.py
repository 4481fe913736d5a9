"""A call captured in a hipGraph (here through torch.cuda.graph, replayed on torch's default stream:
the legacy null stream) replays bit-exactly, any number of times, with direct calls on the same
handle interleaved: the single-launch small path and multi-launch batches alike (round 3: captured
calls zero their partition rows with a kernel node; a memset node faulted on replay under
PyTorch's HIP 7.0 runtime on the null stream).  Calls whose scratch grows on demand
(NBG_LUT_TILED, descriptor batches without lengths above the small path) are refused while capturing.
Reference semantics: test/maglev/src/nf.rs:92-108, operators/group_by.rs:43-55."""
import numpy as np
import pytest

import orc

pytestmark = pytest.mark.gpu

NAMES65 = [f"backend-{i}" for i in range(65)]


def _outs(torch, n):
    return dict(backend=torch.empty(n, dtype=torch.uint16, device="cuda"),
                perm=torch.empty(n, dtype=torch.uint32, device="cuda"),
                counts=torch.empty(66, dtype=torch.uint32, device="cuda"),
                mac_out=torch.empty(n * 12, dtype=torch.uint8, device="cuda"))


def _check(torch, outs, exp, n):
    be, perm, counts, rec = exp
    np.testing.assert_array_equal(outs["backend"].view(torch.int16).cpu().numpy().view(np.uint16), be)
    np.testing.assert_array_equal(outs["perm"].view(torch.int32).cpu().numpy().view(np.uint32)[:n], perm)
    np.testing.assert_array_equal(outs["counts"].view(torch.int32).cpu().numpy().view(np.uint32), counts)
    np.testing.assert_array_equal(outs["mac_out"].cpu().numpy().reshape(n, 12), rec)


def _oracle(buf, n, lut):
    ref = buf.copy()
    be = orc.classify(ref, n, lut, stride=64, fixed_len=60)
    perm, counts = orc.group(be, 65)
    return be, perm, counts, ref.reshape(n, 64)[:, :12]  # the swapped MACs = the egress records


@pytest.mark.parametrize("n", [32, 1000, 2048, 2049, 16384, 300000, 1 << 20])
def test_graph_replay_with_direct_calls(torch_cuda, n):
    torch = torch_cuda
    import netbricks_amd as nb

    lut = orc.lut_build(NAMES65, 65537)
    mg = nb.Maglev(NAMES65, 65537)
    bufs = [nb.make_trace(n, 0, seed=70 + k)[0] for k in range(2)]
    d = [torch.from_numpy(b.copy()).cuda() for b in bufs]
    exp = [_oracle(b, n, lut) for b in bufs]
    og, od = _outs(torch, n), _outs(torch, n)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):  # warm-up outside the capture (first-call attributes, allocations)
        mg.group_by(d[0], n, stream=side.cuda_stream, **og)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        mg.group_by(d[0], n, **og)
    for rep in range(3):
        for o in og.values():
            o.zero_()
        g.replay()
        torch.cuda.synchronize()
        _check(torch, og, exp[0], n)
        # a direct call on another batch between replays: the ping-pong histograms stay consistent
        mg.group_by(d[1], n, **od)
        torch.cuda.synchronize()
        mg.check()
        _check(torch, od, exp[1], n)
    mg.close()


def test_graph_replay_c3_descriptors(torch_cuda):
    """A multi-launch C3-shaped batch (IMIX descriptors with lengths, 1000 backends, u16 LUT:
    classify + hist + scan + group) captured and replayed against direct calls, records mode."""
    torch = torch_cuda
    import netbricks_amd as nb

    names = [f"be{i}" for i in range(1000)]
    mg = nb.Maglev(names, 655373)
    lut = orc.lut_build(names, 655373)
    n = 300000
    buf, off, ln = nb.make_trace(n, 1, seed=1001)
    ref = buf.copy()
    be = orc.classify(ref, n, lut, offs=off, lens=ln)
    perm, counts = orc.group(be, 1000)
    d = torch.from_numpy(buf.copy()).cuda()
    d_off = torch.from_numpy(off.view(np.int32)).cuda().view(torch.uint32)
    d_len = torch.from_numpy(ln.view(np.int16)).cuda().view(torch.uint16)
    outs = dict(backend=torch.empty(n, dtype=torch.uint16, device="cuda"),
                perm=torch.empty(n, dtype=torch.uint32, device="cuda"),
                counts=torch.empty(1001, dtype=torch.uint32, device="cuda"),
                mac_out=torch.empty(n * 12, dtype=torch.uint8, device="cuda"))
    kw = dict(offsets=d_off, lens=d_len, owned_windows=True, **outs)
    mg.group_by(d, n, **kw)  # warm-up (first-call attributes)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        mg.group_by(d, n, **kw)
    for rep in range(3):
        for o in outs.values():
            o.zero_()
        (g.replay if rep % 2 == 0 else (lambda: mg.group_by(d, n, **kw)))()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(outs["backend"].view(torch.int16).cpu().numpy().view(np.uint16), be)
        np.testing.assert_array_equal(outs["perm"].view(torch.int32).cpu().numpy().view(np.uint32), perm)
        np.testing.assert_array_equal(outs["counts"].view(torch.int32).cpu().numpy().view(np.uint32), counts)
    mg.check()
    mg.close()


def _refused_in_capture(torch, mg, nb, call):
    s = torch.cuda.Stream()
    C = __import__("ctypes")
    hip = C.CDLL("libamdhip64.so.7")
    assert hip.hipStreamBeginCapture(C.c_void_p(s.cuda_stream), C.c_int(2)) == 0  # thread-local mode
    with pytest.raises(nb.NbgError):
        call(s.cuda_stream)
    g = C.c_void_p()
    assert hip.hipStreamEndCapture(C.c_void_p(s.cuda_stream), C.byref(g)) == 0
    hip.hipGraphDestroy(g)


def test_graph_capture_refused_for_growing_scratch(torch_cuda):
    """NBG_LUT_TILED and descriptor batches without lengths above the small path use scratch that a
    later eager call may reallocate: refused while capturing (a clear error, nothing captured)."""
    torch = torch_cuda
    import netbricks_amd as nb

    names = [f"be{i}" for i in range(1000)]
    mg = nb.Maglev(names, 655373)
    n = 4096
    buf, off, ln = nb.make_trace(n, 1, seed=5)
    d = torch.from_numpy(buf).cuda()
    d_off = torch.from_numpy(off.view(np.int32)).cuda().view(torch.uint32)
    d_len = torch.from_numpy(ln.view(np.int16)).cuda().view(torch.uint16)
    torch.cuda.synchronize()
    _refused_in_capture(torch, mg, nb, lambda st: mg.group_by(d, n, offsets=d_off, lens=d_len, owned_windows=True,
                                                              lut_tiled=True, stream=st))
    _refused_in_capture(torch, mg, nb, lambda st: mg.group_by(d, n, offsets=d_off, frame_len=60,
                                                              owned_windows=True, stream=st))
    mg.close()
