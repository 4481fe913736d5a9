"""A call captured in a hipGraph (here through torch.cuda.graph) replays bit-exactly, any number
of times, with direct calls on the same handle interleaved.  Only the single-launch small path
(<= 2048 packets) can be captured: it keeps no state across calls.  Larger batches are refused
while capturing.
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


@pytest.mark.parametrize("n", [32, 1000, 2048])
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


@pytest.mark.parametrize("n", [2049, 1 << 20])
def test_graph_capture_refused_above_small_path(torch_cuda, n):
    """Multi-launch batches are refused while capturing (a clear error, nothing captured)."""
    torch = torch_cuda
    import netbricks_amd as nb

    mg = nb.Maglev(NAMES65, 65537)
    d = torch.from_numpy(nb.make_trace(n, 0, seed=5)[0]).cuda()
    og = _outs(torch, n)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    C = __import__("ctypes")
    hip = C.CDLL("libamdhip64.so.7")
    assert hip.hipStreamBeginCapture(C.c_void_p(s.cuda_stream), C.c_int(2)) == 0  # thread-local mode
    with pytest.raises(nb.NbgError):
        mg.group_by(d, n, stream=s.cuda_stream, **og)
    g = C.c_void_p()
    assert hip.hipStreamEndCapture(C.c_void_p(s.cuda_stream), C.byref(g)) == 0
    hip.hipGraphDestroy(g)
    mg.close()
