"""The compact group kernel (group_direct_kernel: wave-segment ranks and direct perm stores, 28 KB of
LDS at 1001 bins) that the library takes for many bins while a persistent ring runs on the device.
nbg_debug_set_group_compact(1) forces it for every grouping; each case is bit-exact against the C oracle's
per-group FIFO order (operators/group_by.rs:46-51): few and many bins, partitions of one and of many
4096-packet chunks, rows summed in the group kernel and from scan_kernel, multi-batch launches, and
counts only."""
import numpy as np
import pytest

import orc

pytestmark = pytest.mark.gpu


@pytest.fixture
def compact():
    from netbricks_amd._lib import lib

    assert lib.nbg_debug_set_group_compact(1) == 0  # every grouping takes the compact kernel
    yield
    assert lib.nbg_debug_set_group_compact(-1) == 0  # back to the library's rule


def _names(k):
    return [f"be{i}" for i in range(k)]


def _check(torch, r, be_exp, nb_, n):
    perm, counts = orc.group(be_exp, nb_)
    np.testing.assert_array_equal(r.backend.view(torch.int16).cpu().numpy().view(np.uint16)[:n], be_exp)
    np.testing.assert_array_equal(r.counts.view(torch.int32).cpu().numpy().view(np.uint32), counts)
    if r.perm is not None:
        np.testing.assert_array_equal(r.perm.view(torch.int32).cpu().numpy().view(np.uint32)[:n], perm)


@pytest.mark.parametrize("nb_,m,n", [(65, 65537, 1 << 20), (65, 65537, 3 << 20), (1000, 655373, 300000),
                                     (1000, 655373, 9000), (300, 65537, 1 << 20), (1, 7, 5000)])
def test_compact_group_fixed_slots(torch_cuda, compact, nb_, m, n):
    import netbricks_amd as nb

    torch = torch_cuda
    mg = nb.Maglev(_names(nb_), m)
    buf = nb.make_trace(n, 0, seed=n + nb_)[0]
    d = torch.from_numpy(buf.copy()).cuda()
    r = mg.group_by(d, n, swap_macs=False)
    torch.cuda.synchronize()
    mg.check()
    _check(torch, r, orc.classify(buf.copy(), n, orc.lut_build(_names(nb_), m), swap=False), nb_, n)
    mg.close()


def test_compact_group_desc_multi_c3(torch_cuda, compact):
    """C3's shape through the descriptor multi path (hist + scan + group over three batches)."""
    import netbricks_amd as nb

    torch = torch_cuda
    mg = nb.Maglev(_names(1000), 655373)
    lut = orc.lut_build(_names(1000), 655373)
    batches, traces = [], []
    for j, n in enumerate((1 << 20, 70000, 1)):
        buf, off, ln = nb.make_trace(n, 1, seed=900 + j)
        traces.append((buf, off, ln, n))
        batches.append((torch.from_numpy(buf.copy()).cuda(),
                        torch.from_numpy(off.view(np.int32)).cuda().view(torch.uint32),
                        torch.from_numpy(ln.view(np.int16)).cuda().view(torch.uint16), n))
    res = mg.group_by_desc_multi(batches, swap_macs=False)
    torch.cuda.synchronize()
    mg.check()
    for (buf, off, ln, n), r in zip(traces, res):
        _check(torch, r, orc.classify(buf.copy(), n, lut, offs=off, lens=ln, swap=False), 1000, n)
    mg.close()


def test_compact_group_multi_and_counts_only(torch_cuda, compact):
    """Fixed-slot multi-batch launches (per-batch outputs) and a counts-only call."""
    import netbricks_amd as nb

    torch = torch_cuda
    names = _names(65)
    mg = nb.Maglev(names, 65537)
    lut = orc.lut_build(names, 65537)
    bufs = [nb.make_trace(n, 0, seed=77 + n)[0] for n in (262144, 300000, 4096)]
    ds = [torch.from_numpy(b.copy()).cuda() for b in bufs]
    res = mg.group_by_multi([(d, b.size // 64) for d, b in zip(ds, bufs)], swap_macs=False)
    torch.cuda.synchronize()
    for b, r in zip(bufs, res):
        n = b.size // 64
        _check(torch, r, orc.classify(b.copy(), n, lut, swap=False), 65, n)
    n = 1 << 20
    buf = nb.make_trace(n, 0, seed=5)[0]
    r = mg.group_by(torch.from_numpy(buf.copy()).cuda(), n, swap_macs=False, scatter=False)
    torch.cuda.synchronize()
    _check(torch, r, orc.classify(buf.copy(), n, lut, swap=False), 65, n)
    mg.close()
