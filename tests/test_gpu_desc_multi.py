"""GPU parity of the multi-batch descriptor path (nbg_maglev_classify_desc_multi,
nbg_chain_lpm_maglev_multi): several IMIX batches (u32 offset + u16 length per packet, configs C3 and
C5) in one launch of each kernel.  Every batch's outputs are bit-exact against the C oracle run on that
batch alone: backend[], the MAC-swapped bytes, the per-group FIFO order (perm) and the group sizes, and
for the chain the lpm gate (test/maglev/src/nf.rs:92-106, test/lpm/src/nf.rs:212-228).
"""
import ctypes as C
import json
import os
import time

import numpy as np
import pytest

import orc

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROUTES = json.load(open(os.path.join(ROOT, "tests", "golden", "lpm_routes.json")))
NAMES65 = [f"backend-{i}" for i in range(65)]
NAMES1000 = [f"be{i}" for i in range(1000)]


def _dev_batch(torch, buf, off, ln, n):
    d = torch.from_numpy(buf.copy()).cuda()
    o = torch.from_numpy(np.ascontiguousarray(off, dtype=np.uint32).view(np.int32)).cuda().view(torch.uint32)
    ln = torch.from_numpy(np.ascontiguousarray(ln, dtype=np.uint16).view(np.int16)).cuda().view(torch.uint16)
    return d, o, ln, n


def _np16(t, n):
    import torch

    return t.view(torch.int16).cpu().numpy().view(np.uint16)[:n]


def _np32(t, n=None):
    import torch

    a = t.view(torch.int32).cpu().numpy().view(np.uint32)
    return a if n is None else a[:n]


def _traces(sizes, seed):
    import netbricks_amd as nb

    out = []
    for j, n in enumerate(sizes):
        buf, off, ln = nb.make_trace(max(n, 1), 1, seed=seed + j)
        out.append((buf, off[:n].copy(), ln[:n].copy(), n))
    return out


def _check_maglev(torch, mg, traces, results, dbatches, lut, nb_, swap=True):
    for (buf, off, ln, n), r, db in zip(traces, results, dbatches):
        ref = buf.copy()
        be = orc.classify(ref, n, lut, offs=off, lens=ln, swap=swap) if n else np.zeros(0, np.uint16)
        perm, counts = orc.group(be, nb_)
        np.testing.assert_array_equal(_np16(r.backend, n), be)
        np.testing.assert_array_equal(_np32(r.counts), counts)
        np.testing.assert_array_equal(_np32(r.perm, n), perm)
        np.testing.assert_array_equal(db[0].cpu().numpy(), ref)


@pytest.mark.parametrize("owned", [False, True])
@pytest.mark.parametrize("sizes", [[262161, 0, 1, 5000, 70000], [1 << 20, 1 << 20], [7, 64, 65, 255, 256, 257, 4097, 3]])
def test_desc_multi_c3(torch_cuda, sizes, owned):
    """Config C3's shape (1000 backends, M = 655373: hist + scan + group over all batches), ragged
    batches including an empty one, in-place MAC swap: only the frame's bytes rewritten, or
    (owned=True, NBG_OWNED_WINDOWS, the mode bench.py times) whole 64-B windows."""
    from netbricks_amd import Maglev

    torch = torch_cuda
    mg = Maglev(NAMES1000, 655373)
    lut = orc.lut_build(NAMES1000, 655373)
    tr = _traces(sizes, seed=3000 + len(sizes))
    dbs = [_dev_batch(torch, *t) for t in tr]
    res = mg.group_by_desc_multi(dbs, owned_windows=owned)
    torch.cuda.synchronize()
    mg.check()
    _check_maglev(torch, mg, tr, res, dbs, lut, 1000)
    mg.close()


def test_desc_multi_few_backends_consecutive(torch_cuda):
    """65 backends (partition rows from the classify kernel, zeroed by the previous call's group
    launch): three consecutive multi calls, read only and in place, and a fixed-slot multi call on
    the same handle in between (the two multi paths share the handle's partition-row sets)."""
    from netbricks_amd import Maglev, make_trace

    torch = torch_cuda
    mg = Maglev(NAMES65, 65537)
    lut = orc.lut_build(NAMES65, 65537)
    for call, swap in enumerate((True, False, True)):
        tr = _traces([300000, 1, 0, 99999], seed=4000 + 10 * call)
        dbs = [_dev_batch(torch, *t) for t in tr]
        res = mg.group_by_desc_multi(dbs, swap_macs=swap)
        torch.cuda.synchronize()
        mg.check()
        _check_maglev(torch, mg, tr, res, dbs, lut, 65, swap=swap)
        # fixed 64-B slots through nbg_maglev_classify_device_multi on the same handle
        n = 262144
        buf, _, _ = make_trace(n, 0, seed=4100 + call)
        d = torch.from_numpy(buf.copy()).cuda()
        (g,) = mg.group_by_multi([(d, n)])
        torch.cuda.synchronize()
        ref = buf.copy()
        be = orc.classify(ref, n, lut)
        perm, counts = orc.group(be, 65)
        np.testing.assert_array_equal(_np16(g.backend, n), be)
        np.testing.assert_array_equal(_np32(g.counts), counts)
        np.testing.assert_array_equal(_np32(g.perm, n), perm)
    mg.close()


def test_desc_multi_defer_group_other_stream(torch_cuda):
    """NBG_DEFER_GROUP: classify on one stream, the hist + scan + group launches of all batches by
    finish_group on another."""
    from netbricks_amd import Maglev

    torch = torch_cuda
    mg = Maglev(NAMES1000, 655373)
    lut = orc.lut_build(NAMES1000, 655373)
    tr = _traces([200000, 131072, 1], seed=5000)
    dbs = [_dev_batch(torch, *t) for t in tr]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    res = mg.group_by_desc_multi(dbs, defer_group=True, stream=s1.cuda_stream)
    mg.finish_group(s2.cuda_stream)
    torch.cuda.synchronize()
    mg.check()
    _check_maglev(torch, mg, tr, res, dbs, lut, 1000)
    mg.close()


@pytest.mark.parametrize("owned", [False, True])
@pytest.mark.parametrize("sizes", [[1 << 20, 1000, 262144], [1, 2, 3, 4, 5, 6, 7, 70000],
                                   [65536 + 7 * i for i in range(16)]])
def test_chain_multi_vs_oracle(torch_cuda, sizes, owned):
    """Config C5's chain over several IMIX batches in one launch: gate, backend, perm, counts of every
    batch as the oracle gives them for that batch alone; packet bytes unchanged (with and without
    NBG_OWNED_WINDOWS, the mode bench.py times)."""
    from netbricks_amd import Lpm, Maglev, chain_lpm_maglev_multi

    torch = torch_cuda
    lpm = Lpm(ROUTES["mixed"])
    mg = Maglev(NAMES65, 65537)
    rc, t24, tl = orc.lpm_build(ROUTES["mixed"])
    assert rc == 0
    lut = orc.lut_build(NAMES65, 65537)
    tr = _traces(sizes, seed=6000 + len(sizes))
    rng = np.random.default_rng(len(sizes))
    for buf, off, _, n in tr:  # sources in the mixed route space (10/8 and 172.16/12)
        hi = rng.integers(0, 4, n)
        ip = np.where(hi > 0, 0x0A000000 | rng.integers(0, 1 << 24, n), 0xAC100000 | rng.integers(0, 1 << 20, n))
        b = ip.astype(">u4").view(np.uint8).reshape(n, 4)
        for k in range(4):
            buf[off.astype(np.int64) + 26 + k] = b[:, k]
    dbs = [_dev_batch(torch, *t) for t in tr]
    res = chain_lpm_maglev_multi(mg, lpm, dbs, owned_windows=owned)
    torch.cuda.synchronize()
    mg.check()
    rejected = False
    for (buf, off, ln, n), r, db in zip(tr, res, dbs):
        eg, eb = orc.chain_classify(buf, n, t24, tl, lut, offs=off, lens=ln)
        perm, counts = orc.group(eb, 65)
        np.testing.assert_array_equal(_np16(r.gate, n), eg)
        np.testing.assert_array_equal(_np16(r.backend, n), eb)
        np.testing.assert_array_equal(_np32(r.counts), counts)
        np.testing.assert_array_equal(_np32(r.perm, n), perm)
        np.testing.assert_array_equal(db[0].cpu().numpy(), buf)
        rejected |= bool((eg == 3).any())
    assert rejected  # gate >= lpm_groups rejections exercised
    mg.close()
    lpm.close()


def test_desc_multi_refusals(torch_cuda):
    """0 or NBG_MAX_MULTI + 1 batches, a batch without offsets, unknown flags: NBG_EINVAL, nothing
    launched."""
    from netbricks_amd import Maglev
    from netbricks_amd._lib import NBG_EINVAL, NBG_LUT_LDS, NBG_MAX_MULTI, NbgDescBatch, lib

    torch = torch_cuda
    mg = Maglev(NAMES65, 65537)
    (buf, off, ln, n), = _traces([1000], seed=7000)
    d, o, lt, _ = _dev_batch(torch, buf, off, ln, n)
    be = torch.empty(n, dtype=torch.uint16, device="cuda")
    good = NbgDescBatch(d.data_ptr(), o.data_ptr(), lt.data_ptr(), n, be.data_ptr(), None, None, None)
    over = NBG_MAX_MULTI + 1
    arr = (NbgDescBatch * over)(*([good] * over))
    assert lib.nbg_maglev_classify_desc_multi(mg._h, arr, 0, 0, None) == NBG_EINVAL
    assert lib.nbg_maglev_classify_desc_multi(mg._h, arr, over, 0, None) == NBG_EINVAL
    assert lib.nbg_maglev_classify_desc_multi(mg._h, arr, 1, NBG_LUT_LDS, None) == NBG_EINVAL
    bad = (NbgDescBatch * 1)(NbgDescBatch(d.data_ptr(), None, lt.data_ptr(), n, be.data_ptr(), None, None, None))
    assert lib.nbg_maglev_classify_desc_multi(mg._h, bad, 1, 0, None) == NBG_EINVAL
    assert lib.nbg_chain_lpm_maglev_multi(mg._h, None, 3, arr, 1, 0, None) == NBG_EINVAL
    assert lib.nbg_maglev_classify_desc_multi(mg._h, arr, 1, 0, None) == 0
    torch.cuda.synchronize()
    mg.check()
    mg.close()


@pytest.mark.parametrize("swap", [False, True])
def test_desc_multi_beside_running_ring(torch_cuda, swap):
    """Several RX queues' IMIX batches (C3 and the C5 chain, multi-batch launches on other handles)
    while the device's persistent ring runs and takes fixed-slot batches, read only or in place: the
    tile-per-wave classify blocks and the group blocks (C3's 1001 bins included: 28 KB of LDS) co-run
    in the LDS the ring leaves, so the grouping finishes while the ring still runs (well before its
    5 s idle exit); every output bit-exact, and the ring's batches too."""
    import netbricks_amd as nb
    from netbricks_amd import Lpm, Maglev, chain_lpm_maglev_multi

    torch = torch_cuda
    ring_mg = Maglev(NAMES65, 65537)
    c3 = Maglev(NAMES1000, 655373)
    c5 = Maglev(NAMES65, 65537)
    lpm = Lpm(ROUTES["mixed"])
    lut65, lut1000 = orc.lut_build(NAMES65, 65537), orc.lut_build(NAMES1000, 655373)
    rc, t24, tl = orc.lpm_build(ROUTES["mixed"])
    assert rc == 0
    n = 100000
    rbuf = nb.make_trace(n, 0, seed=8100)[0]
    rd = torch.from_numpy(rbuf.copy()).cuda()
    rout = torch.empty(n, dtype=torch.uint16, device="cuda")
    tr3 = _traces([120000, 7, 65537], seed=8200)
    tr5 = _traces([90000, 1, 30000], seed=8300)
    db3 = [_dev_batch(torch, *t) for t in tr3]
    db5 = [_dev_batch(torch, *t) for t in tr5]
    torch.cuda.synchronize()
    s3, s5 = torch.cuda.Stream(), torch.cuda.Stream()
    with ring_mg.ring(swap_macs=swap, idle_ms=5000) as ring:
        t = ring.post(rd, n, rout)
        t0 = time.perf_counter()
        r3 = c3.group_by_desc_multi(db3, stream=s3.cuda_stream)
        r5 = chain_lpm_maglev_multi(c5, lpm, db5, stream=s5.cuda_stream)
        ring.wait(t)
        s3.synchronize()
        s5.synchronize()
        assert time.perf_counter() - t0 < 2.0  # the ring (5 s idle exit) is still resident
    c3.check()
    c5.check()
    ref = rbuf.copy()
    np.testing.assert_array_equal(_np16(rout, n), orc.classify(ref, n, lut65, swap=swap))
    np.testing.assert_array_equal(rd.cpu().numpy(), ref)
    _check_maglev(torch, c3, tr3, r3, db3, lut1000, 1000)
    for (buf, off, ln, m), r in zip(tr5, r5):
        eg, eb = orc.chain_classify(buf, m, t24, tl, lut65, offs=off, lens=ln)
        perm, counts = orc.group(eb, 65)
        np.testing.assert_array_equal(_np16(r.gate, m), eg)
        np.testing.assert_array_equal(_np16(r.backend, m), eb)
        np.testing.assert_array_equal(_np32(r.counts), counts)
        np.testing.assert_array_equal(_np32(r.perm, m), perm)
    for h in (ring_mg, c3, c5):
        h.close()
    lpm.close()
