"""GPU parity of the chained test/lpm -> test/maglev path (BASELINE config C5) through the C-ABI.

Bit-exact against the C oracle / golden fixtures on: lookup_entry gates (test/lpm/src/nf.rs:88-98),
per-packet (gate, backend) of lpm() -> maglev(), the per-backend FIFO order and group sizes,
and packet bytes left unchanged (the two NFs' MAC swaps cancel).
"""
import json
import os

import numpy as np
import pytest

import orc

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
ROUTES = json.load(open(os.path.join(GOLD, "lpm_routes.json")))
LPM_GOLD = json.load(open(os.path.join(GOLD, "lpm_golden.json")))
NAMES65 = [f"backend-{i}" for i in range(65)]


@pytest.fixture(scope="module")
def tables(torch_cuda):
    from netbricks_amd import Lpm, Maglev

    t = {k: Lpm(ROUTES[k]) for k in ("reference", "mixed")}
    mg = Maglev(NAMES65, 65537)
    yield t, mg
    for v in t.values():
        v.close()
    mg.close()


def _u32(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32).view(np.int32)).cuda().view(torch.uint32)


def _u16(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint16).view(np.int16)).cuda().view(torch.uint16)


def _np16(t):
    import torch

    return t.view(torch.int16).cpu().numpy().view(np.uint16)


def _np32(t):
    import torch

    return t.view(torch.int32).cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("key", ["reference", "mixed"])
def test_lpm_lookup_golden(torch_cuda, tables, key):
    torch = torch_cuda
    t, _ = tables
    g = LPM_GOLD[key]
    gate = t[key].lookup(_u32(torch, g["ips"]))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_np16(gate), np.array(g["gates"], dtype=np.uint16))


def _chain(torch, mg, lpm, buf, n, **kw):
    from netbricks_amd import chain_lpm_maglev

    d = torch.from_numpy(buf.copy()).cuda()
    if kw.get("offsets") is not None:
        kw["offsets"] = _u32(torch, kw["offsets"])
    if kw.get("lens") is not None:
        kw["lens"] = _u16(torch, kw["lens"])
    r = chain_lpm_maglev(mg, lpm, d, n, **kw)
    torch.cuda.synchronize()
    mg.check()
    return d.cpu().numpy(), _np16(r.gate)[:n], _np16(r.backend)[:n], _np32(r.perm)[:n], _np32(r.counts)


def test_chain_golden_fixture(torch_cuda, tables):
    torch = torch_cuda
    t, mg = tables
    g = np.load(os.path.join(GOLD, "lpm_chain.npz"))
    n = g["off"].size
    buf, gate, be, perm, counts = _chain(torch, mg, t["mixed"], g["buf"], n, offsets=g["off"], lens=g["len"])
    np.testing.assert_array_equal(gate, g["gate"])
    np.testing.assert_array_equal(be, g["backend"])
    np.testing.assert_array_equal(counts, g["counts"])
    np.testing.assert_array_equal(perm, g["perm"])
    np.testing.assert_array_equal(buf, g["buf"])


def _mixed_sources(buf, off, n, seed):
    """Rewrite the trace's source addresses into the mixed route space (10/8 and 172.16/12)."""
    rng = np.random.default_rng(seed)
    hi = rng.integers(0, 4, n)
    ip = np.where(hi > 0, 0x0A000000 | rng.integers(0, 1 << 24, n), 0xAC100000 | rng.integers(0, 1 << 20, n))
    b = ip.astype(">u4").view(np.uint8).reshape(n, 4)
    for k in range(4):
        buf[off.astype(np.int64) + 26 + k] = b[:, k]


@pytest.mark.parametrize("mode,n,lut_lds", [(0, 1 << 20, False), (1, 262144, False), (1, 1000, False),
                                            (0, 1 << 20, True), (1, 262144, True)])
def test_chain_vs_oracle_at_size(torch_cuda, tables, mode, n, lut_lds):
    """C2 layout (fixed 64-B slots) at full size and the IMIX descriptor layout of config C5
    (L2-gathered and LDS-staged Maglev LUT)."""
    import netbricks_amd as nb

    torch = torch_cuda
    t, mg = tables
    buf, off, ln = nb.make_trace(n, mode, seed=99 + mode)
    _mixed_sources(buf, off, n, seed=n)
    kw = dict(stride=64, frame_len=60) if mode == 0 else dict(offsets=off, lens=ln, owned_windows=True)
    got = _chain(torch, mg, t["mixed"], buf, n, lut_lds=lut_lds, **kw)
    rc, t24, tl = orc.lpm_build(ROUTES["mixed"])
    assert rc == 0
    lut = orc.lut_build(NAMES65, 65537)
    okw = dict(stride=64, fixed_len=60) if mode == 0 else dict(offs=off, lens=ln)
    eg, eb = orc.chain_classify(buf, n, t24, tl, lut, **okw)
    perm, counts = orc.group(eb, 65)
    np.testing.assert_array_equal(got[1], eg)
    np.testing.assert_array_equal(got[2], eb)
    np.testing.assert_array_equal(got[4], counts)
    np.testing.assert_array_equal(got[3], perm)
    np.testing.assert_array_equal(got[0], buf)
    assert (eg == 3).any() and (eb == 0xFFFF).any()  # gate >= lpm_groups rejections exercised


def test_chain_c5_bench_workload_1m_imix(torch_cuda, tables):
    """Config C5 exactly as tools/config_bench.py measures it: a 1M-packet IMIX descriptor batch
    (seed 1000), owned windows, the reference's 105 routes + the mixed route set, 65 backends /
    65537 slots; every output bit-exact against the oracle."""
    import netbricks_amd as nb
    from netbricks_amd.lpm import Lpm

    torch = torch_cuda
    _, mg = tables
    n = 1 << 20
    routes = ROUTES["reference"] + ROUTES["mixed"]
    lpm = Lpm(routes)
    buf, off, ln = nb.make_trace(n, 1, seed=1000)
    got = _chain(torch, mg, lpm, buf, n, offsets=off, lens=ln, owned_windows=True)
    rc, t24, tl = orc.lpm_build(routes)
    assert rc == 0
    eg, eb = orc.chain_classify(buf, n, t24, tl, orc.lut_build(NAMES65, 65537), offs=off, lens=ln)
    perm, counts = orc.group(eb, 65)
    np.testing.assert_array_equal(got[1], eg)
    np.testing.assert_array_equal(got[2], eb)
    np.testing.assert_array_equal(got[4], counts)
    np.testing.assert_array_equal(got[3], perm)
    np.testing.assert_array_equal(got[0], buf)
    lpm.close()


def test_chain_reference_routes_and_groups(torch_cuda, tables):
    """test/lpm's own table on the synthetic trace (10/8 sources: every gate 0), and a
    smaller lpm_groups that turns gate 1 into a rejection."""
    import netbricks_amd as nb

    torch = torch_cuda
    t, mg = tables
    n = 50000
    buf, off, ln = nb.make_trace(n, 0, seed=5)
    _, gate, be, _, counts = _chain(torch, mg, t["reference"], buf, n)
    assert (gate == 0).all()
    lut = orc.lut_build(NAMES65, 65537)
    np.testing.assert_array_equal(be, orc.classify(buf.copy(), n, lut, stride=64, fixed_len=60))
    _mixed_sources(buf, off, n, seed=3)
    _, gate, be, _, _ = _chain(torch, mg, t["mixed"], buf, n, lpm_groups=1)
    assert ((gate >= 1) == (be == 0xFFFF)).all()


def test_chain_empty_and_deferred(torch_cuda, tables):
    from netbricks_amd import chain_lpm_maglev

    torch = torch_cuda
    t, mg = tables
    d = torch.zeros(64, dtype=torch.uint8, device="cuda")
    r = chain_lpm_maglev(mg, t["mixed"], d, 0)
    torch.cuda.synchronize()
    assert int(r.counts.view(torch.int32).sum()) == 0
    import netbricks_amd as nb

    n = 20000
    buf, off, ln = nb.make_trace(n, 0, seed=8)
    _mixed_sources(buf, off, n, seed=9)
    d = torch.from_numpy(buf.copy()).cuda()
    r = chain_lpm_maglev(mg, t["mixed"], d, n, defer_group=True)
    mg.finish_group()
    torch.cuda.synchronize()
    rc, t24, tl = orc.lpm_build(ROUTES["mixed"])
    eg, eb = orc.chain_classify(buf, n, t24, tl, orc.lut_build(NAMES65, 65537))
    perm, counts = orc.group(eb, 65)
    np.testing.assert_array_equal(_np32(r.perm)[:n], perm)
    np.testing.assert_array_equal(_np16(r.gate)[:n], eg)
