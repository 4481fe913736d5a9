"""GPU parity of the exact C3 and C5 configurations bench.py times (variants c3_multi8 / c3_multi16 /
c5_multi8 / c5_multi16): k = 8 and 16 RX queues' 1M IMIX batches (seeds 1000 + b, as bench.py's
imix_multi_setup) per launch of nbg_maglev_classify_desc_multi (1000 backends / M = 655373, NBG_SWAP_MACS,
NBG_OWNED_WINDOWS: whole 64-B windows rewritten in place) and nbg_chain_lpm_maglev_multi (65 backends /
65537, the reference's 105 routes + the 902 mixed ones, lpm_groups 3, NBG_OWNED_WINDOWS).  Every batch's
backend[], perm, counts (and gate) and its packet bytes are bit-exact against the C oracle run on that
batch alone (test/maglev/src/nf.rs:92-106, test/lpm/src/nf.rs:88-98,212-228, operators/group_by.rs:43-55).
"""
import json
import os

import numpy as np
import pytest

import orc

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BATCH = 1 << 20
NAMES65 = [f"backend-{i}" for i in range(65)]
NAMES1000 = [f"be{i}" for i in range(1000)]


@pytest.fixture(scope="module")
def traces():
    """bench.py's 16 distinct 1M IMIX batches (host copies; 374 MB each)."""
    import netbricks_amd as nb

    return [nb.make_trace(BATCH, 1, seed=1000 + b) for b in range(16)]


def _upload(torch, buf, off, ln):
    return (torch.from_numpy(buf.copy()).cuda(), torch.from_numpy(off.view(np.int32)).cuda().view(torch.uint32),
            torch.from_numpy(ln.view(np.int16)).cuda().view(torch.uint16), BATCH)


def _u16(torch, t):
    return t.view(torch.int16).cpu().numpy().view(np.uint16)


def _u32(torch, t):
    return t.view(torch.int32).cpu().numpy().view(np.uint32)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("k", [8, 16])
def test_c3_bench_shape_owned_windows(torch_cuda, traces, k):
    from netbricks_amd import Maglev

    torch = torch_cuda
    mg = Maglev(NAMES1000, 655373)
    lut = orc.lut_build(NAMES1000, 655373)
    dbs = [_upload(torch, *traces[b]) for b in range(k)]
    res = mg.group_by_desc_multi(dbs, swap_macs=True, owned_windows=True, bounds_check=False)
    torch.cuda.synchronize()
    mg.check()
    for (buf, off, ln), r, db in zip(traces, res, dbs):
        ref = buf.copy()
        be = orc.classify(ref, BATCH, lut, offs=off, lens=ln, swap=True)
        perm, counts = orc.group(be, 1000)
        np.testing.assert_array_equal(_u16(torch, r.backend), be)
        np.testing.assert_array_equal(_u32(torch, r.counts), counts)
        np.testing.assert_array_equal(_u32(torch, r.perm), perm)
        np.testing.assert_array_equal(db[0].cpu().numpy(), ref)  # whole windows rewritten, MACs swapped
    mg.close()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("k", [8, 16])
def test_c5_bench_shape_owned_windows(torch_cuda, traces, k):
    from netbricks_amd import Lpm, Maglev, chain_lpm_maglev_multi

    torch = torch_cuda
    routes = json.load(open(os.path.join(ROOT, "tests", "golden", "lpm_routes.json")))
    rset = routes["reference"] + routes["mixed"]
    lpm = Lpm(rset)
    rc, t24, tl = orc.lpm_build(rset)
    assert rc == 0
    lut = orc.lut_build(NAMES65, 65537)
    mg = Maglev(lut=lut.astype(np.uint16), n_backends=65)
    dbs = [_upload(torch, *traces[b]) for b in range(k)]
    res = chain_lpm_maglev_multi(mg, lpm, dbs, lpm_groups=3, owned_windows=True, bounds_check=False)
    torch.cuda.synchronize()
    mg.check()
    gates = set()
    for (buf, off, ln), r, db in zip(traces, res, dbs):
        eg, eb = orc.chain_classify(buf, BATCH, t24, tl, lut, offs=off, lens=ln, lpm_groups=3)
        perm, counts = orc.group(eb, 65)
        np.testing.assert_array_equal(_u16(torch, r.gate), eg)
        np.testing.assert_array_equal(_u16(torch, r.backend), eb)
        np.testing.assert_array_equal(_u32(torch, r.counts), counts)
        np.testing.assert_array_equal(_u32(torch, r.perm), perm)
        np.testing.assert_array_equal(db[0].cpu().numpy(), buf)  # the two MAC swaps cancel: read only
        gates.update(np.unique(eg).tolist())
    assert {0, 1, 2}.issubset(gates)
    mg.close()
    lpm.close()
