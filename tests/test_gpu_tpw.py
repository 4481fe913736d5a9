"""GPU parity of the tile-per-wave classify kernel with 2 and 4 tiles per wave (NBG_TPW) on descriptor
layouts, where every wave loads the descriptors of all its tiles up front: the perturbed IMIX trace of
test_gpu_stream_desc.py (runts, IHL 0..15, non-IPv4, starts off the 16-B grid; ragged last tile) with
1000 backends / 655373 in place, records and read only, 65 backends read only, and the lpm -> maglev
chain, each bit-exact against the C oracle.  Reference semantics: test/maglev/src/nf.rs:92-108,
test/lpm/src/nf.rs:205-221."""
import json
import os

import numpy as np
import pytest

import orc
from test_gpu_stream_desc import N, _dev, _perturb

pytestmark = pytest.mark.gpu


def _handle(nb_, names, m, tpw):
    os.environ["NBG_TPW"] = str(tpw)  # read when the handle is created
    try:
        return nb_.Maglev(names, m)
    finally:
        os.environ.pop("NBG_TPW", None)


@pytest.mark.parametrize("tpw", [2, 4])
@pytest.mark.parametrize("nb,m,mode", [(1000, 655373, "in_place"), (1000, 655373, "records"),
                                       (1000, 655373, "read_only"), (65, 65537, "read_only")])
def test_desc_tiles_per_wave(torch_cuda, tpw, nb, m, mode):
    import netbricks_amd as nb_
    torch = torch_cuda
    names = [f"t{i}" for i in range(nb)]
    mg = _handle(nb_, names, m, tpw)
    lut = orc.lut_build(names, m)
    buf, off, ln = nb_.make_trace(N, 1, seed=tpw * 31 + nb)
    off, ln = _perturb(buf, off, ln, seed=tpw + nb)
    swap = mode != "read_only"
    ref = buf.copy()
    be = orc.classify(ref, N, lut, offs=off, lens=ln, swap=swap)
    perm, counts = orc.group(be, nb)
    d = torch.from_numpy(buf.copy()).cuda()
    mac = torch.zeros(N * 12, dtype=torch.uint8, device="cuda") if mode == "records" else None
    r = mg.group_by(d, N, offsets=_dev(torch, off, np.uint32), lens=_dev(torch, ln, np.uint16), owned_windows=True,
                    swap_macs=swap, mac_out=mac)
    torch.cuda.synchronize()
    mg.check()
    np.testing.assert_array_equal(r.backend.view(torch.int16).cpu().numpy().view(np.uint16), be)
    np.testing.assert_array_equal(r.counts.view(torch.int32).cpu().numpy().view(np.uint32), counts)
    np.testing.assert_array_equal(r.perm.view(torch.int32).cpu().numpy().view(np.uint32)[:N], perm)
    got = d.cpu().numpy()
    np.testing.assert_array_equal(got, ref if mode == "in_place" else buf)
    if mode == "records":
        rec = mac.cpu().numpy().reshape(N, 12)
        o = off.astype(np.int64)
        has = ln >= 14
        np.testing.assert_array_equal(rec[has], ref[o[has, None] + np.arange(12)[None, :]])
    mg.close()


@pytest.mark.parametrize("tpw", [2, 4])
def test_chain_tiles_per_wave(torch_cuda, tpw):
    import netbricks_amd as nb_
    from netbricks_amd import chain_lpm_maglev
    from netbricks_amd.lpm import Lpm

    torch = torch_cuda
    here = os.path.dirname(__file__)
    routes = json.load(open(os.path.join(here, "golden", "lpm_routes.json")))
    routes = routes["reference"] + routes["mixed"]
    names = [f"backend-{i}" for i in range(65)]
    mg = _handle(nb_, names, 65537, tpw)
    lpm = Lpm(routes)
    buf, off, ln = nb_.make_trace(N, 1, seed=50 + tpw)
    rng = np.random.default_rng(60 + tpw)
    hi = rng.integers(0, 4, N)
    ip = np.where(hi > 0, 0x0A000000 | rng.integers(0, 1 << 24, N), 0xAC100000 | rng.integers(0, 1 << 20, N))
    b = ip.astype(">u4").view(np.uint8).reshape(N, 4)
    for k in range(4):
        buf[off.astype(np.int64) + 26 + k] = b[:, k]
    off, ln = _perturb(buf, off, ln, seed=70 + tpw)
    d = torch.from_numpy(buf.copy()).cuda()
    r = chain_lpm_maglev(mg, lpm, d, N, offsets=_dev(torch, off, np.uint32), lens=_dev(torch, ln, np.uint16),
                         owned_windows=True)
    torch.cuda.synchronize()
    mg.check()
    rc, t24, tl = orc.lpm_build(routes)
    assert rc == 0
    eg, eb = orc.chain_classify(buf, N, t24, tl, orc.lut_build(names, 65537), offs=off, lens=ln)
    perm, counts = orc.group(eb, 65)
    np.testing.assert_array_equal(r.gate.view(torch.int16).cpu().numpy().view(np.uint16)[:N], eg)
    np.testing.assert_array_equal(r.backend.view(torch.int16).cpu().numpy().view(np.uint16)[:N], eb)
    np.testing.assert_array_equal(r.counts.view(torch.int32).cpu().numpy().view(np.uint32), counts)
    np.testing.assert_array_equal(r.perm.view(torch.int32).cpu().numpy().view(np.uint32)[:N], perm)
    np.testing.assert_array_equal(d.cpu().numpy(), buf)
    lpm.close()
    mg.close()
