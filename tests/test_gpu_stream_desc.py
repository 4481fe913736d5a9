"""GPU parity of the descriptor-layout streaming classify kernel (NBG_STREAM_DESC,
classify_stream_desc_kernel: IMIX offsets + lengths, owned windows, batches of >= 262144 packets)
against the C oracle.

The IMIX trace is perturbed so that every tile mixes fast-path packets with byte-wise ones: runts
(lengths 0..63 inside the original frame), IHL 0..15, non-IPv4 ethertypes and frame starts shifted
off the 16-B grid (inside frames of >= 128 B, so every window stays owned).  Covered: the u16 LUT
gathered from L2 (1000 backends / 655373) in place, as records and read only; the u8 LUT staged in
LDS (65 / 65537) as records and read only (in place falls back to the tile-per-wave kernel); and the
lpm -> maglev chain.  Reference semantics: test/maglev/src/nf.rs:92-108, test/lpm/src/nf.rs:205-221.
"""
import json
import os

import numpy as np
import pytest

import orc

pytestmark = pytest.mark.gpu

N = 300000 + 77  # above the streaming threshold, ragged last unit and tile


def _perturb(buf, off, ln, seed):
    rng = np.random.default_rng(seed)
    n = off.size
    off = off.copy()
    ln = ln.copy()
    o = off.astype(np.int64)
    runt = rng.random(n) < 0.004
    ln[runt] = rng.integers(0, 64, int(runt.sum()))
    ihl = (rng.random(n) < 0.004) & (ln > 14)
    buf[o[ihl] + 14] = (0x40 | rng.integers(0, 16, int(ihl.sum()))).astype(np.uint8)
    et = (rng.random(n) < 0.002) & (ln > 13)
    buf[o[et] + 12] = 0x86
    buf[o[et] + 13] = 0xDD
    mis = (rng.random(n) < 0.004) & (ln >= 128)
    s = rng.integers(1, 16, int(mis.sum())).astype(np.uint32)
    off[mis] += s
    ln[mis] -= s.astype(np.uint16)
    return off, ln


def _dev(torch, a, dt):
    if dt == np.uint32:
        return torch.from_numpy(np.ascontiguousarray(a, np.uint32).view(np.int32)).cuda().view(torch.uint32)
    return torch.from_numpy(np.ascontiguousarray(a, np.uint16).view(np.int16)).cuda().view(torch.uint16)


@pytest.mark.parametrize("nb,m,mode", [(1000, 655373, "in_place"), (1000, 655373, "records"),
                                       (1000, 655373, "read_only"), (65, 65537, "records"),
                                       (65, 65537, "read_only"), (65, 65537, "in_place")])
def test_stream_desc_modes(torch_cuda, nb, m, mode):
    import netbricks_amd as nb_
    torch = torch_cuda
    names = [f"s{i}" for i in range(nb)]
    mg = nb_.Maglev(names, m)
    lut = orc.lut_build(names, m)
    buf, off, ln = nb_.make_trace(N, 1, seed=nb + len(mode))
    off, ln = _perturb(buf, off, ln, seed=nb)
    swap = mode != "read_only"
    ref = buf.copy()
    be = orc.classify(ref, N, lut, offs=off, lens=ln, swap=swap)
    perm, counts = orc.group(be, nb)
    d = torch.from_numpy(buf.copy()).cuda()
    kw = {}
    mac = None
    if mode == "records":
        mac = torch.zeros(N * 12, dtype=torch.uint8, device="cuda")
        kw["mac_out"] = mac
    r = mg.group_by(d, N, offsets=_dev(torch, off, np.uint32), lens=_dev(torch, ln, np.uint16), owned_windows=True,
                    swap_macs=swap, stream_desc=True, **kw)
    torch.cuda.synchronize()
    mg.check()
    np.testing.assert_array_equal(r.backend.view(torch.int16).cpu().numpy().view(np.uint16), be)
    np.testing.assert_array_equal(r.counts.view(torch.int32).cpu().numpy().view(np.uint32), counts)
    np.testing.assert_array_equal(r.perm.view(torch.int32).cpu().numpy().view(np.uint32)[:N], perm)
    got = d.cpu().numpy()
    if mode == "in_place":
        np.testing.assert_array_equal(got, ref)
    else:
        np.testing.assert_array_equal(got, buf)  # packets untouched
    if mode == "records":
        rec = mac.cpu().numpy().reshape(N, 12)
        o = off.astype(np.int64)
        has = ln >= 14
        idx = o[has, None] + np.arange(12)[None, :]
        np.testing.assert_array_equal(rec[has], ref[idx])
        assert not rec[~has].any()
    assert (be == 0xFFFF).any() and (be != 0xFFFF).any()
    mg.close()


def test_stream_desc_chain(torch_cuda):
    """The lpm -> maglev chain through the streaming kernel (u8 LUT in LDS, tbl24 gathered, the
    routes longer than /24 through tbl_long) on the perturbed trace."""
    import netbricks_amd as nb_
    from netbricks_amd import chain_lpm_maglev
    from netbricks_amd.lpm import Lpm

    torch = torch_cuda
    here = os.path.dirname(__file__)
    routes = json.load(open(os.path.join(here, "golden", "lpm_routes.json")))
    routes = routes["reference"] + routes["mixed"]
    names = [f"backend-{i}" for i in range(65)]
    mg = nb_.Maglev(names, 65537)
    lpm = Lpm(routes)
    buf, off, ln = nb_.make_trace(N, 1, seed=5)
    rng = np.random.default_rng(6)
    hi = rng.integers(0, 4, N)
    ip = np.where(hi > 0, 0x0A000000 | rng.integers(0, 1 << 24, N), 0xAC100000 | rng.integers(0, 1 << 20, N))
    b = ip.astype(">u4").view(np.uint8).reshape(N, 4)
    for k in range(4):
        buf[off.astype(np.int64) + 26 + k] = b[:, k]
    off, ln = _perturb(buf, off, ln, seed=7)
    d = torch.from_numpy(buf.copy()).cuda()
    r = chain_lpm_maglev(mg, lpm, d, N, offsets=_dev(torch, off, np.uint32), lens=_dev(torch, ln, np.uint16),
                         owned_windows=True, stream_desc=True)
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
    assert (eb == 0xFFFF).any()
    lpm.close()
    mg.close()
