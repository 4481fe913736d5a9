"""Zero-copy host path: frames in a registered host region (an mbuf pool), read by the GPU over
PCIe and MAC-swapped in place there; bit-exact against the C oracle on the same pool.  Covers
IMIX frames at mbuf headroom, the byte-wise cases (runts, IHL 0-15, non-IPv4, frame starts off the
16-B grid) and a 100k-mbuf batch.  Reference semantics: test/maglev/src/nf.rs:92-108 over mbufs
(native/zcsi/mbuf.rs:34-49)."""
import numpy as np
import pytest

import orc

pytestmark = pytest.mark.gpu

NAMES = [f"backend-{i}" for i in range(65)]
ROOM, HEADROOM = 2048, 128


def _pool(n, seed):
    """n mbufs of ROOM bytes; frame i at HEADROOM (+ a small shift for some) in mbuf i."""
    import netbricks_amd as nb

    rng = np.random.default_rng(seed)
    buf, off, ln = nb.make_trace(n, 1, seed=seed)
    pool = np.zeros(n * ROOM, dtype=np.uint8)
    offs = np.arange(n, dtype=np.uint64) * ROOM + HEADROOM
    shift = np.where(rng.random(n) < 0.01, rng.integers(1, 16, n), 0).astype(np.uint64)
    offs += shift
    lens = np.minimum(ln.astype(np.int64), ROOM - HEADROOM - 16).astype(np.uint16)
    runt = rng.random(n) < 0.005
    lens[runt] = rng.integers(0, 64, int(runt.sum()))
    for i in range(n):
        pool[offs[i]:offs[i] + lens[i]] = buf[off[i]:off[i] + lens[i]]
    ihl = (rng.random(n) < 0.005) & (lens > 14)
    pool[offs[ihl] + 14] = (0x40 | rng.integers(0, 16, int(ihl.sum()))).astype(np.uint8)
    et = (rng.random(n) < 0.003) & (lens > 13)
    pool[offs[et] + 12] = 0x86
    pool[offs[et] + 13] = 0xDD
    return pool, offs.astype(np.uint32), lens


@pytest.mark.parametrize("n,group", [(5000, True), (100000, True), (3000, False)])
def test_region_classify_in_place(torch_cuda, n, group):
    import netbricks_amd as nb

    torch = torch_cuda
    pool, offs, lens = _pool(n, seed=n)
    ref = pool.copy()
    be = orc.classify(ref, n, orc.lut_build(NAMES, 65537), offs=offs, lens=lens)
    mg = nb.Maglev(NAMES, 65537)
    d_off = torch.from_numpy(offs.view(np.int32)).cuda().view(torch.uint32)
    d_len = torch.from_numpy(lens.view(np.int16)).cuda().view(torch.uint16)
    with nb.HostRegion(pool) as reg:
        r = mg.group_by_region(reg, n, d_off, d_len, group=group)
        torch.cuda.synchronize()
        mg.check()
    np.testing.assert_array_equal(r.backend.view(torch.int16).cpu().numpy().view(np.uint16)[:n], be)
    if group:
        perm, counts = orc.group(be, 65)
        np.testing.assert_array_equal(r.perm.view(torch.int32).cpu().numpy().view(np.uint32)[:n], perm)
        np.testing.assert_array_equal(r.counts.view(torch.int32).cpu().numpy().view(np.uint32), counts)
    np.testing.assert_array_equal(pool, ref)  # the MAC swap landed in the host frames, nothing else changed
    assert (be == 0xFFFF).any() and (be != 0xFFFF).any()
    mg.close()


def test_region_rejects_closed_and_bad_arrays(torch_cuda):
    import netbricks_amd as nb

    torch = torch_cuda
    pool = np.zeros(1 << 16, dtype=np.uint8)
    reg = nb.HostRegion(pool)
    reg.close()
    mg = nb.Maglev(NAMES, 65537)
    z32 = torch.zeros(4, dtype=torch.int32, device="cuda").view(torch.uint32)
    z16 = torch.zeros(4, dtype=torch.int16, device="cuda").view(torch.uint16)
    with pytest.raises(ValueError):
        mg.group_by_region(reg, 4, z32, z16)
    with pytest.raises(ValueError):
        nb.HostRegion(np.zeros(16, dtype=np.uint16))
    with pytest.raises(ValueError):
        nb.HostRegion(np.zeros((4, 16), dtype=np.uint8)[:, :8])
    mg.close()


@pytest.mark.parametrize("n", [20000, 992, 1])
def test_host_submit_takes_zero_copy_for_registered_pool(torch_cuda, n):
    """nbg_maglev_host_submit over mbufs inside a registered region: the GPU rewrites the frames
    itself (the swap is in host memory once the device is idle, before host_wait), results
    bit-exact; the same batch from an unregistered pool takes the gather path, which swaps the MACs
    in the mbufs as it stages them (also before host_wait).  Batches of at most 2,048 packets take
    the direct path (offsets or windows, lengths and results in pinned memory, one kernel launch,
    no copy)."""
    import netbricks_amd as nb

    torch = torch_cuda
    pool, offs, lens = _pool(n, seed=11)
    ref = pool.copy()
    be = orc.classify(ref, n, orc.lut_build(NAMES, 65537), offs=offs, lens=lens)
    perm, counts = orc.group(be, 65)
    mg = nb.Maglev(NAMES, 65537)
    for registered in (True, False):
        work = pool.copy()
        ptrs = (offs.astype(np.uint64) + np.uint64(work.ctypes.data)).astype(np.uint64)
        reg = nb.HostRegion(work) if registered else None
        out_be, out_pm, out_ct = np.empty(n, np.uint16), np.empty(n, np.uint32), np.empty(66, np.uint32)
        tk = mg.host_submit(ptrs, lens, out_be, out_pm, out_ct)
        torch.cuda.synchronize()
        swapped_before_wait = np.array_equal(work, ref)
        mg.host_wait(tk)
        np.testing.assert_array_equal(out_be, be)
        np.testing.assert_array_equal(out_pm, perm)
        np.testing.assert_array_equal(out_ct, counts)
        np.testing.assert_array_equal(work, ref)
        assert swapped_before_wait
        if reg is not None:
            reg.close()
    mg.close()
