"""GPU parity: the HIP path (through the C-ABI) vs the C oracle on the same seeded inputs.

Bit-exact on backend[], on the MAC-swapped packet bytes, on the per-group FIFO order
(perm) and on the group sizes.  Reference semantics: test/maglev/src/nf.rs:92-108.
"""
import numpy as np
import pytest

import orc

pytestmark = pytest.mark.gpu

NAMES65 = [f"backend-{i}" for i in range(65)]


@pytest.fixture(scope="module")
def mg65(torch_cuda):
    from netbricks_amd import Maglev

    m = Maglev(NAMES65, 65537)
    yield m
    m.close()


def _run(torch, mg, buf, n, *, offs=None, lens=None, stride=64, frame_len=60, swap=True, lut_lds=False):
    dev = torch.device("cuda:0")
    d_buf = torch.from_numpy(buf.copy()).to(dev)
    d_off = None if offs is None else torch.from_numpy(offs.astype(np.uint32).view(np.int32)).to(dev)
    d_len = None if lens is None else torch.from_numpy(lens.astype(np.uint16).view(np.int16)).to(dev)
    d_off = None if d_off is None else d_off.view(torch.uint32)
    d_len = None if d_len is None else d_len.view(torch.uint16)
    r = mg.group_by(d_buf, n, stride=stride, frame_len=frame_len, offsets=d_off, lens=d_len, swap_macs=swap,
                    lut_lds=lut_lds)
    torch.cuda.synchronize()
    mg.check()
    backend = r.backend.view(torch.int16).cpu().numpy().view(np.uint16)
    perm = r.perm.view(torch.int32).cpu().numpy().view(np.uint32)[:n]
    counts = r.counts.view(torch.int32).cpu().numpy().view(np.uint32)
    return d_buf.cpu().numpy(), backend, perm, counts


def _oracle(buf, n, lut, nb, **kw):
    ref = buf.copy()
    be = orc.classify(ref, n, lut, **kw)
    perm, counts = orc.group(be, nb)
    return ref, be, perm, counts


def _assert_same(got, exp):
    gbuf, gbe, gperm, gcnt = got
    ebuf, ebe, eperm, ecnt = exp
    np.testing.assert_array_equal(gbe, ebe)
    np.testing.assert_array_equal(gcnt, ecnt)
    np.testing.assert_array_equal(gperm, eperm)
    np.testing.assert_array_equal(gbuf, ebuf)


def test_lut_matches_oracle(mg65):
    np.testing.assert_array_equal(mg65.lut(), orc.lut_build(NAMES65, 65537).astype(np.uint16))


@pytest.mark.parametrize("n", [1, 63, 64, 1000, 1024, 1025, 4096, 65536 + 77])
@pytest.mark.parametrize("lut_lds", [False, True])
def test_c2_small(torch_cuda, mg65, n, lut_lds):
    from netbricks_amd import make_trace

    buf, _, _ = make_trace(n, 0, seed=1234 + n)
    lut = orc.lut_build(NAMES65, 65537)
    got = _run(torch_cuda, mg65, buf, n, lut_lds=lut_lds)
    _assert_same(got, _oracle(buf, n, lut, 65, stride=64, fixed_len=60))


@pytest.mark.parametrize("lut_lds", [False, True])
def test_c2_full_1m(torch_cuda, mg65, lut_lds):
    """BASELINE config C2 size: 1,048,576 x 64-B frames, 65 backends, M=65537 (L2-gathered LUT, and
    the LDS-staged LUT whose waves keep two tiles' loads in flight)."""
    from netbricks_amd import make_trace

    n = 1 << 20
    buf, _, _ = make_trace(n, 0)
    lut = orc.lut_build(NAMES65, 65537)
    got = _run(torch_cuda, mg65, buf, n, lut_lds=lut_lds)
    exp = _oracle(buf, n, lut, 65, stride=64, fixed_len=60)
    _assert_same(got, exp)
    # size-independent properties: perm is a permutation, groups sorted, counts sum to n
    perm, counts = got[2], got[3]
    assert counts.sum() == n
    assert np.array_equal(np.sort(perm), np.arange(n, dtype=np.uint32))


@pytest.mark.parametrize("n", [(1 << 21) + 12345, (1 << 24) + 1000])
def test_c2_multi_chunk_partitions(torch_cuda, mg65, n):
    """Batches above 1M packets: partitions of several 4096-packet chunks per group block; above
    15.7M the partition counts no longer fit 16 bits and the rows stay 32-bit."""
    from netbricks_amd import make_trace

    buf, _, _ = make_trace(n, 0, seed=n & 0xFFFF)
    lut = orc.lut_build(NAMES65, 65537)
    got = _run(torch_cuda, mg65, buf, n)
    exp = _oracle(buf, n, lut, 65, stride=64, fixed_len=60)
    _assert_same(got, exp)


@pytest.mark.parametrize("nb", [1, 63, 64, 127, 128])
@pytest.mark.parametrize("n", [2 * 4096 + 37, 300001, (1 << 21) + 777])
def test_group_bin_widths(torch_cuda, nb, n):
    """The group kernel's rank forms at their edges: up to 128 bins the per-wave LDS table of lane
    masks (nb = 127: 128 bins, the table's scratch entry 128 for lanes past the end; nb = 1: every lane
    of a round in one of two bins), 129 bins the ballot multisplit; batches with a ragged last round,
    several partitions, and partitions of several chunks (group_by.rs:46-51 FIFO order)."""
    import netbricks_amd as nb_
    from netbricks_amd import make_trace

    names = [f"backend-{i}" for i in range(nb)]
    mg = nb_.Maglev(names, 65537)
    try:
        buf, _, _ = make_trace(n, 0, seed=nb * 7919 + n % 1000)
        lut = orc.lut_build(names, 65537)
        _assert_same(_run(torch_cuda, mg, buf, n), _oracle(buf, n, lut, nb, stride=64, fixed_len=60))
    finally:
        mg.close()


@pytest.mark.parametrize("shift", [0, 1, 3])
def test_backend_output_alignment(torch_cuda, mg65, shift):
    """backend[] at any 2-B alignment: the streaming kernel stores a whole tile's backends as 16-B
    words only into a 16-B-aligned buffer, else one 2-B store per lane (same values)."""
    from netbricks_amd import make_trace

    torch = torch_cuda
    n = 300001
    buf, _, _ = make_trace(n, 0, seed=4242 + shift)
    dev = torch.device("cuda:0")
    d_buf = torch.from_numpy(buf.copy()).to(dev)
    room = torch.zeros(n + 16, dtype=torch.int16, device=dev).view(torch.uint16)
    be = room[shift:shift + n]
    r = mg65.group_by(d_buf, n, backend=be)
    torch.cuda.synchronize()
    mg65.check()
    lut = orc.lut_build(NAMES65, 65537)
    ref = buf.copy()
    ebe = orc.classify(ref, n, lut, stride=64, fixed_len=60)
    eperm, ecnt = orc.group(ebe, 65)
    got = room.view(torch.int16).cpu().numpy().view(np.uint16)
    np.testing.assert_array_equal(got[shift:shift + n], ebe)
    assert not got[:shift].any() and not got[shift + n:].any()  # nothing written outside the view
    np.testing.assert_array_equal(r.perm.view(torch.int32).cpu().numpy().view(np.uint32)[:n], eperm)
    np.testing.assert_array_equal(r.counts.view(torch.int32).cpu().numpy().view(np.uint32), ecnt)
    np.testing.assert_array_equal(d_buf.cpu().numpy(), ref)


def test_many_backends_multi_chunk(torch_cuda):
    """1000 backends at 16.8M packets: hist_kernel + scan_kernel over partitions of several chunks
    (partition counts above 16 bits)."""
    import netbricks_amd as nb
    from netbricks_amd import make_trace

    names = [f"backend-{i}" for i in range(1000)]
    mg = nb.Maglev(names, 655373)
    n = (1 << 24) + 1000
    buf, _, _ = make_trace(n, 0, seed=77)
    lut = orc.lut_build(names, 655373)
    _assert_same(_run(torch_cuda, mg, buf, n), _oracle(buf, n, lut, 1000, stride=64, fixed_len=60))


def test_no_swap_and_no_group(torch_cuda, mg65):
    from netbricks_amd import make_trace

    n = 5000
    buf, _, _ = make_trace(n, 0, seed=7)
    lut = orc.lut_build(NAMES65, 65537)
    dev = torch_cuda.device("cuda:0")
    d_buf = torch_cuda.from_numpy(buf.copy()).to(dev)
    r = mg65.group_by(d_buf, n, swap_macs=False, group=False)
    torch_cuda.cuda.synchronize()
    ref = buf.copy()
    exp = orc.classify(ref, n, lut, stride=64, fixed_len=60, swap=False)
    np.testing.assert_array_equal(r.backend.view(torch_cuda.int16).cpu().numpy().view(np.uint16), exp)
    np.testing.assert_array_equal(d_buf.cpu().numpy(), buf)  # untouched


def test_reference_names_lut3(torch_cuda):
    """The reference's own backend list (test/maglev/src/main.rs:36)."""
    from netbricks_amd import Maglev, make_trace

    names = ["Larry", "Curly", "Moe"]
    mg = Maglev(names, 65537)
    n = 10000
    buf, _, _ = make_trace(n, 0, seed=99)
    lut = orc.lut_build(names, 65537)
    _assert_same(_run(torch_cuda, mg, buf, n), _oracle(buf, n, lut, 3, stride=64, fixed_len=60))
    mg.close()


@pytest.mark.parametrize("lut_lds", [False, True])
@pytest.mark.parametrize("nb,m", [(1000, 655373), (300, 65537), (2, 7), (257, 1009), (65, 65537)])
def test_imix_descriptors(torch_cuda, nb, m, lut_lds):
    """C3-like: IMIX frames at 64-B aligned offsets with a length array; wide/global LUTs (the LDS
    flag stages the LUTs that fit: u8 65537, u16 1009, u8 7)."""
    from netbricks_amd import Maglev, make_trace

    names = [f"be{i}" for i in range(nb)]
    mg = Maglev(names, m)
    n = 20000
    buf, off, ln = make_trace(n, 1, seed=nb)
    lut = orc.lut_build(names, m)
    got = _run(torch_cuda, mg, buf, n, offs=off, lens=ln, lut_lds=lut_lds)
    _assert_same(got, _oracle(buf, n, lut, nb, offs=off, lens=ln))
    mg.close()


@pytest.mark.parametrize("tiled", [False, True])
def test_c3_full_1m(torch_cuda, tiled):
    """BASELINE config C3 size: 1,048,576 IMIX frames (64-B aligned descriptors, in-place swap over
    owned windows), 1000 backends, M = 655373 (u16 LUT, hist_kernel + scan_kernel grouping); with
    the L2-gathered LUT and with the LDS-tiled lookup (NBG_LUT_TILED: 21 tiles of 64 KiB)."""
    from netbricks_amd import Maglev, make_trace

    names = [f"be{i}" for i in range(1000)]
    mg = Maglev(names, 655373)
    n = 1 << 20
    buf, off, ln = make_trace(n, 1, seed=1000)
    lut = orc.lut_build(names, 655373)
    dev = torch_cuda.device("cuda:0")
    d_buf = torch_cuda.from_numpy(buf.copy()).to(dev)
    d_off = torch_cuda.from_numpy(off.view(np.int32)).to(dev).view(torch_cuda.uint32)
    d_len = torch_cuda.from_numpy(ln.view(np.int16)).to(dev).view(torch_cuda.uint16)
    r = mg.group_by(d_buf, n, offsets=d_off, lens=d_len, owned_windows=True, lut_tiled=tiled)
    torch_cuda.cuda.synchronize()
    mg.check()
    got = (d_buf.cpu().numpy(), r.backend.view(torch_cuda.int16).cpu().numpy().view(np.uint16),
           r.perm.view(torch_cuda.int32).cpu().numpy().view(np.uint32),
           r.counts.view(torch_cuda.int32).cpu().numpy().view(np.uint32))
    exp = _oracle(buf, n, lut, 1000, offs=off, lens=ln)
    _assert_same(got, exp)
    assert got[3].sum() == n and (got[3][:1000] > 0).all()
    mg.close()


def _edge_frames(rng):
    """Hand-built edge cases: IHL 0..15 with options, runts, non-IPv4, odd lengths."""
    frames = []
    base = bytearray(rng.integers(0, 256, 128, dtype=np.uint8).tobytes())
    base[12:14] = b"\x08\x00"
    for ihl in range(16):
        for ln in (13, 14, 15, 33, 34, 37, 38, 39, 40, 41, 47, 48, 49, 60, 64, 78, 79, 100, 128):
            f = bytearray(base[:ln])
            if ln > 14:
                f[14] = 0x40 | ihl
            frames.append(f)
    for et in (b"\x86\xdd", b"\x08\x06", b"\x81\x00"):
        f = bytearray(base[:64])
        f[12:14] = et
        frames.append(f)
    frames.append(bytearray())
    return frames


def _pack(frames, align):
    offs, lens, pos = [], [], 0
    for f in frames:
        offs.append(pos)
        lens.append(len(f))
        pos += (len(f) + align - 1) // align * align + align
    buf = np.zeros(pos + 128, dtype=np.uint8)
    for o, f in zip(offs, frames):
        buf[o:o + len(f)] = np.frombuffer(bytes(f), dtype=np.uint8)
    return buf, np.array(offs, dtype=np.uint32), np.array(lens, dtype=np.uint16)


@pytest.mark.parametrize("n,mode,nb,m", [(1, 0, 300, 65537), (5000, 0, 300, 65537), (70000, 1, 1000, 655373),
                                        (300000, 0, 4096, 655373)])
def test_lut_tiled_variants(torch_cuda, n, mode, nb, m):
    """NBG_LUT_TILED at several sizes, layouts and table sizes (a LUT of 2 to 21 tiles)."""
    from netbricks_amd import Maglev, make_trace

    names = [f"t{i}" for i in range(nb)]
    mg = Maglev(names, m)
    lut = orc.lut_build(names, m)
    buf, off, ln = make_trace(n, mode, seed=n + nb)
    dev = torch_cuda.device("cuda:0")
    d_buf = torch_cuda.from_numpy(buf.copy()).to(dev)
    kw = {}
    if mode:
        kw = dict(offsets=torch_cuda.from_numpy(off.view(np.int32)).to(dev).view(torch_cuda.uint32),
                  lens=torch_cuda.from_numpy(ln.view(np.int16)).to(dev).view(torch_cuda.uint16))
    r = mg.group_by(d_buf, n, lut_tiled=True, **kw)
    torch_cuda.cuda.synchronize()
    mg.check()
    got = (d_buf.cpu().numpy(), r.backend.view(torch_cuda.int16).cpu().numpy().view(np.uint16),
           r.perm.view(torch_cuda.int32).cpu().numpy().view(np.uint32)[:n],
           r.counts.view(torch_cuda.int32).cpu().numpy().view(np.uint32))
    okw = dict(stride=64, fixed_len=60) if mode == 0 else dict(offs=off, lens=ln)
    _assert_same(got, _oracle(buf, n, lut, nb, **okw))
    mg.close()


@pytest.mark.parametrize("align", [1, 4, 64])
def test_edge_cases(torch_cuda, mg65, align):
    rng = np.random.default_rng(5)
    frames = _edge_frames(rng)
    buf, off, ln = _pack(frames, align)
    if align == 1:
        off = off + 3  # deliberately misaligned frame starts
        buf = np.concatenate([np.zeros(3, np.uint8), buf])
    lut = orc.lut_build(NAMES65, 65537)
    n = len(frames)
    got = _run(torch_cuda, mg65, buf, n, offs=off, lens=ln)
    exp = _oracle(buf, n, lut, 65, offs=off, lens=ln)
    _assert_same(got, exp)
    assert (got[1] == 0xFFFF).any() and (got[1] != 0xFFFF).any()


def test_repeat_calls_epochs(torch_cuda, mg65):
    """Many back-to-back calls reuse the look-back scratch via epochs (no memset)."""
    from netbricks_amd import make_trace

    lut = orc.lut_build(NAMES65, 65537)
    for k, n in enumerate([3000, 100000, 1024, 77777, 3000]):
        buf, _, _ = make_trace(n, 0, seed=k)
        _assert_same(_run(torch_cuda, mg65, buf, n), _oracle(buf, n, lut, 65, stride=64, fixed_len=60))


@pytest.mark.parametrize("n", [1, 32, 100])
def test_many_small_batches(torch_cuda, n):
    """Dozens of small back-to-back batches on one handle (both histogram buffers, every
    partition-row and super-row reset), on the device and the host path."""
    import netbricks_amd as nb
    from netbricks_amd import make_trace

    mg = nb.Maglev(NAMES65, 65537)
    lut = orc.lut_build(NAMES65, 65537)
    for k in range(40):
        buf, _, _ = make_trace(n, 0, seed=100 + k)
        _assert_same(_run(torch_cuda, mg, buf, n), _oracle(buf, n, lut, 65, stride=64, fixed_len=60))
    for k in range(40):
        buf, off, ln = make_trace(n, 1, seed=200 + k)
        frames = [bytearray(buf[o:o + l].tobytes()) for o, l in zip(off, ln)]
        pbuf, poff, pln = _pack([bytearray(f) for f in frames], 64)
        exp = _oracle(pbuf, len(frames), lut, 65, offs=poff, lens=pln)
        be, perm, counts = mg.group_by_host(frames)
        np.testing.assert_array_equal(be, exp[1])
        np.testing.assert_array_equal(perm, exp[2])
        np.testing.assert_array_equal(counts, exp[3])
        for f, o, l in zip(frames, poff, pln):
            assert bytes(f) == exp[0][o:o + l].tobytes()


def test_host_path(torch_cuda, mg65):
    """nbg_maglev_classify_host: mbuf-like host frames -> H2D -> kernel -> D2H, MACs swapped in place."""
    rng = np.random.default_rng(11)
    from netbricks_amd import make_trace

    n = 3000
    buf, off, ln = make_trace(n, 1, seed=3)
    frames = [bytearray(buf[o:o + l].tobytes()) for o, l in zip(off, ln)]
    frames += _edge_frames(rng)
    lut = orc.lut_build(NAMES65, 65537)
    pbuf, poff, pln = _pack([bytearray(f) for f in frames], 64)
    exp = _oracle(pbuf, len(frames), lut, 65, offs=poff, lens=pln)
    be, perm, counts = mg65.group_by_host(frames)
    np.testing.assert_array_equal(be, exp[1])
    np.testing.assert_array_equal(perm, exp[2])
    np.testing.assert_array_equal(counts, exp[3])
    for f, o, l in zip(frames, poff, pln):
        assert bytes(f) == exp[0][o:o + l].tobytes()


def test_mac_out_record(torch_cuda, mg65):
    """classify_device_ex with d_mac_out: 12-B swapped-MAC records, packet bytes untouched."""
    from netbricks_amd import make_trace

    rng = np.random.default_rng(2)
    frames = [bytearray(f) for f in _edge_frames(rng)]
    buf0, off0, ln0 = make_trace(2000, 1, seed=21)
    frames += [bytearray(buf0[o:o + l].tobytes()) for o, l in zip(off0, ln0)]
    buf, off, ln = _pack(frames, 64)
    n = len(frames)
    lut = orc.lut_build(NAMES65, 65537)
    exp = _oracle(buf, n, lut, 65, offs=off, lens=ln)
    dev = torch_cuda.device("cuda:0")
    d_buf = torch_cuda.from_numpy(buf.copy()).to(dev)
    d_off = torch_cuda.from_numpy(off.view(np.int32)).to(dev).view(torch_cuda.uint32)
    d_len = torch_cuda.from_numpy(ln.view(np.int16)).to(dev).view(torch_cuda.uint16)
    mac = torch_cuda.zeros(n * 12, dtype=torch_cuda.uint8, device=dev)
    r = mg65.group_by(d_buf, n, offsets=d_off, lens=d_len, mac_out=mac)
    torch_cuda.cuda.synchronize()
    np.testing.assert_array_equal(r.backend.view(torch_cuda.int16).cpu().numpy().view(np.uint16), exp[1])
    np.testing.assert_array_equal(r.perm.view(torch_cuda.int32).cpu().numpy().view(np.uint32), exp[2])
    np.testing.assert_array_equal(d_buf.cpu().numpy(), buf)  # packets untouched
    m = mac.cpu().numpy().reshape(n, 12)
    for i, (o, l) in enumerate(zip(off, ln)):
        if l >= 14:
            assert m[i].tobytes() == exp[0][o:o + 12].tobytes(), i
        else:
            assert not m[i].any()


@pytest.mark.parametrize("nb,m,n,mode", [(1500, 65537, 3000, 0), (4096, 655373, 1 << 20, 0),
                                        (4096, 655373, 300000, 1), (32767, 655373, 200000, 0)])
def test_many_backends_wide_grouping(torch_cuda, nb, m, n, mode):
    """More than 1023 backends (up to 32767, the LUT sentinel bound of nf.rs:46): the wide grouping
    path (hist_kernel + scan_kernel + bin_base_kernel + group_wide_kernel) gives the oracle's
    per-group FIFO order; fixed slots and IMIX descriptors, deferred grouping too."""
    from netbricks_amd import Maglev, make_trace

    names = [f"b{i}" for i in range(nb)]
    mg = Maglev(names, m)
    lut = orc.lut_build(names, m)
    np.testing.assert_array_equal(mg.lut(), lut.astype(np.uint16))
    buf, off, ln = make_trace(n, mode, seed=nb + n)
    kw = dict(stride=64, fixed_len=60) if mode == 0 else dict(offs=off, lens=ln)
    exp = _oracle(buf, n, lut, nb, **kw)
    rkw = dict(stride=64, frame_len=60) if mode == 0 else dict(offs=off, lens=ln)
    _assert_same(_run(torch_cuda, mg, buf, n, **rkw), exp)
    mg.close()


def test_group_limit_32767(torch_cuda):
    """Grouping past 32767 backends is refused (the reference's 0x8000 fill sentinel collides just
    above, nf.rs:46); backend-only classify has no such limit."""
    from netbricks_amd import Maglev, NbgError, make_trace

    names = [f"b{i}" for i in range(32768)]
    mg = Maglev(names, 655373)
    n = 3000
    buf, _, _ = make_trace(n, 0, seed=8)
    d = torch_cuda.from_numpy(buf.copy()).to("cuda:0")
    with pytest.raises(NbgError):
        mg.group_by(d, n)
    r = mg.group_by(d, n, group=False, swap_macs=False)
    torch_cuda.cuda.synchronize()
    exp = orc.classify(buf.copy(), n, orc.lut_build(names, 655373), stride=64, fixed_len=60, swap=False)
    np.testing.assert_array_equal(r.backend.view(torch_cuda.int16).cpu().numpy().view(np.uint16), exp)
    mg.close()


def test_defer_group_split(torch_cuda, mg65):
    """NBG_DEFER_GROUP + nbg_maglev_finish_group == one combined call."""
    from netbricks_amd import make_trace

    n = 50000
    buf, _, _ = make_trace(n, 0, seed=31)
    lut = orc.lut_build(NAMES65, 65537)
    exp = _oracle(buf, n, lut, 65, stride=64, fixed_len=60)
    d = torch_cuda.from_numpy(buf.copy()).to("cuda:0")
    r = mg65.group_by(d, n, defer_group=True)
    mg65.finish_group()
    torch_cuda.cuda.synchronize()
    got = (d.cpu().numpy(), r.backend.view(torch_cuda.int16).cpu().numpy().view(np.uint16),
           r.perm.view(torch_cuda.int32).cpu().numpy().view(np.uint32),
           r.counts.view(torch_cuda.int32).cpu().numpy().view(np.uint32))
    _assert_same(got, exp)


def test_golden_packets_fixture(torch_cuda, mg65):
    """The committed golden vectors (tests/golden/packets.npz, made by the Python oracle)."""
    import os

    pk = dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "packets.npz")))
    n = pk["off"].size
    buf = pk["buf"].copy()
    got = _run(torch_cuda, mg65, buf, n, offs=pk["off"], lens=pk["len"])
    np.testing.assert_array_equal(got[1], pk["backend65"])
    np.testing.assert_array_equal(got[2], pk["perm65"])
    np.testing.assert_array_equal(got[3], pk["counts65"])
    for i in range(n):
        ln = min(12, int(pk["len"][i]))
        o = int(pk["off"][i])
        assert got[0][o:o + ln].tobytes() == pk["mac12"][i, :ln].tobytes(), i


def test_golden_lemmy_pcap_host_path(torch_cuda):
    """The reference's macswap fixture (http_lemmy.pcap) through nbg_maglev_classify_host."""
    import json
    import os
    import struct

    from netbricks_amd import Maglev

    gold_dir = os.path.join(os.path.dirname(__file__), "golden")
    data = open(os.path.join(gold_dir, "http_lemmy.pcap"), "rb").read()
    pos, frames = 24, []
    while pos + 16 <= len(data):
        incl = struct.unpack("<IIII", data[pos:pos + 16])[2]
        frames.append(bytearray(data[pos + 16:pos + 16 + incl]))
        pos += 16 + incl
    gold = json.load(open(os.path.join(gold_dir, "lemmy.json")))
    mg = Maglev(["Larry", "Curly", "Moe"], 65537)
    be, perm, counts = mg.group_by_host(frames)
    assert be.tolist() == [g["backend3"] for g in gold]
    assert [f[:12].hex() for f in frames] == [g["swapped_head12"] for g in gold]
    assert counts.tolist() == [8, 7, 0, 0]
    assert perm.tolist() == [0, 2, 3, 6, 8, 10, 11, 14, 1, 4, 5, 7, 9, 12, 13]
    mg.close()


def _mbuf_pool(frames, room=2048):
    """Frames copied into 2-KiB "mbuf" data rooms of one host array: (pool, ptrs u64, lens u16)."""
    pool = np.zeros(max(len(frames), 1) * room, dtype=np.uint8)
    for i, f in enumerate(frames):
        pool[i * room:i * room + len(f)] = np.frombuffer(bytes(f), dtype=np.uint8)
    ptrs = (np.arange(len(frames), dtype=np.uint64) * room + np.uint64(pool.ctypes.data)).astype(np.uint64)
    return pool, ptrs, np.array([len(f) for f in frames], dtype=np.uint16)


def _host_case(kind, seed):
    """Host batches that select each header-window stride: 32 B (frame bytes 8..39 for a direct batch
    whose frames longer than 40 B have IHL <= 5), 48 B (IHL <= 7), 64 B (IHL <= 11), 80 B (IHL up to
    15); all with runts and non-IPv4 frames."""
    from netbricks_amd import make_trace

    rng = np.random.default_rng(seed)
    buf, off, ln = make_trace(3000 + seed, 1, seed=seed)
    frames = [bytearray(buf[o:o + l].tobytes()) for o, l in zip(off, ln)]
    edge = _edge_frames(rng)
    if kind == 32:
        edge = [f for f in edge if len(f) <= 40 or (f[14] & 0xF) <= 5]
    elif kind == 48:
        edge = [f for f in edge if len(f) <= 48 or (f[14] & 0xF) <= 7]
    elif kind == 64:
        edge = [f for f in edge if len(f) <= 48 or (f[14] & 0xF) <= 11]
    frames += edge
    rng.shuffle(frames)
    return frames


def test_host_pipeline_submit_wait(torch_cuda, mg65):
    """nbg_maglev_host_submit / _wait: more batches than staging slots, waits in and out of order,
    every window stride; results and MAC rewrites bit-exact vs the oracle."""
    from netbricks_amd import NBG_HOST_SLOTS  # noqa: F401  (exported constant)

    lut = orc.lut_build(NAMES65, 65537)
    cases = [_host_case(k, s) for s, k in enumerate([48, 64, 80, 32, 48, 64, 80])]
    batches, tickets = [], []
    for frames in cases:
        pool, ptrs, lens = _mbuf_pool(frames)
        out = dict(backend=np.empty(len(frames), np.uint16), perm=np.empty(len(frames), np.uint32),
                   counts=np.empty(66, np.uint32))
        batches.append((frames, pool, ptrs, lens, out))
        tickets.append(mg65.host_submit(ptrs, lens, **out))
        if len(tickets) == 2:
            mg65.host_wait(tickets[1])  # out of order: the first stays in flight
    for t in tickets:
        mg65.host_wait(t)
    for frames, pool, ptrs, lens, out in batches:
        pbuf, poff, pln = _pack([bytearray(f) for f in frames], 64)
        exp = _oracle(pbuf, len(frames), lut, 65, offs=poff, lens=pln)
        np.testing.assert_array_equal(out["backend"], exp[1])
        np.testing.assert_array_equal(out["perm"], exp[2])
        np.testing.assert_array_equal(out["counts"], exp[3])
        for i, (o, l) in enumerate(zip(poff.tolist(), pln.tolist())):
            assert pool[i * 2048:i * 2048 + l].tobytes() == exp[0][o:o + l].tobytes(), i


@pytest.mark.parametrize("kind", [32, 48, 64, 80])
def test_host_pipeline_direct_small_batches(torch_cuda, mg65, kind):
    """Batches of at most 2,048 frames take host_submit's direct path (the small kernel reads the
    staged windows out of pinned memory and stores backend / perm / counts / MAC records there): every
    window stride with runts, IHL options and non-IPv4 frames, three batches in flight, completion
    polled with nbg_maglev_host_query before each wait; bit-exact vs the oracle."""
    lut = orc.lut_build(NAMES65, 65537)
    frames_all = _host_case(kind, 40 + kind)
    batches = []
    for lo, hi in ((0, 2048), (2048, 2048 + 992), (3040, 3072)):
        frames = frames_all[lo:hi]
        pool, ptrs, lens = _mbuf_pool(frames)
        out = dict(backend=np.empty(len(frames), np.uint16), perm=np.empty(len(frames), np.uint32),
                   counts=np.empty(66, np.uint32))
        batches.append((frames, pool, ptrs, lens, out, mg65.host_submit(ptrs, lens, **out)))
    from netbricks_amd._lib import lib

    wins = [lib.nbg_debug_host_win(mg65._h, t) for *_, t in batches]
    if kind == 32:  # the first two batches hold edge frames; every batch is staged at 32 B
        assert wins == [32, 32, 32], wins
    else:  # a longer IP header in a batch stages it from byte 0 at the stride it needs
        assert all(w in (32, 48, 64, 80) for w in wins) and max(wins) >= min(kind, 48), wins
    for *_, t in batches:
        for _ in range(100000):
            if mg65.host_query(t):
                break
        assert mg65.host_query(t)
        mg65.host_wait(t)
    for frames, pool, ptrs, lens, out, _ in batches:
        pbuf, poff, pln = _pack([bytearray(f) for f in frames], 64)
        exp = _oracle(pbuf, len(frames), lut, 65, offs=poff, lens=pln)
        np.testing.assert_array_equal(out["backend"], exp[1])
        np.testing.assert_array_equal(out["perm"], exp[2])
        np.testing.assert_array_equal(out["counts"], exp[3])
        for i, (o, l) in enumerate(zip(poff.tolist(), pln.tolist())):
            assert pool[i * 2048:i * 2048 + l].tobytes() == exp[0][o:o + l].tobytes(), i


def test_host_pipeline_large_batch(torch_cuda, mg65):
    """A 300k-packet host batch (the parallel gather and write-back) through submit/wait."""
    from netbricks_amd import make_trace

    n = 300_000
    buf, off, ln = make_trace(n, 0, seed=77)
    room = 128
    pool = np.zeros(n * room, dtype=np.uint8)
    pool.reshape(n, room)[:, :64] = buf.reshape(n, 64)
    ptrs = (np.arange(n, dtype=np.uint64) * room + np.uint64(pool.ctypes.data)).astype(np.uint64)
    lens = np.full(n, 60, dtype=np.uint16)
    out = dict(backend=np.empty(n, np.uint16), perm=np.empty(n, np.uint32), counts=np.empty(66, np.uint32))
    mg65.host_wait(mg65.host_submit(ptrs, lens, **out))
    exp = _oracle(buf, n, orc.lut_build(NAMES65, 65537), 65, stride=64, fixed_len=60)
    np.testing.assert_array_equal(out["backend"], exp[1])
    np.testing.assert_array_equal(out["perm"], exp[2])
    np.testing.assert_array_equal(out["counts"], exp[3])
    np.testing.assert_array_equal(pool.reshape(n, room)[:, :60], exp[0].reshape(n, 64)[:, :60])


def test_host_pipeline_many_handles_and_streams(torch_cuda):
    """Three handles with interleaved submits (batches of 1 to 3000 frames, waits out of order)
    while device batches run on torch streams of the same process: the host path keeps each
    batch's copies and kernels in order with no cross-stream events to lose."""
    import netbricks_amd as nb
    from netbricks_amd import make_trace

    lut = orc.lut_build(NAMES65, 65537)
    handles = [nb.Maglev(NAMES65, 65537) for _ in range(3)]
    streams = [torch_cuda.cuda.Stream() for _ in range(4)]
    dev_bufs = [torch_cuda.from_numpy(make_trace(65536, 0, seed=500 + k)[0]).cuda() for k in range(4)]
    rng = np.random.default_rng(5)
    pending = []
    for k in range(24):
        n = int(rng.choice([1, 32, 100, 1000, 3000]))
        buf, off, ln = make_trace(n, 1, seed=600 + k)
        frames = [bytearray(buf[o:o + l].tobytes()) for o, l in zip(off, ln)]
        pool, ptrs, lens = _mbuf_pool(frames)
        out = dict(backend=np.empty(n, np.uint16), perm=np.empty(n, np.uint32), counts=np.empty(66, np.uint32))
        h = handles[k % 3]
        pending.append((h, h.host_submit(ptrs, lens, **out), frames, pool, out))
        # device work of another handle on other streams meanwhile
        j = k % 4
        handles[(k + 1) % 3].group_by(dev_bufs[j], 65536, stream=streams[j].cuda_stream)
        if k % 5 == 4:  # some waits early, out of order
            h2, t2, *_ = pending[-2]
            h2.host_wait(t2)
    for h, t, *_ in reversed(pending):
        h.host_wait(t)
    torch_cuda.cuda.synchronize()
    for h, t, frames, pool, out in pending:
        pbuf, poff, pln = _pack([bytearray(f) for f in frames], 64)
        exp = _oracle(pbuf, len(frames), lut, 65, offs=poff, lens=pln)
        np.testing.assert_array_equal(out["backend"], exp[1])
        np.testing.assert_array_equal(out["perm"], exp[2])
        np.testing.assert_array_equal(out["counts"], exp[3])
        for i, (o, l) in enumerate(zip(poff.tolist(), pln.tolist())):
            assert pool[i * 2048:i * 2048 + l].tobytes() == exp[0][o:o + l].tobytes(), i
    for h in handles:
        h.close()
