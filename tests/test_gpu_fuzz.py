"""GPU parity over seeded random combinations of the C-ABI's options, against the C oracle.

Each case draws a table (1..5000 backends, prime sizes 7..655373), a layout (fixed slots at a
16-B-aligned or unaligned stride, or descriptors over an IMIX trace, optionally with owned
windows), a batch size (1 .. 300k, so the small, tile-per-wave and streaming kernels are all
reached) and the flags (swap or not, records, grouping or backend only, LDS LUT, streaming
descriptors, deferred grouping), perturbs the trace (runts, IHL 0..15, non-IPv4 ethertypes,
unaligned starts), and checks backend[], perm, counts, the packet bytes and the records bit-exact.
The chain cases (lpm -> maglev) draw random route sets over the trace's source space (prefix
lengths 0..32, so tbl_long is exercised), lpm_groups 1..4 and the same layouts and kernels, and
check gate[], backend[], perm, counts and the unchanged packets.  The cases are fixed by the seed,
so a failure names a reproducible case.  Reference semantics:
test/maglev/src/nf.rs:78-81,92-108; framework/src/operators/group_by.rs:46-51;
test/lpm/src/nf.rs:49-98,205-223.
"""
import numpy as np
import pytest

import orc

pytestmark = pytest.mark.gpu

PRIMES = [7, 1009, 65537, 131071, 655373]


def _cases(count=120, seed=20261016):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(count):
        m = int(rng.choice(PRIMES))
        nb = int(rng.choice([1, 2, 3, 65, 256, 257, 1000, 5000]))
        nb = min(nb, m - 1)
        layout = str(rng.choice(["fixed64", "fixed_stride", "desc", "desc_owned"]))
        size_class = rng.random()
        if size_class < 0.4:
            n = int(rng.integers(1, 2100))
        elif size_class < 0.7:
            n = int(rng.integers(2100, 80000))
        else:
            n = int(rng.integers(262144, 300000))
        swap = bool(rng.random() < 0.7)
        records = swap and bool(rng.random() < 0.3)
        group = bool(rng.random() < 0.85)
        lut_lds = bool(rng.random() < 0.3)
        stream_desc = layout.startswith("desc") and bool(rng.random() < 0.5)
        if stream_desc and rng.random() < 0.7:
            layout = "desc_owned"  # the streaming descriptor kernel takes owned windows only
        defer = group and bool(rng.random() < 0.2)
        out.append(pytest.param(i, m, nb, layout, n, swap, records, group, lut_lds, stream_desc, defer,
                                id=f"{i}-{layout}-n{n}-nb{nb}-m{m}-s{int(swap)}r{int(records)}g{int(group)}"
                                   f"l{int(lut_lds)}d{int(stream_desc)}f{int(defer)}"))
    return out


def _perturb_headers(buf, off, ln, rng, frame_ok):
    """IHL, ethertype and protocol changes inside frames (lengths unchanged)."""
    n = off.size
    o = off.astype(np.int64)
    ihl = (rng.random(n) < 0.01) & (ln > 14) & frame_ok
    buf[o[ihl] + 14] = (0x40 | rng.integers(0, 16, int(ihl.sum()))).astype(np.uint8)
    et = (rng.random(n) < 0.005) & (ln > 13) & frame_ok
    buf[o[et] + 12] = 0x86
    buf[o[et] + 13] = 0xDD
    pr = (rng.random(n) < 0.01) & (ln > 23) & frame_ok
    buf[o[pr] + 23] = rng.integers(0, 256, int(pr.sum())).astype(np.uint8)


def _layout(layout, n, seed, rng):
    """(buf, offsets or None, lens or None, stride, frame_len, owned, every frame's offset, length)."""
    import netbricks_amd as nb_

    if layout in ("fixed64", "fixed_stride"):
        stride = 64 if layout == "fixed64" else int(rng.choice([72, 80, 96, 128, 100]))
        frame_len = 60 if layout == "fixed64" else int(rng.choice([14, 40, 60, min(stride, 90)]))
        src, soff, sln = nb_.make_trace(n, 0, seed=seed)
        buf = np.zeros(n * stride + 64, dtype=np.uint8)
        w = min(frame_len, 60)
        for k in range(w):
            buf[np.arange(n, dtype=np.int64) * stride + k] = src[soff.astype(np.int64) + k]
        off = (np.arange(n, dtype=np.int64) * stride).astype(np.uint32)
        ln = np.full(n, frame_len, dtype=np.uint16)
        _perturb_headers(buf, off, ln, rng, np.ones(n, dtype=bool))
        return buf, None, None, stride, frame_len, False, off, ln
    buf, off, ln = nb_.make_trace(n, 1, seed=seed)
    off = off.copy()
    ln = ln.copy()
    _perturb_headers(buf, off, ln, rng, np.ones(n, dtype=bool))
    runt = rng.random(n) < 0.005
    ln[runt] = rng.integers(0, 64, int(runt.sum()))
    owned = layout == "desc_owned"
    # shifted starts: inside frames of >= 128 B, so an owned window stays inside its frame's room
    mis = (rng.random(n) < 0.01) & (ln >= 128)
    s = rng.integers(1, 16 if owned else 60, int(mis.sum())).astype(np.uint32)
    off[mis] += s
    ln[mis] -= s.astype(np.uint16)
    return buf, off, ln, 64, 60, owned, off, ln


@pytest.mark.parametrize("i,m,nb,layout,n,swap,records,group,lut_lds,stream_desc,defer", _cases())
def test_fuzz_options(torch_cuda, i, m, nb, layout, n, swap, records, group, lut_lds, stream_desc, defer):
    import netbricks_amd as nb_

    torch = torch_cuda
    rng = np.random.default_rng(1000 + i)
    names = [f"f{i}-{k}" for k in range(nb)]
    buf, offs, lens, stride, frame_len, owned, all_off, all_len = _layout(layout, n, 77 + i, rng)
    lut = orc.lut_build(names, m)
    ref = buf.copy()
    if offs is None:
        be = orc.classify(ref, n, lut, stride=stride, fixed_len=frame_len, swap=swap)
    else:
        be = orc.classify(ref, n, lut, offs=offs, lens=lens, swap=swap)
    perm, counts = orc.group(be, nb)

    mg = nb_.Maglev(names, m)
    dev = torch.device("cuda:0")
    d = torch.from_numpy(buf.copy()).to(dev)
    d_off = None if offs is None else torch.from_numpy(offs.astype(np.uint32).view(np.int32)).to(dev).view(torch.uint32)
    d_len = None if lens is None else torch.from_numpy(lens.astype(np.uint16).view(np.int16)).to(dev).view(torch.uint16)
    mac = torch.zeros(max(n, 1) * 12, dtype=torch.uint8, device=dev) if records else None
    r = mg.group_by(d, n, stride=stride, frame_len=frame_len, offsets=d_off, lens=d_len, swap_macs=swap, group=group,
                    lut_lds=lut_lds, owned_windows=owned, stream_desc=stream_desc, defer_group=defer, mac_out=mac)
    if defer:
        mg.finish_group()
    torch.cuda.synchronize()
    mg.check()
    np.testing.assert_array_equal(r.backend.view(torch.int16).cpu().numpy().view(np.uint16), be)
    if group:
        np.testing.assert_array_equal(r.counts.view(torch.int32).cpu().numpy().view(np.uint32), counts)
        np.testing.assert_array_equal(r.perm.view(torch.int32).cpu().numpy().view(np.uint32)[:n], perm[:n])
    got = d.cpu().numpy()
    if records:
        np.testing.assert_array_equal(got, buf)  # the swap goes to the records, not the packets
        rec = mac.cpu().numpy()[:n * 12].reshape(n, 12)
        o = all_off.astype(np.int64)
        has = all_len >= 14
        idx = o[has, None] + np.arange(12)[None, :]
        np.testing.assert_array_equal(rec[has], ref[idx])
    else:
        np.testing.assert_array_equal(got, ref)
    mg.close()


def _chain_cases(count=40, seed=61):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(count):
        m = int(rng.choice(PRIMES))
        nb = min(int(rng.choice([1, 3, 65, 256, 1000])), m - 1)
        layout = str(rng.choice(["fixed64", "desc", "desc_owned"]))
        size_class = rng.random()
        n = int(rng.integers(1, 2100) if size_class < 0.4 else
                (rng.integers(2100, 80000) if size_class < 0.7 else rng.integers(262144, 300000)))
        n_routes = int(rng.integers(1, 300))
        groups = int(rng.integers(1, 5))
        lut_lds = bool(rng.random() < 0.3)
        stream_desc = layout == "desc_owned" and bool(rng.random() < 0.6)
        group = bool(rng.random() < 0.85)
        defer = group and bool(rng.random() < 0.2)
        out.append(pytest.param(i, m, nb, layout, n, n_routes, groups, lut_lds, stream_desc, group, defer,
                                id=f"{i}-{layout}-n{n}-nb{nb}-m{m}-r{n_routes}-g{groups}"
                                   f"l{int(lut_lds)}d{int(stream_desc)}g{int(group)}f{int(defer)}"))
    return out


def _routes(rng, count):
    """Random routes over 10/8 and 172.16/12 (the trace's rewritten sources), lengths 0..32."""
    out = []
    for _ in range(count):
        ln = int(rng.choice([0, 8, 12, 16, 20, 24, 24, 25, 28, 30, 32, 32]))
        base = 0x0A000000 if rng.random() < 0.75 else 0xAC100000
        span = (1 << 24) if base == 0x0A000000 else (1 << 20)
        ip = base | int(rng.integers(0, span))
        ip &= (0xFFFFFFFF << (32 - ln)) & 0xFFFFFFFF if ln else 0
        out.append([f"{ip >> 24}.{(ip >> 16) & 255}.{(ip >> 8) & 255}.{ip & 255}", ln, int(rng.integers(0, 5))])
    return out


@pytest.mark.parametrize("i,m,nb,layout,n,n_routes,groups,lut_lds,stream_desc,group,defer", _chain_cases())
def test_fuzz_chain(torch_cuda, i, m, nb, layout, n, n_routes, groups, lut_lds, stream_desc, group, defer):
    import netbricks_amd as nb_
    from netbricks_amd import chain_lpm_maglev
    from netbricks_amd.lpm import Lpm

    torch = torch_cuda
    rng = np.random.default_rng(5000 + i)
    names = [f"c{i}-{k}" for k in range(nb)]
    buf, offs, lens, stride, frame_len, owned, all_off, all_len = _layout(layout, n, 300 + i, rng)
    # sources into the route space (only where the frame holds the address)
    hi = rng.integers(0, 4, n)
    ip = np.where(hi > 0, 0x0A000000 | rng.integers(0, 1 << 24, n), 0xAC100000 | rng.integers(0, 1 << 20, n))
    b = ip.astype(">u4").view(np.uint8).reshape(n, 4)
    ok = all_len >= 30
    o = all_off.astype(np.int64)[ok]
    for k in range(4):
        buf[o + 26 + k] = b[ok, k]
    routes = _routes(rng, n_routes)
    rc, t24, tl = orc.lpm_build(routes)
    assert rc == 0
    okw = dict(stride=stride, fixed_len=frame_len) if offs is None else dict(offs=offs, lens=lens)
    eg, eb = orc.chain_classify(buf, n, t24, tl, orc.lut_build(names, m), lpm_groups=groups, **okw)
    perm, counts = orc.group(eb, nb)

    mg = nb_.Maglev(names, m)
    lpm = Lpm(routes)
    dev = torch.device("cuda:0")
    d = torch.from_numpy(buf.copy()).to(dev)
    kw = dict(stride=stride, frame_len=frame_len)
    if offs is not None:
        kw["offsets"] = torch.from_numpy(offs.astype(np.uint32).view(np.int32)).to(dev).view(torch.uint32)
        kw["lens"] = torch.from_numpy(lens.astype(np.uint16).view(np.int16)).to(dev).view(torch.uint16)
    r = chain_lpm_maglev(mg, lpm, d, n, lpm_groups=groups, owned_windows=owned, lut_lds=lut_lds,
                         stream_desc=stream_desc, group=group, defer_group=defer, **kw)
    if defer:
        mg.finish_group()
    torch.cuda.synchronize()
    mg.check()
    np.testing.assert_array_equal(r.gate.view(torch.int16).cpu().numpy().view(np.uint16)[:n], eg)
    np.testing.assert_array_equal(r.backend.view(torch.int16).cpu().numpy().view(np.uint16)[:n], eb)
    if group:
        np.testing.assert_array_equal(r.counts.view(torch.int32).cpu().numpy().view(np.uint32), counts)
        np.testing.assert_array_equal(r.perm.view(torch.int32).cpu().numpy().view(np.uint32)[:n], perm[:n])
    np.testing.assert_array_equal(d.cpu().numpy(), buf)
    lpm.close()
    mg.close()
