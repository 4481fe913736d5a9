"""The persistent RX ring (nbg_ring_*, include/nbgpu.h): one resident classify kernel takes batches as
they are posted.  Every batch's backend[] (and in-place MAC swap) is bit-exact against the C oracle
run on that batch alone, over consecutive batches of every size class (one packet, partial tiles,
partial units, 1M), more batches than ring slots (posts wait for free slots), the idle timeout (the
kernel's own exit) and direct calls on the handle after the ring stopped.
Never torch.cuda.synchronize() while a ring runs: it would wait for the resident kernel.
Reference semantics: test/maglev/src/nf.rs:92-106 per packet; receive_batch.rs:26,52-61 (the RX loop).
"""
import time

import numpy as np
import pytest

import orc

pytestmark = pytest.mark.gpu

NAMES65 = [f"backend-{i}" for i in range(65)]


def _expect(buf, n, lut, swap):
    ref = buf.copy()
    be = orc.classify(ref, n, lut, stride=64, fixed_len=60, swap=swap)
    return be, ref


def _got(torch, t):
    return t.view(torch.int16).cpu().numpy().view(np.uint16)


@pytest.mark.parametrize("swap", [False, True])
def test_ring_consecutive_batches(torch_cuda, swap):
    torch = torch_cuda
    import netbricks_amd as nb

    lut = orc.lut_build(NAMES65, 65537)
    mg = nb.Maglev(NAMES65, 65537)
    sizes = [1, 100, 511, 512, 513, 4097, 65543, 300000, 1 << 20, 7, 262144]
    bufs = [nb.make_trace(n, 0, seed=400 + i)[0] for i, n in enumerate(sizes)]
    d = [torch.from_numpy(b.copy()).cuda() for b in bufs]
    outs = [torch.full((n,), 0x7777, dtype=torch.int16, device="cuda").view(torch.uint16) for n in sizes]
    torch.cuda.synchronize()
    with mg.ring(swap_macs=swap) as ring:
        tickets = [ring.post(d[i], n, outs[i]) for i, n in enumerate(sizes)]
        assert tickets == list(range(len(sizes)))
        ring.wait(tickets[-1])
        assert ring.poll() == len(sizes)
        for i, n in enumerate(sizes):
            be, ref = _expect(bufs[i], n, lut, swap)
            np.testing.assert_array_equal(_got(torch, outs[i]), be, err_msg=f"batch {i} ({n} packets)")
            np.testing.assert_array_equal(d[i].cpu().numpy(), ref, err_msg=f"batch {i} bytes")
    mg.check()
    mg.close()


def test_ring_more_batches_than_slots(torch_cuda):
    """40 batches through 16 slots (posts wait for the oldest), each waited for in post order."""
    torch = torch_cuda
    import netbricks_amd as nb

    lut = orc.lut_build(NAMES65, 65537)
    mg = nb.Maglev(NAMES65, 65537)
    rng = np.random.default_rng(7)
    sizes = [int(x) for x in rng.integers(1, 200000, 40)]
    bufs = [nb.make_trace(n, 0, seed=500 + i)[0] for i, n in enumerate(sizes)]
    d = [torch.from_numpy(b).cuda() for b in bufs]
    outs = [torch.empty(n, dtype=torch.uint16, device="cuda") for n in sizes]
    torch.cuda.synchronize()
    with mg.ring() as ring:
        tickets = [ring.post(d[i], n, outs[i]) for i, n in enumerate(sizes)]
        for t in tickets:
            ring.wait(t)
    for i, n in enumerate(sizes):
        be, _ = _expect(bufs[i], n, lut, False)
        np.testing.assert_array_equal(_got(torch, outs[i]), be, err_msg=f"batch {i} ({n} packets)")
    mg.close()


@pytest.mark.parametrize("swap", [False, True])
def test_ring_post_burst(torch_cuda, swap):
    """RX bursts (nbg_ring_post_burst): 102 batches offered 24 at a time; each call posts what fits
    the 64 slots (the rest is offered again), tickets stay consecutive, and every batch is bit-exact."""
    torch = torch_cuda
    import netbricks_amd as nb

    lut = orc.lut_build(NAMES65, 65537)
    mg = nb.Maglev(NAMES65, 65537)
    rng = np.random.default_rng(11)
    sizes = [int(x) for x in rng.integers(1, 40000, 100)] + [131072, 131072]
    bufs = [nb.make_trace(n, 0, seed=800 + i)[0] for i, n in enumerate(sizes)]
    d = [torch.from_numpy(b.copy()).cuda() for b in bufs]
    outs = [torch.empty(n, dtype=torch.uint16, device="cuda") for n in sizes]
    torch.cuda.synchronize()
    with mg.ring(swap_macs=swap) as ring:
        nxt = 0
        while nxt < len(sizes):
            offer = [(d[i], sizes[i], outs[i]) for i in range(nxt, min(nxt + 24, len(sizes)))]
            k, first = ring.post_burst(offer)
            assert first == nxt
            nxt += k
            if k == 0:  # the ring is full: wait for the oldest outstanding batch
                ring.wait(nxt - 64)
        ring.wait(len(sizes) - 1)
        with pytest.raises(nb.NbgError):
            ring.post_burst([(d[-1][8:], 10, outs[-1])])  # misaligned packet buffer
    for i, n in enumerate(sizes):
        be, ref = _expect(bufs[i], n, lut, swap)
        np.testing.assert_array_equal(_got(torch, outs[i]), be, err_msg=f"batch {i} ({n} packets)")
        np.testing.assert_array_equal(d[i].cpu().numpy(), ref, err_msg=f"batch {i} bytes")
    mg.close()


@pytest.mark.parametrize("swap", [False, True])
def test_ring_group(torch_cuda, swap):
    """nbg_ring_group: every completed batch grouped on side streams while the ring keeps running
    (the ring kernel stays resident), perm / counts bit-exact against the oracle's grouping of that
    batch; sizes from one packet to 1M (direct scan) and 2.1M (several chunks per partition)."""
    torch = torch_cuda
    import netbricks_amd as nb

    lut = orc.lut_build(NAMES65, 65537)
    mg = nb.Maglev(NAMES65, 65537)
    sizes = [1, 700, 4096, 4097, 131072, 1 << 20, 300001, 2_100_000, 65536]
    bufs = [nb.make_trace(n, 0, seed=900 + i)[0] for i, n in enumerate(sizes)]
    d = [torch.from_numpy(b.copy()).cuda() for b in bufs]
    outs = [torch.empty(n, dtype=torch.uint16, device="cuda") for n in sizes]
    perms = [torch.empty(n, dtype=torch.uint32, device="cuda") for n in sizes]
    counts = [torch.zeros(66, dtype=torch.uint32, device="cuda") for _ in sizes]
    # five side streams round-robin: four own a scratch set, the fifth takes one over
    sides = [torch.cuda.Stream() for _ in range(5)]
    torch.cuda.synchronize()
    with mg.ring(swap_macs=swap) as ring:
        for i, n in enumerate(sizes):
            t = ring.post(d[i], n, outs[i])
            if i:  # group each batch once complete, while the next one is still running
                ring.wait(t - 1)
                ring.group(t - 1, perms[i - 1], counts[i - 1], stream=sides[(i - 1) % 5])
        ring.wait(len(sizes) - 1)
        ring.group(len(sizes) - 1, perms[-1], counts[-1], stream=sides[(len(sizes) - 1) % 5])
        for st in sides:
            st.synchronize()
        with pytest.raises(nb.NbgError):  # not complete: not posted
            ring.group(len(sizes), perms[0], counts[0], stream=sides[0])
    for i, n in enumerate(sizes):
        be, _ = _expect(bufs[i], n, lut, swap)
        exp_perm, exp_cnt = orc.group(be, 65)
        np.testing.assert_array_equal(_np32(torch, perms[i]), exp_perm, err_msg=f"batch {i} ({n}) perm")
        np.testing.assert_array_equal(_np32(torch, counts[i]), exp_cnt, err_msg=f"batch {i} ({n}) counts")
    mg.close()


def _np32(torch, t):
    return t.view(torch.int32).cpu().numpy().view(np.uint32)


def test_ring_post_while_running(torch_cuda):
    """Batches posted one at a time while the kernel is idle between them (each post wakes a polling
    block), then a burst; the same handle's direct calls work after stop()."""
    torch = torch_cuda
    import netbricks_amd as nb

    lut = orc.lut_build(NAMES65, 65537)
    mg = nb.Maglev(NAMES65, 65537)
    n = 131072
    bufs = [nb.make_trace(n, 0, seed=600 + i)[0] for i in range(6)]
    d = [torch.from_numpy(b).cuda() for b in bufs]
    outs = [torch.empty(n, dtype=torch.uint16, device="cuda") for _ in range(6)]
    torch.cuda.synchronize()
    ring = mg.ring()
    try:
        for i in range(3):
            time.sleep(0.02)
            ring.wait(ring.post(d[i], n, outs[i]))
        last = [ring.post(d[i], n, outs[i]) for i in range(3, 6)][-1]
        ring.wait(last)
    finally:
        ring.stop()
    for i in range(6):
        np.testing.assert_array_equal(_got(torch, outs[i]), _expect(bufs[i], n, lut, False)[0])
    import ctypes as C

    from netbricks_amd._lib import lib

    ms = C.c_float()
    assert lib.nbg_ring_kernel_ms(mg._h, C.byref(ms)) == 0 and ms.value > 0  # the kernel's HIP-event time
    # a second and third ring reuse the handle's ring buffers and stream
    for rep in range(2):
        outs[0].zero_()
        with mg.ring(swap_macs=False) as ring:
            ring.wait(ring.post(d[0], n, outs[0]))
        np.testing.assert_array_equal(_got(torch, outs[0]), _expect(bufs[0], n, lut, False)[0], err_msg=f"rerun {rep}")
    r = mg.group_by(d[0], n, swap_macs=False)  # the handle after the ring
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_got(torch, r.backend), _expect(bufs[0], n, lut, False)[0])
    mg.close()


def test_ring_idle_timeout_ends_kernel(torch_cuda):
    """With no post for idle_ms the kernel ends by itself; the next post reports it; a new ring on
    the same handle works."""
    torch = torch_cuda
    import netbricks_amd as nb

    lut = orc.lut_build(NAMES65, 65537)
    mg = nb.Maglev(NAMES65, 65537)
    n = 5000
    buf = nb.make_trace(n, 0, seed=700)[0]
    d = torch.from_numpy(buf).cuda()
    out = torch.empty(n, dtype=torch.uint16, device="cuda")
    torch.cuda.synchronize()
    ring = mg.ring(idle_ms=50)
    ring.wait(ring.post(d, n, out))
    time.sleep(0.5)
    with pytest.raises(nb.NbgError) as e:
        ring.post(d, n, out)
    assert e.value.code == -110
    ring.stop()  # the kernel already ended; every posted batch was complete
    np.testing.assert_array_equal(_got(torch, out), _expect(buf, n, lut, False)[0])
    out.zero_()
    with mg.ring() as ring2:
        ring2.wait(ring2.post(d, n, out))
    np.testing.assert_array_equal(_got(torch, out), _expect(buf, n, lut, False)[0])
    mg.close()


def test_ring_refuses_unsupported(torch_cuda):
    torch = torch_cuda
    import netbricks_amd as nb

    wide = nb.Maglev([f"b{i}" for i in range(300)], 65537)  # u16 LUT
    with pytest.raises(nb.NbgError):
        wide.ring()
    wide.close()
    mg = nb.Maglev(NAMES65, 65537)
    with pytest.raises(nb.NbgError):
        mg.ring(stride=48)
    with mg.ring() as ring:
        with pytest.raises(nb.NbgError):
            mg.ring()  # one ring per handle
        d = torch.zeros(64 * 10 + 8, dtype=torch.uint8, device="cuda")
        out = torch.empty(10, dtype=torch.uint16, device="cuda")
        with pytest.raises(nb.NbgError):
            ring.post(d[8:], 10, out)  # misaligned packet buffer
    mg.close()
