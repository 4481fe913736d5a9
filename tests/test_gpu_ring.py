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


def _slices(rng, count, lo, hi):
    """`count` batch sizes in [lo, hi) laid out back to back in one trace, every batch starting on a
    multiple of 8 packets (16-B aligned backend slices): [(start, n)], total packets."""
    out, pos = [], 0
    for n in rng.integers(lo, hi, count):
        out.append((pos, int(n)))
        pos += (int(n) + 7) & ~7
    return out, pos


@pytest.mark.parametrize("swap", [False, True])
def test_ring_1200_batches_wraparound(torch_cuda, swap):
    """1,200 batches (about 19 wraps of the 64 slots and of the relay's descriptor replicas), posted in
    RX bursts as slots free up: slices of one 10M-packet trace, each classified once, so one oracle
    pass over the trace checks every batch's backend[] and (in place) its bytes."""
    torch = torch_cuda
    import netbricks_amd as nb

    lut = orc.lut_build(NAMES65, 65537)
    mg = nb.Maglev(NAMES65, 65537)
    rng = np.random.default_rng(1200 + swap)
    batches, total = _slices(rng, 1200, 1, 16000)
    buf = nb.make_trace(total, 0, seed=4242 + swap)[0]
    d = torch.from_numpy(buf.copy()).cuda()
    out = torch.full((total,), 0x7777, dtype=torch.int16, device="cuda").view(torch.uint16)
    torch.cuda.synchronize()
    with mg.ring(swap_macs=swap) as ring:
        nxt = 0
        while nxt < len(batches):
            offer = [(d[s * 64:], n, out[s:]) for s, n in batches[nxt:nxt + 40]]
            k, first = ring.post_burst(offer)
            assert first == nxt
            nxt += k
            if k == 0:
                ring.wait(nxt - 64)
        ring.wait(len(batches) - 1)
        assert ring.poll() == len(batches)
    got = _got(torch, out)
    ref = buf.copy()
    be = orc.classify(ref, total, lut, stride=64, fixed_len=60, swap=swap)
    covered = np.zeros(total, dtype=bool)
    for s, n in batches:
        covered[s:s + n] = True
    np.testing.assert_array_equal(got[covered], be[covered])
    assert (got[~covered] == 0x7777).all()  # the alignment gaps are no batch's packets
    byte_mask = np.repeat(covered, 64)
    now = d.cpu().numpy()
    np.testing.assert_array_equal(now[byte_mask], ref[byte_mask])
    np.testing.assert_array_equal(now[~byte_mask], buf[~byte_mask])
    mg.close()


def test_ring_group_gated_mixed_streams(torch_cuda):
    """nbg_ring_group enqueued right after each post, before the batch is complete (a gate kernel
    waits on the stream), alternating torch's default stream (the null stream: ADVICE r3) with side
    streams so that the scratch sets change owners; perm / counts bit-exact for every batch."""
    torch = torch_cuda
    import netbricks_amd as nb

    lut = orc.lut_build(NAMES65, 65537)
    mg = nb.Maglev(NAMES65, 65537)
    sizes = [131072, 4097, 1 << 20, 65536, 300001, 777, 131072, 262144, 1, 524288, 9000, 131072]
    bufs = [nb.make_trace(n, 0, seed=1300 + i)[0] for i, n in enumerate(sizes)]
    d = [torch.from_numpy(b.copy()).cuda() for b in bufs]
    outs = [torch.empty(n, dtype=torch.uint16, device="cuda") for n in sizes]
    perms = [torch.empty(n, dtype=torch.uint32, device="cuda") for n in sizes]
    counts = [torch.zeros(66, dtype=torch.uint32, device="cuda") for _ in sizes]
    sides = [torch.cuda.Stream() for _ in range(5)]
    torch.cuda.synchronize()
    with mg.ring(swap_macs=True) as ring:
        for i, n in enumerate(sizes):
            t = ring.post(d[i], n, outs[i])
            st = None if i % 3 == 0 else sides[i % 5]  # None: torch's current (default) stream
            ring.group(t, perms[i], counts[i], stream=st)
        ring.wait(len(sizes) - 1)
        for st in sides:
            st.synchronize()
        torch.cuda.current_stream().synchronize()  # the null stream's groups (the ring is on its own stream)
    for i, n in enumerate(sizes):
        be, _ = _expect(bufs[i], n, lut, True)
        np.testing.assert_array_equal(_got(torch, outs[i]), be, err_msg=f"batch {i} ({n}) backend")
        exp_perm, exp_cnt = orc.group(be, 65)
        np.testing.assert_array_equal(_np32(torch, perms[i]), exp_perm, err_msg=f"batch {i} ({n}) perm")
        np.testing.assert_array_equal(_np32(torch, counts[i]), exp_cnt, err_msg=f"batch {i} ({n}) counts")
    mg.close()


@pytest.mark.parametrize("n_queues", [2, 4])
def test_ring_queues_interleaved(torch_cuda, n_queues):
    """Several RX queues on one ring (nbg_ring_queue_*): each queue's tickets run 0, 1, 2, ...
    whatever the interleaving, its completion count and grouping are its own, and every batch is
    bit-exact against the oracle run on that batch alone (120 batches through the 64 shared slots)."""
    torch = torch_cuda
    import netbricks_amd as nb

    lut = orc.lut_build(NAMES65, 65537)
    mg = nb.Maglev(NAMES65, 65537)
    rng = np.random.default_rng(50 + n_queues)
    per_q = 120 // n_queues
    sizes = [[int(x) for x in rng.integers(1, 70000, per_q)] for _ in range(n_queues)]
    bufs = [[nb.make_trace(n, 0, seed=2000 + 100 * q + i)[0] for i, n in enumerate(sz)] for q, sz in enumerate(sizes)]
    d = [[torch.from_numpy(b.copy()).cuda() for b in bq] for bq in bufs]
    outs = [[torch.empty(n, dtype=torch.uint16, device="cuda") for n in sz] for sz in sizes]
    perms = [[torch.empty(n, dtype=torch.uint32, device="cuda") for n in sz] for sz in sizes]
    counts = [[torch.zeros(66, dtype=torch.uint32, device="cuda") for _ in sz] for sz in sizes]
    sides = [torch.cuda.Stream() for _ in range(n_queues)]
    torch.cuda.synchronize()
    with mg.ring(swap_macs=True) as ring:
        qs = [ring.queue() for _ in range(n_queues)]
        order = rng.permutation(np.repeat(np.arange(n_queues), per_q))  # an arbitrary interleaving
        nxt = [0] * n_queues
        for q in order:
            i = nxt[q]
            t = qs[q].post(d[q][i], sizes[q][i], outs[q][i])
            assert t == i  # per-queue tickets
            qs[q].group(t, perms[q][i], counts[q][i], stream=sides[q])
            nxt[q] += 1
        for q in range(n_queues):
            qs[q].wait(per_q - 1)
            assert qs[q].poll() == per_q
        assert ring.poll() == n_queues * per_q
        for st in sides:
            st.synchronize()
        qs[0].close()
        with pytest.raises(RuntimeError):
            qs[0].post(d[0][0], sizes[0][0], outs[0][0])
    for q in range(n_queues):
        for i, n in enumerate(sizes[q]):
            be, ref = _expect(bufs[q][i], n, lut, True)
            np.testing.assert_array_equal(_got(torch, outs[q][i]), be, err_msg=f"queue {q} batch {i} backend")
            np.testing.assert_array_equal(d[q][i].cpu().numpy(), ref, err_msg=f"queue {q} batch {i} bytes")
            exp_perm, exp_cnt = orc.group(be, 65)
            np.testing.assert_array_equal(_np32(torch, perms[q][i]), exp_perm, err_msg=f"queue {q} batch {i} perm")
            np.testing.assert_array_equal(_np32(torch, counts[q][i]), exp_cnt, err_msg=f"queue {q} batch {i} counts")
    mg.close()


def test_ring_queues_from_threads(torch_cuda):
    """Four producer threads, one RX queue each, posting and waiting concurrently (the ring's mutex);
    every batch bit-exact."""
    import threading

    torch = torch_cuda
    import netbricks_amd as nb

    lut = orc.lut_build(NAMES65, 65537)
    mg = nb.Maglev(NAMES65, 65537)
    nq, per_q, n = 4, 40, 50000
    bufs = [[nb.make_trace(n, 0, seed=3000 + 100 * q + i)[0] for i in range(per_q)] for q in range(nq)]
    d = [[torch.from_numpy(b).cuda() for b in bq] for bq in bufs]
    outs = [[torch.empty(n, dtype=torch.uint16, device="cuda") for _ in range(per_q)] for _ in range(nq)]
    torch.cuda.synchronize()
    errs = []
    with mg.ring() as ring:
        qs = [ring.queue() for _ in range(nq)]

        def producer(q):
            try:
                for i in range(per_q):
                    assert qs[q].post(d[q][i], n, outs[q][i]) == i
                    if i % 7 == 6:
                        qs[q].wait(i - 3)
                qs[q].wait(per_q - 1)
            except Exception as e:  # noqa: BLE001
                errs.append(e)

        th = [threading.Thread(target=producer, args=(q,)) for q in range(nq)]
        for t in th:
            t.start()
        for t in th:
            t.join(60)
        assert not errs, errs
        assert ring.poll() == nq * per_q
    for q in range(nq):
        for i in range(per_q):
            np.testing.assert_array_equal(_got(torch, outs[q][i]), _expect(bufs[q][i], n, lut, False)[0])
    mg.close()


def test_second_ring_on_device_is_busy(torch_cuda):
    """One ring per GPU: a second nbg_ring_start on the device (another handle) returns NBG_EBUSY at
    once instead of stalling until the first ring's idle exit; after the first stops, it starts."""
    torch = torch_cuda
    import netbricks_amd as nb

    lut = orc.lut_build(NAMES65, 65537)
    a, b = nb.Maglev(NAMES65, 65537), nb.Maglev(NAMES65, 65537)
    n = 70000
    buf = nb.make_trace(n, 0, seed=77)[0]
    dd = torch.from_numpy(buf).cuda()
    out = torch.empty(n, dtype=torch.uint16, device="cuda")
    torch.cuda.synchronize()
    with a.ring() as ring:
        t0 = time.perf_counter()
        with pytest.raises(nb.NbgError) as e:
            b.ring()
        assert e.value.code == -16 and time.perf_counter() - t0 < 0.5
        with pytest.raises(nb.NbgError) as e:  # the ring's own handle refuses direct classify calls
            a.group_by(dd, n, swap_macs=False)
        assert e.value.code == -16
        # another handle's batch co-runs (tile-per-wave kernel while the ring holds the CUs' LDS)
        r = b.group_by(dd, n, swap_macs=False, stream=torch.cuda.current_stream().cuda_stream)
        ring.wait(ring.post(dd, n, out))
        torch.cuda.current_stream().synchronize()
        be = _expect(buf, n, lut, False)[0]
        np.testing.assert_array_equal(_got(torch, r.backend), be)
        np.testing.assert_array_equal(_got(torch, out), be)
    with b.ring() as ring2:  # the device is free again
        out.zero_()
        ring2.wait(ring2.post(dd, n, out))
    np.testing.assert_array_equal(_got(torch, out), _expect(buf, n, lut, False)[0])
    a.close()
    b.close()


def test_ring_starts_while_kernels_hold_cus(torch_cuda):
    """A ring started while another stream's kernel holds CUs: 16 workgroups that each hold 100 KB of
    a CU's LDS for 60 ms (nbg_debug_hold_cus), so 16 of the ring's blocks (the relay included, the
    grid's last block) cannot become resident until they leave.  The ring then runs every batch to
    completion, bit-exact, no earlier than the holders' exit."""
    import ctypes as C

    torch = torch_cuda
    import netbricks_amd as nb
    from netbricks_amd._lib import lib

    lut = orc.lut_build(NAMES65, 65537)
    mg = nb.Maglev(NAMES65, 65537)
    n = 262144
    bufs = [nb.make_trace(n, 0, seed=90 + i)[0] for i in range(6)]
    d = [torch.from_numpy(b.copy()).cuda() for b in bufs]
    outs = [torch.empty(n, dtype=torch.uint16, device="cuda") for _ in range(6)]
    busy = torch.cuda.Stream()
    torch.cuda.synchronize()
    hold = lib.nbg_debug_hold_cus
    hold.restype, hold.argtypes = C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p]
    t0 = time.perf_counter()
    assert hold(16, 100 * 1024, 60000, busy.cuda_stream) == 0
    time.sleep(0.005)  # the holders are resident before the ring launches
    with mg.ring(swap_macs=True) as ring:
        tickets = [ring.post(d[i], n, outs[i]) for i in range(6)]
        ring.wait(tickets[-1], timeout_ms=20000)
        t_done = time.perf_counter() - t0
    busy.synchronize()
    assert 0.04 < t_done < 10, t_done
    for i in range(6):
        be, ref = _expect(bufs[i], n, lut, True)
        np.testing.assert_array_equal(_got(torch, outs[i]), be)
        np.testing.assert_array_equal(d[i].cpu().numpy(), ref)
    mg.close()


def test_ring_group_burst(torch_cuda):
    """nbg_ring_group_burst: bursts of 1..8 consecutive batches grouped by one gate + hist + group
    launch each, enqueued right after the posts (C4 shard-size batches and mixed sizes, an empty batch
    in one burst: the per-batch fallback); every batch's perm / counts bit-exact."""
    torch = torch_cuda
    import netbricks_amd as nb

    lut = orc.lut_build(NAMES65, 65537)
    mg = nb.Maglev(NAMES65, 65537)
    sizes = [131072] * 8 + [1, 5000, 131072, 262144, 65536] + [0, 4096, 300000] + [131072] * 6
    bursts = [8, 5, 3, 6]
    bufs = [nb.make_trace(max(n, 1), 0, seed=1700 + i)[0] for i, n in enumerate(sizes)]
    d = [torch.from_numpy(b.copy()).cuda() for b in bufs]
    outs = [torch.empty(max(n, 1), dtype=torch.uint16, device="cuda") for n in sizes]
    perms = [torch.empty(max(n, 1), dtype=torch.uint32, device="cuda") for n in sizes]
    counts = [torch.full((66,), 7, dtype=torch.uint32, device="cuda") for _ in sizes]
    sides = [torch.cuda.Stream() for _ in range(2)]
    torch.cuda.synchronize()
    with mg.ring(swap_macs=True) as ring:
        i = 0
        for k, bsz in enumerate(bursts):
            first = None
            for j in range(bsz):
                t = ring.post(d[i + j], sizes[i + j], outs[i + j])
                first = t if first is None else first
            ring.group_burst(first, perms[i:i + bsz], counts[i:i + bsz], stream=sides[k % 2])
            i += bsz
        ring.wait(len(sizes) - 1)
        for st in sides:
            st.synchronize()
    for i, n in enumerate(sizes):
        be, _ = _expect(bufs[i], n, lut, True)
        exp_perm, exp_cnt = orc.group(be[:n], 65)
        if n:
            np.testing.assert_array_equal(_got(torch, outs[i])[:n], be[:n], err_msg=f"batch {i} ({n}) backend")
            np.testing.assert_array_equal(_np32(torch, perms[i])[:n], exp_perm, err_msg=f"batch {i} ({n}) perm")
        np.testing.assert_array_equal(_np32(torch, counts[i]), exp_cnt, err_msg=f"batch {i} ({n}) counts")
    mg.close()


def test_ring_repeated_inputs_in_place(torch_cuda):
    """Four 262,144-packet buffers posted round-robin 101 times in place, each reposted only once its
    previous batch is complete (the contract the bench's ring passes keep): every buffer ends swapped
    iff it was classified an odd number of times, and the last batches' backend[] are exact."""
    torch = torch_cuda
    import netbricks_amd as nb

    lut = orc.lut_build(NAMES65, 65537)
    mg = nb.Maglev(NAMES65, 65537)
    n, k, posts = 262144, 4, 101
    bufs = [nb.make_trace(n, 0, seed=1900 + i)[0] for i in range(k)]
    d = [torch.from_numpy(b.copy()).cuda() for b in bufs]
    outs = [torch.empty(n, dtype=torch.uint16, device="cuda") for _ in range(posts)]
    torch.cuda.synchronize()
    with mg.ring(swap_macs=True) as ring:
        for t in range(posts):
            if t >= k:
                ring.wait(t - k)  # the buffer's previous batch is complete
            assert ring.post(d[t % k], n, outs[t]) == t
        ring.wait(posts - 1)
    for i in range(k):
        times = len(range(i, posts, k))
        be, swapped = _expect(bufs[i], n, lut, True)
        np.testing.assert_array_equal(d[i].cpu().numpy(), swapped if times % 2 else bufs[i], err_msg=f"buffer {i}")
        np.testing.assert_array_equal(_got(torch, outs[posts - k + ((i - posts) % k)]), be)
    mg.close()


@pytest.mark.parametrize("swap", [False, True])
def test_ring_stop_while_producers_blocked(torch_cuda, swap):
    """nbg_ring_stop while other producer threads are blocked inside nbg_ring_queue_post (more batches
    outstanding than the ring's 64 slots) or nbg_ring_queue_wait: stop waits for them to leave, their
    calls return (a completion or the ring's end, never a crash or a hang), and every later call on a
    closed queue fails cleanly.  Every batch a producer saw complete is bit-exact; the handle starts a
    new ring afterwards."""
    import threading

    torch = torch_cuda
    import netbricks_amd as nb

    lut = orc.lut_build(NAMES65, 65537)
    mg = nb.Maglev(NAMES65, 65537)
    nq, per_q, n = 4, 20, 262144  # 80 buffers in flight at most: more than the 64 slots, so posts block
    bufs = [[nb.make_trace(n, 0, seed=5000 + 100 * q + i)[0] for i in range(per_q)] for q in range(nq)]
    d = [[torch.from_numpy(b.copy()).cuda() for b in bq] for bq in bufs]
    outs = [[torch.empty(n, dtype=torch.uint16, device="cuda") for _ in range(per_q)] for _ in range(nq)]
    torch.cuda.synchronize()
    done = [[] for _ in range(nq)]  # (ticket, buffer) a producer saw complete
    errs, started = [], threading.Barrier(nq + 1)
    ring = mg.ring(swap_macs=swap)
    qs = [ring.queue() for _ in range(nq)]

    def producer(q):
        started.wait()
        i = 0
        try:
            while True:
                if i >= per_q:  # the buffer's previous batch must be complete before it is reposted
                    qs[q].wait(i - per_q)
                    done[q].append(i - per_q)
                qs[q].post(d[q][i % per_q], n, outs[q][i % per_q])
                i += 1
        except (nb.NbgError, RuntimeError) as e:  # the ring stopped under the call
            errs.append(type(e).__name__)

    th = [threading.Thread(target=producer, args=(q,), daemon=True) for q in range(nq)]
    for t in th:
        t.start()
    started.wait()
    time.sleep(0.05)
    t0 = time.perf_counter()
    ring.stop()
    assert time.perf_counter() - t0 < 10
    for t in th:
        t.join(10)
    assert not any(t.is_alive() for t in th)
    assert len(errs) == nq, errs
    with pytest.raises(RuntimeError):
        qs[0].post(d[0][0], n, outs[0][0])
    with pytest.raises(nb.NbgError):
        qs[1].wait(0)
    if not swap:  # read only: every buffer is pristine, so each completed batch checks against it
        for q in range(nq):
            for i in done[q][-3:]:
                np.testing.assert_array_equal(_got(torch, outs[q][i % per_q]), _expect(bufs[q][i % per_q], n, lut,
                                                                                       False)[0])
    buf = nb.make_trace(n, 0, seed=99)[0]
    dd = torch.from_numpy(buf.copy()).cuda()
    out = torch.empty(n, dtype=torch.uint16, device="cuda")
    with mg.ring(swap_macs=False) as ring2:  # the handle runs a new ring
        ring2.wait(ring2.post(dd, n, out))
    np.testing.assert_array_equal(_got(torch, out), _expect(buf, n, lut, False)[0])
    mg.close()


@pytest.mark.parametrize("compact", [False, True])
def test_ring_group_many_backends(torch_cuda, compact):
    """Ring grouping above 128 bins (200 backends: partition rows from hist_kernel's packed 16-bit rows
    in the XCD-aware partition order, the 10-bit group kernel; compact=True forces the compact
    group_direct_kernel the library takes for many bins beside a ring), for single tickets
    (nbg_ring_group) and a burst (nbg_ring_group_burst), with partition counts that are multiples of 8
    (131,072 packets: 32 partitions) and not (300,000: 74; 5,000: 2; 1); bit-exact against the oracle's
    per-group FIFO order (operators/group_by.rs:46-51)."""
    torch = torch_cuda
    import netbricks_amd as nb
    from netbricks_amd._lib import lib

    names = [f"be{i}" for i in range(200)]
    lut = orc.lut_build(names, 65537)
    mg = nb.Maglev(names, 65537)
    sizes = [131072, 300000, 5000, 1, 131072, 300000, 5000, 262144]
    bufs = [nb.make_trace(n, 0, seed=2100 + i)[0] for i, n in enumerate(sizes)]
    d = [torch.from_numpy(b.copy()).cuda() for b in bufs]
    outs = [torch.empty(n, dtype=torch.uint16, device="cuda") for n in sizes]
    perms = [torch.empty(n, dtype=torch.uint32, device="cuda") for n in sizes]
    counts = [torch.full((201,), 7, dtype=torch.uint32, device="cuda") for _ in sizes]
    sides = [torch.cuda.Stream() for _ in range(2)]
    torch.cuda.synchronize()
    assert lib.nbg_debug_set_group_compact(1 if compact else -1) == 0
    try:
        with mg.ring(swap_macs=True) as ring:
            for i in range(4):  # single tickets, grouped right after their posts
                t = ring.post(d[i], sizes[i], outs[i])
                ring.group(t, perms[i], counts[i], stream=sides[i % 2])
            first = None
            for i in range(4, 8):  # one burst of four
                t = ring.post(d[i], sizes[i], outs[i])
                first = t if first is None else first
            ring.group_burst(first, perms[4:8], counts[4:8], stream=sides[0])
            ring.wait(len(sizes) - 1)
            for st in sides:
                st.synchronize()
    finally:
        assert lib.nbg_debug_set_group_compact(-1) == 0
    for i, n in enumerate(sizes):
        be, ref = _expect(bufs[i], n, lut, True)
        exp_perm, exp_cnt = orc.group(be, 200)
        np.testing.assert_array_equal(_got(torch, outs[i]), be, err_msg=f"batch {i} ({n}) backend")
        np.testing.assert_array_equal(_np32(torch, perms[i]), exp_perm, err_msg=f"batch {i} ({n}) perm")
        np.testing.assert_array_equal(_np32(torch, counts[i]), exp_cnt, err_msg=f"batch {i} ({n}) counts")
        np.testing.assert_array_equal(d[i].cpu().numpy(), ref, err_msg=f"batch {i} bytes")
    mg.close()


def test_ring_stop_twice_and_restart(torch_cuda):
    """nbg_ring_stop is idempotent: a second stop of the same ring returns the first stop's result and
    touches neither the handle nor its spare ring (no double free at destroy); the handle then starts
    a new ring (reusing the stopped one's buffers) that classifies bit-exact, and closes cleanly."""
    torch = torch_cuda
    import netbricks_amd as nb
    from netbricks_amd._lib import lib

    lut = orc.lut_build(NAMES65, 65537)
    mg = nb.Maglev(NAMES65, 65537)
    n = 70000
    buf = nb.make_trace(n, 0, seed=2300)[0]
    d = torch.from_numpy(buf.copy()).cuda()
    out = torch.empty(n, dtype=torch.uint16, device="cuda")
    torch.cuda.synchronize()
    ring = mg.ring()
    raw = ring._r
    ring.wait(ring.post(d, n, out))
    ring.stop()
    assert lib.nbg_ring_stop(raw) == 0
    assert lib.nbg_ring_stop(raw) == 0
    be, _ = _expect(buf, n, lut, False)
    np.testing.assert_array_equal(_got(torch, out), be)
    out2 = torch.empty(n, dtype=torch.uint16, device="cuda")
    with mg.ring(swap_macs=True) as ring2:
        ring2.wait(ring2.post(d, n, out2))
    be2, ref = _expect(buf, n, lut, True)
    np.testing.assert_array_equal(_got(torch, out2), be2)
    np.testing.assert_array_equal(d.cpu().numpy(), ref)
    mg.check()
    mg.close()
