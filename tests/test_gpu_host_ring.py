"""The host-batch server (nbg_host_ring_*, include/nbgpu.h): one persistent kernel per GPU takes the
direct host batches (<= 2,048 packets) of every attached handle from a descriptor ring in pinned host
memory, so a batch costs no kernel launch.  Results must be exactly those of the small-kernel launch:
backend[], perm, counts and the MAC swap of every frame, bit-exact against the C oracle
(test/maglev/src/nf.rs:92-106, operators/group_by.rs:43-55), for concurrent producer threads, the
zero-copy path, the idle exit (later batches are launched) and the start / stop refusals.
"""
import threading
import time

import numpy as np
import pytest

import orc
from test_gpu_parity import _host_case, _mbuf_pool, _oracle, _pack

pytestmark = pytest.mark.gpu

NAMES65 = [f"backend-{i}" for i in range(65)]


def _check_batch(frames, pool, out, lut, nb_):
    pbuf, poff, pln = _pack([bytearray(f) for f in frames], 64)
    exp = _oracle(pbuf, len(frames), lut, nb_, offs=poff, lens=pln)
    np.testing.assert_array_equal(out["backend"], exp[1])
    np.testing.assert_array_equal(out["perm"], exp[2])
    np.testing.assert_array_equal(out["counts"], exp[3])
    for i, (o, l) in enumerate(zip(poff.tolist(), pln.tolist())):
        assert pool[i * 2048:i * 2048 + l].tobytes() == exp[0][o:o + l].tobytes(), i


@pytest.mark.parametrize("kind", [32, 48, 64, 80])
def test_host_ring_small_batches(torch_cuda, kind):
    """Every window stride (IHL options, runts, non-IPv4 frames), batches of 2048, 992 and 32 frames,
    three in flight, through the server: bit-exact."""
    import netbricks_amd as nb

    lut = orc.lut_build(NAMES65, 65537)
    mg = nb.Maglev(NAMES65, 65537)
    with nb.HostRing(blocks=8) as ring:
        mg.use_host_ring(ring)
        frames_all = _host_case(kind, 80 + kind)
        batches = []
        for lo, hi in ((0, 2048), (2048, 3040), (3040, 3072)):
            frames = frames_all[lo:hi]
            pool, ptrs, lens = _mbuf_pool(frames)
            out = dict(backend=np.empty(len(frames), np.uint16), perm=np.empty(len(frames), np.uint32),
                       counts=np.empty(66, np.uint32))
            batches.append((frames, pool, out, mg.host_submit(ptrs, lens, **out)))
        for *_, t in batches:
            mg.host_wait(t)
        mg.use_host_ring(None)
    for frames, pool, out, _ in batches:
        _check_batch(frames, pool, out, lut, 65)
    mg.close()


def test_host_ring_concurrent_producers(torch_cuda):
    """Six producer threads, each with its own handle (65 or 1000 backends), 40 batches of 1 to 2048
    frames each through one server (concurrent posts, slots reused many times over 256 slots):
    every batch bit-exact."""
    import netbricks_amd as nb
    from netbricks_amd import make_trace

    luts = {65: orc.lut_build(NAMES65, 65537), 1000: orc.lut_build([f"be{i}" for i in range(1000)], 655373)}
    errors = []

    def producer(k, ring):
        try:
            nb_ = 65 if k % 2 == 0 else 1000
            names = NAMES65 if nb_ == 65 else [f"be{i}" for i in range(1000)]
            mg = nb.Maglev(names, 65537 if nb_ == 65 else 655373)
            mg.use_host_ring(ring)
            rng = np.random.default_rng(k)
            pending = []
            for j in range(40):
                n = int(rng.choice([1, 32, 500, 992, 2048]))
                buf, off, ln = make_trace(n, 1, seed=10000 + 100 * k + j)
                frames = [bytearray(buf[o:o + l].tobytes()) for o, l in zip(off, ln)]
                pool, ptrs, lens = _mbuf_pool(frames)
                out = dict(backend=np.empty(n, np.uint16), perm=np.empty(n, np.uint32),
                           counts=np.empty(nb_ + 1, np.uint32))
                pending.append((frames, pool, out, mg.host_submit(ptrs, lens, **out)))
                if len(pending) == 3:  # three in flight (the handle's staging slots)
                    fr, pl, ou, t = pending.pop(0)
                    mg.host_wait(t)
                    _check_batch(fr, pl, ou, luts[nb_], nb_)
            for fr, pl, ou, t in pending:
                mg.host_wait(t)
                _check_batch(fr, pl, ou, luts[nb_], nb_)
            mg.close()  # detaches
        except Exception as e:  # noqa: BLE001 (reported below)
            errors.append(f"producer {k}: {e!r}")

    with nb.HostRing(blocks=16) as ring:
        th = [threading.Thread(target=producer, args=(k, ring)) for k in range(6)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=240)
    assert not errors, errors


def test_host_ring_zero_copy(torch_cuda):
    """A registered mbuf pool (zero-copy: the server's block reads the frames and writes the MAC swap
    over PCIe): 992-frame batches, bit-exact, swapped in the pool."""
    import netbricks_amd as nb
    from netbricks_amd import make_trace

    lut = orc.lut_build(NAMES65, 65537)
    n, room = 992, 2048
    buf, off, ln = make_trace(n, 1, seed=77)
    pool = np.zeros(n * room, dtype=np.uint8)
    for i, (o, l) in enumerate(zip(off.tolist(), ln.tolist())):
        pool[i * room:i * room + l] = buf[o:o + l]
    ref = pool.copy()
    offs = (np.arange(n, dtype=np.uint64) * room)
    be = orc.classify(ref, n, lut, offs=offs, lens=ln)
    perm, counts = orc.group(be, 65)
    mg = nb.Maglev(NAMES65, 65537)
    with nb.HostRing(blocks=4) as ring, nb.HostRegion(pool) as reg:
        mg.use_host_ring(ring)
        ptrs = (offs + np.uint64(pool.ctypes.data)).astype(np.uint64)
        out = dict(backend=np.empty(n, np.uint16), perm=np.empty(n, np.uint32), counts=np.empty(66, np.uint32))
        mg.host_wait(mg.host_submit(ptrs, ln, **out))
        mg.use_host_ring(None)
        np.testing.assert_array_equal(out["backend"], be)
        np.testing.assert_array_equal(out["perm"], perm)
        np.testing.assert_array_equal(out["counts"], counts)
        np.testing.assert_array_equal(pool, ref)
        assert reg.dev_ptr is not None
    mg.close()


def test_host_ring_refusals_and_idle_exit(torch_cuda):
    """One server per device, none beside a persistent RX ring (each start refuses the other), stop
    refused while a handle is attached; after its idle exit the handle's batches are launched as
    before (still exact), and the ended server stops cleanly."""
    import netbricks_amd as nb
    from netbricks_amd._lib import NBG_EBUSY, NbgError

    lut = orc.lut_build(NAMES65, 65537)
    mg = nb.Maglev(NAMES65, 65537)
    ring = nb.HostRing(blocks=2, idle_ms=300)
    with pytest.raises(NbgError) as e:
        nb.HostRing()
    assert e.value.code == NBG_EBUSY
    dev = nb.Maglev(NAMES65, 65537)
    with pytest.raises(NbgError) as e:
        dev.ring()
    assert e.value.code == NBG_EBUSY
    mg.use_host_ring(ring)
    with pytest.raises(NbgError) as e:
        ring.stop()
    assert e.value.code == NBG_EBUSY
    time.sleep(1.0)  # the server's idle exit
    frames = _host_case(48, 9)[:700]
    pool, ptrs, lens = _mbuf_pool(frames)
    out = dict(backend=np.empty(len(frames), np.uint16), perm=np.empty(len(frames), np.uint32),
               counts=np.empty(66, np.uint32))
    mg.host_wait(mg.host_submit(ptrs, lens, **out))
    _check_batch(frames, pool, out, lut, 65)
    mg.use_host_ring(None)
    ring.stop()
    with dev.ring() as r:  # the device is free for an RX ring again
        assert r is not None
    dev.close()
    mg.close()
