"""GPU parity of NBG_GROUP_LAG (pipelined grouping): each call classifies its batch and the handle's
next call groups it inside its own streaming-classify launch (or nbg_maglev_finish_group does).  Every
batch's backend[], MAC-swapped bytes, perm and counts are checked bit-exactly against the C oracle run
on that batch alone, once the call that completes it has run.

Covers: back-to-back 1M batches on one handle; batches of unequal size (the pending batch larger than
the current one, so pieces run after the unit loop, and smaller); read-only, 12-B records and counts
only; calls that cannot carry the pending group (a 131,072-packet batch, a descriptor batch, a
multi-batch call) and so launch it alone first; finish_group on another stream; three handles on three
streams interleaved as bench.py issues them.

Reference semantics: the producer classifies and enqueues per batch (framework/src/operators/
group_by.rs:43-55); per-group FIFO order of the MPSC queues (queues/mpsc_mbuf_queue.rs:91-115).
"""
import numpy as np
import pytest

import orc

pytestmark = pytest.mark.gpu

NAMES65 = [f"backend-{i}" for i in range(65)]


@pytest.fixture(scope="module")
def lut65():
    return orc.lut_build(NAMES65, 65537)


def _np(t, dt):
    import torch

    view = {np.uint16: torch.int16, np.uint32: torch.int32, np.uint8: torch.uint8}[dt]
    return t.view(view).cpu().numpy().view(dt)


class _Batch:
    def __init__(self, torch, n, seed, *, records=False, counts_only=False, nb=65):
        import netbricks_amd as nb_

        dev = torch.device("cuda:0")
        self.n = n
        self.host = nb_.make_trace(n, 0, seed=seed)[0]
        self.d = torch.from_numpy(self.host.copy()).to(dev)
        self.backend = torch.empty(n, dtype=torch.uint16, device=dev)
        self.perm = None if counts_only else torch.empty(n, dtype=torch.uint32, device=dev)
        self.counts = torch.empty(nb + 1, dtype=torch.uint32, device=dev)
        self.mac = torch.empty(12 * n, dtype=torch.uint8, device=dev) if records else None

    def run(self, mg, stream=None, swap=True, lag=True):
        mg.group_by(self.d, self.n, swap_macs=swap, group_lag=lag, backend=self.backend, perm=self.perm,
                    scatter=self.perm is not None, counts=self.counts, mac_out=self.mac, stream=stream)

    def check(self, lut, swap=True, nb=65):
        ref = self.host.copy()
        be = orc.classify(ref, self.n, lut, swap=swap)
        perm, counts = orc.group(be, nb)
        np.testing.assert_array_equal(_np(self.backend, np.uint16), be)
        np.testing.assert_array_equal(_np(self.counts, np.uint32), counts)
        if self.perm is not None:
            np.testing.assert_array_equal(_np(self.perm, np.uint32), perm)
        got = self.d.cpu().numpy()
        if self.mac is not None:
            np.testing.assert_array_equal(got, self.host)
            np.testing.assert_array_equal(self.mac.cpu().numpy().reshape(self.n, 12), ref.reshape(self.n, 64)[:, :12])
        else:
            np.testing.assert_array_equal(got, ref)


def _mg(lut=None):
    from netbricks_amd import Maglev

    return Maglev(NAMES65, 65537)


def test_lag_back_to_back_1m(torch_cuda, lut65):
    mg = _mg()
    bs = [_Batch(torch_cuda, 1 << 20, 500 + i) for i in range(5)]
    for b in bs:
        b.run(mg)
    mg.finish_group()
    torch_cuda.cuda.synchronize()
    mg.check()
    for b in bs:
        b.check(lut65)
    mg.close()


@pytest.mark.parametrize("sizes", [[1 << 20, 262_144, 2_100_000, 300_001, 4_194_304, 1 << 20],
                                   [262_144, 4_194_304, 262_145, 999_999]])
def test_lag_unequal_sizes(torch_cuda, lut65, sizes):
    """A pending batch larger than the launch carrying it: pieces beyond the unit steps run after them."""
    mg = _mg()
    bs = [_Batch(torch_cuda, n, 600 + i) for i, n in enumerate(sizes)]
    for b in bs:
        b.run(mg)
    mg.finish_group()
    torch_cuda.cuda.synchronize()
    mg.check()
    for b in bs:
        b.check(lut65)
    mg.close()


def test_lag_read_only_records_counts_only(torch_cuda, lut65):
    mg = _mg()
    ro = _Batch(torch_cuda, 1 << 20, 700)
    rec = _Batch(torch_cuda, 700_000, 701, records=True)
    co = _Batch(torch_cuda, 1 << 20, 702, counts_only=True)
    last = _Batch(torch_cuda, 300_000, 703)
    ro.run(mg, swap=False)
    rec.run(mg)
    co.run(mg)
    last.run(mg)
    mg.finish_group()
    torch_cuda.cuda.synchronize()
    mg.check()
    ro.check(lut65, swap=False)
    rec.check(lut65)
    co.check(lut65)
    last.check(lut65)
    mg.close()


def test_lag_flushed_by_calls_that_cannot_carry_it(torch_cuda, lut65):
    """A small batch, a descriptor batch and a multi-batch call launch the pending group alone first."""
    import netbricks_amd as nb

    torch = torch_cuda
    dev = torch.device("cuda:0")
    mg = _mg()
    a = _Batch(torch, 1 << 20, 800)
    small = _Batch(torch, 131_072, 801)
    b = _Batch(torch, 500_000, 802)
    a.run(mg)
    small.run(mg)  # below the streaming threshold: grouped at once, after a's group
    b.run(mg)
    buf, off, ln = nb.make_trace(50_000, 1, seed=803)
    d = torch.from_numpy(buf.copy()).to(dev)
    do = torch.from_numpy(off.view(np.int32)).to(dev).view(torch.uint32)
    dl = torch.from_numpy(ln.view(np.int16)).to(dev).view(torch.uint16)
    r = mg.group_by(d, 50_000, offsets=do, lens=dl, owned_windows=True, group_lag=True)  # descriptors
    c = _Batch(torch, 1 << 20, 804)
    c.run(mg)
    multi = [_Batch(torch, 400_000, 805 + j) for j in range(2)]
    out = mg.group_by_multi([(m.d, m.n) for m in multi])
    torch.cuda.synchronize()
    mg.check()
    a.check(lut65)
    small.check(lut65)
    b.check(lut65)
    ref = buf.copy()
    be = orc.classify(ref, 50_000, lut65, offs=off, lens=ln)
    perm, counts = orc.group(be, 65)
    np.testing.assert_array_equal(_np(r.backend, np.uint16), be)
    np.testing.assert_array_equal(_np(r.perm, np.uint32)[:50_000], perm)
    np.testing.assert_array_equal(_np(r.counts, np.uint32), counts)
    c.check(lut65)
    for m, g in zip(multi, out):
        m.backend, m.perm, m.counts = g.backend, g.perm, g.counts
        m.check(lut65)
    mg.close()


def test_lag_finish_on_other_stream_and_three_handles(torch_cuda, lut65):
    """bench.py's issue pattern: three handles, three streams, batches round-robin, then every
    handle's pending group finished on the default stream."""
    torch = torch_cuda
    dev = torch.device("cuda:0")
    mgs = [_mg() for _ in range(3)]
    sts = [torch.cuda.Stream(dev) for _ in range(3)]
    bs = [_Batch(torch, 1 << 20, 900 + i) for i in range(9)]
    for i, b in enumerate(bs):
        b.run(mgs[i % 3], stream=sts[i % 3].cuda_stream)
    for m in mgs:
        m.finish_group()  # torch's current stream: ordered after the handle's last stream
    torch.cuda.synchronize()
    for m in mgs:
        m.check()
    for b in bs:
        b.check(lut65)
    for m in mgs:
        m.close()


def test_lag_many_backends_nine_bits(torch_cuda):
    """200 backends (9-bit multisplit) at 262,144 packets per batch (direct-scan limit)."""
    from netbricks_amd import Maglev

    names = [f"b{i}" for i in range(200)]
    lut = orc.lut_build(names, 65537)
    mg = Maglev(names, 65537)
    bs = [_Batch(torch_cuda, 262_144 + 64 * i, 950 + i, nb=200) for i in range(4)]
    for b in bs:
        b.run(mg)
    mg.finish_group()
    torch_cuda.cuda.synchronize()
    mg.check()
    for b in bs:
        b.check(lut, nb=200)
    mg.close()


def test_lag_refused_with_defer(torch_cuda):
    from netbricks_amd._lib import NbgError

    mg = _mg()
    b = _Batch(torch_cuda, 1 << 20, 990)
    with pytest.raises(NbgError):
        mg.group_by(b.d, b.n, group_lag=True, defer_group=True)
    mg.close()
