"""GPU parity of nbg_maglev_classify_device_multi: several fixed-slot batches in one launch of the
streaming classify kernel and one of the group kernel, each batch bit-exact against the C oracle
run on that batch alone (backend[], the MAC swap in place or as 12-B records, perm, counts).

Reference semantics: test/maglev/src/nf.rs:92-108, one pipeline per RX queue
(framework/src/scheduler/context.rs:241-255); grouping never crosses batches.
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


@pytest.fixture(scope="module")
def lut65():
    return orc.lut_build(NAMES65, 65537)


def _np(t, dt):
    import torch

    view = {np.uint16: torch.int16, np.uint32: torch.int32, np.uint8: torch.uint8}[dt]
    return t.view(view).cpu().numpy().view(dt)


def _batches(torch, sizes, seed):
    from netbricks_amd import make_trace

    dev = torch.device("cuda:0")
    host = [make_trace(n, 0, seed=seed + j)[0] for j, n in enumerate(sizes)]
    return host, [(torch.from_numpy(h.copy()).to(dev), n) for h, n in zip(host, sizes)]


def _check(torch, mg, lut, sizes, seed, *, swap=True, records=False, scatter=True):
    host, dev = _batches(torch, sizes, seed)
    out = mg.group_by_multi(dev, swap_macs=swap, records=records, scatter=scatter)
    torch.cuda.synchronize()
    mg.check()
    for j, (h, n) in enumerate(zip(host, sizes)):
        ref = h.copy()
        be = orc.classify(ref, n, lut, swap=swap)
        perm, counts = orc.group(be, 65)
        g, mac = out[j] if records else (out[j], None)
        np.testing.assert_array_equal(_np(g.backend, np.uint16)[:n], be, err_msg=f"batch {j}")
        np.testing.assert_array_equal(_np(g.counts, np.uint32), counts, err_msg=f"batch {j}")
        if scatter:
            np.testing.assert_array_equal(_np(g.perm, np.uint32)[:n], perm, err_msg=f"batch {j}")
        else:
            assert g.perm is None
        got_pkts = dev[j][0].cpu().numpy()
        if records:
            np.testing.assert_array_equal(got_pkts, h)  # packets untouched
            m = mac.cpu().numpy()[:12 * n].reshape(n, 12)
            np.testing.assert_array_equal(m, ref.reshape(n, 64)[:, :12], err_msg=f"batch {j} records")
        else:
            np.testing.assert_array_equal(got_pkts, ref, err_msg=f"batch {j} bytes")


@pytest.mark.parametrize("sizes", [[1 << 20] * 4, [300_000, 1 << 20, 262_145], [1 << 20, 64, 4097, 700_001],
                                   [2_100_000, 1 << 20]])
def test_multi_in_place(torch_cuda, mg65, lut65, sizes):
    _check(torch_cuda, mg65, lut65, sizes, seed=100 + len(sizes))


@pytest.mark.parametrize("swap,records", [(False, False), (True, True)])
def test_multi_read_only_and_records(torch_cuda, mg65, lut65, swap, records):
    _check(torch_cuda, mg65, lut65, [1 << 20, 500_000, 1 << 20], seed=7, swap=swap, records=records)


def test_multi_counts_only(torch_cuda, mg65, lut65):
    _check(torch_cuda, mg65, lut65, [600_000, 1 << 20], seed=9, scatter=False)


def test_multi_fallback_small_batches(torch_cuda, mg65, lut65):
    """Below 262,144 packets in all the batches run one after another through the single path."""
    _check(torch_cuda, mg65, lut65, [1000, 5000, 64, 33], seed=11)


def test_multi_alternating_batch_counts(torch_cuda, mg65, lut65):
    """Ping-pong partition histograms across calls with 4, 2, 8, 1, 3 and 16 batches, single calls between."""
    from netbricks_amd import make_trace

    for i, sizes in enumerate([[1 << 20] * 4, [400_000, 300_000], [131_072] * 8, [1 << 20], [262_144, 1, 262_144],
                               [65_536 + 64 * k for k in range(16)]]):
        _check(torch_cuda, mg65, lut65, sizes, seed=200 + 10 * i)
        buf, _, _ = make_trace(300_000, 0, seed=300 + i)
        d = torch_cuda.from_numpy(buf.copy()).to(torch_cuda.device("cuda:0"))
        r = mg65.group_by(d, 300_000)
        torch_cuda.cuda.synchronize()
        ref = buf.copy()
        be = orc.classify(ref, 300_000, lut65)
        perm, counts = orc.group(be, 65)
        np.testing.assert_array_equal(_np(r.perm, np.uint32)[:300_000], perm)
        np.testing.assert_array_equal(_np(r.counts, np.uint32), counts)


def test_multi_rejects_bad_counts(torch_cuda, mg65):
    with pytest.raises(ValueError):
        mg65.group_by_multi([])
    d = torch_cuda.zeros(64 * 10, dtype=torch_cuda.uint8, device="cuda:0")
    from netbricks_amd._lib import NBG_MAX_MULTI

    with pytest.raises(ValueError):
        mg65.group_by_multi([(d, 10)] * (NBG_MAX_MULTI + 1))


def test_multi_deferred_group_on_second_stream(torch_cuda, mg65, lut65):
    """NBG_DEFER_GROUP on the fused multi-batch path: the classify launch on one stream,
    the one group launch of all batches by finish_group on a second stream (ordered after it by the
    handle's event), then a single group_by on the first stream: every batch bit-exact."""
    torch = torch_cuda
    sizes = [1 << 20, 300_000, 700_001]
    host, dev = _batches(torch, sizes, seed=400)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    out = mg65.group_by_multi(dev, defer_group=True, stream=s1.cuda_stream)
    mg65.finish_group(s2.cuda_stream)
    buf, _, _ = __import__("netbricks_amd").make_trace(400_000, 0, seed=410)
    d = torch.from_numpy(buf.copy()).to(torch.device("cuda:0"))
    r = mg65.group_by(d, 400_000, stream=s1.cuda_stream)
    torch.cuda.synchronize()
    mg65.check()
    for j, (h, n) in enumerate(zip(host, sizes)):
        ref = h.copy()
        be = orc.classify(ref, n, lut65)
        perm, counts = orc.group(be, 65)
        np.testing.assert_array_equal(_np(out[j].backend, np.uint16)[:n], be, err_msg=f"batch {j}")
        np.testing.assert_array_equal(_np(out[j].perm, np.uint32)[:n], perm, err_msg=f"batch {j}")
        np.testing.assert_array_equal(_np(out[j].counts, np.uint32), counts, err_msg=f"batch {j}")
    ref = buf.copy()
    be = orc.classify(ref, 400_000, lut65)
    perm, counts = orc.group(be, 65)
    np.testing.assert_array_equal(_np(r.perm, np.uint32)[:400_000], perm)
    np.testing.assert_array_equal(_np(r.counts, np.uint32), counts)
