"""Config C4's per-GPU workload on the one GPU a test box has: one 1M-packet C2 batch split into 8
contiguous 131,072-packet shards (what ncclScatter hands rank r), each shard
classified through the HIP path by its own handle on its own stream, as the 8 ranks would.

Checked bit-exactly against the C oracle:
  * every shard's backend[], perm, counts and MAC-swapped bytes against the oracle on that slice;
  * composition: for every group g, the concatenation over shards (shard-major) of shard s's group-g
    packets rebased by s * 131072 equals the oracle's group g of the whole batch, and the shard counts
    sum to the whole batch's counts.  This is why C4 needs no data-path collective: contiguous shards
    keep the reference's per-group FIFO order (operators/group_by.rs:46-51) when concatenated.

Reference analogue: RSS split into per-queue pipelines (native/pmd.c:16-21,
framework/src/scheduler/context.rs:241-255).
"""
import numpy as np
import pytest

import orc

pytestmark = pytest.mark.gpu

NAMES65 = [f"backend-{i}" for i in range(65)]
BATCH = 1 << 20
SHARDS = 8
SHARD = BATCH // SHARDS


def _np(t, dt):
    import torch

    view = {np.uint16: torch.int16, np.uint32: torch.int32}[dt]
    return t.view(view).cpu().numpy().view(dt)


@pytest.mark.parametrize("swap", [True, False])
def test_c4_shards_compose_to_global_grouping(torch_cuda, swap):
    import netbricks_amd as nb

    torch = torch_cuda
    dev = torch.device("cuda:0")
    lut = nb.build_lut(NAMES65, 65537)  # rank 0 builds it and broadcasts it (bench.shared_lut)
    buf, _, _ = nb.make_trace(BATCH, 0, seed=0x4E42474D41474C56)
    d = torch.from_numpy(buf.copy()).to(dev)
    mgs = [nb.Maglev(lut=lut, n_backends=65) for _ in range(SHARDS)]
    sts = [torch.cuda.Stream(dev) for _ in range(SHARDS)]
    outs = []
    for s in range(SHARDS):
        shard = d[s * SHARD * 64:(s + 1) * SHARD * 64]  # contiguous slice: the bytes rank s receives
        outs.append(mgs[s].group_by(shard, SHARD, swap_macs=swap, stream=sts[s].cuda_stream))
    torch.cuda.synchronize()
    for m in mgs:
        m.check()

    ref = buf.copy()
    be_all = orc.classify(ref, BATCH, orc.lut_build(NAMES65, 65537), swap=swap)
    perm_all, counts_all = orc.group(be_all, 65)
    starts_all = np.concatenate([[0], np.cumsum(counts_all.astype(np.int64))[:-1]])
    composed = [[] for _ in range(66)]
    counts_sum = np.zeros(66, dtype=np.int64)
    for s, r in enumerate(outs):
        lo = s * SHARD
        be_s = _np(r.backend, np.uint16)[:SHARD]
        perm_s = _np(r.perm, np.uint32)[:SHARD]
        cnt_s = _np(r.counts, np.uint32)
        exp_perm_s, exp_cnt_s = orc.group(be_all[lo:lo + SHARD], 65)
        np.testing.assert_array_equal(be_s, be_all[lo:lo + SHARD], err_msg=f"shard {s} backend")
        np.testing.assert_array_equal(perm_s, exp_perm_s, err_msg=f"shard {s} perm")
        np.testing.assert_array_equal(cnt_s, exp_cnt_s, err_msg=f"shard {s} counts")
        counts_sum += cnt_s
        st = np.concatenate([[0], np.cumsum(cnt_s.astype(np.int64))[:-1]])
        for g in range(66):
            composed[g].append(perm_s[st[g]:st[g] + cnt_s[g]].astype(np.int64) + lo)
    np.testing.assert_array_equal(counts_sum, counts_all)
    for g in range(66):
        got = np.concatenate(composed[g])
        np.testing.assert_array_equal(got, perm_all[starts_all[g]:starts_all[g] + counts_all[g]],
                                      err_msg=f"group {g}: shard-major concatenation != global FIFO order")
    np.testing.assert_array_equal(d.cpu().numpy(), ref, err_msg="MAC swap bytes")
    for m in mgs:
        m.close()
