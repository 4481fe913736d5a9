"""Multi-process (world_size 2, gloo on CPU) test of the bench's multi-GPU logic.

The Maglev path shards trivially (every packet is independent): each rank owns
distinct batches and there is no data-path collective.  What does cross ranks is the LUT,
built once on rank 0 and broadcast (RCCL on GPUs; gloo here).  Checks: every rank ends up with
the identical LUT, shards are distinct, and the per-group counts of the shards sum to those of
the concatenated input (shard-major concatenation == global order for contiguous shards).
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import sys

    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch

    import bench
    import netbricks_amd as nb
    import orc

    names = [f"backend-{i}" for i in range(bench.N_BACKENDS)]
    lut = bench.shared_lut(names, bench.TABLE, rank, world, torch.device("cpu"))
    n = 4096
    buf, _, _ = nb.make_trace(n, 0, seed=bench.shard_seed(rank, 0))
    be = orc.classify(buf.copy(), n, lut, stride=64, fixed_len=60)
    _, counts = orc.group(be, bench.N_BACKENDS)
    c = torch.from_numpy(counts.astype(np.int64))
    dist.all_reduce(c)
    digest = torch.tensor([int(np.uint64(lut.astype(np.uint64).sum()))], dtype=torch.int64)
    all_d = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(all_d, digest)
    # C4's scatter from rank 0: rank r receives exactly shard r of the global batch
    glob = torch.from_numpy(np.concatenate([nb.make_trace(n, 0, seed=bench.shard_seed(r, 0))[0]
                                            for r in range(world)])) if rank == 0 else None
    recv = torch.empty(n * 64, dtype=torch.uint8)
    bench.scatter_shard(glob, recv, rank, world)
    scatter_ok = np.array_equal(recv.numpy(), buf)
    # ... and its return leg: rank 0 gathers every shard's backend[] and group counts
    be_t = torch.from_numpy(be.astype(np.uint16).view(np.int16).copy())
    cnt_t = torch.from_numpy(counts.astype(np.uint32).view(np.int32).copy())
    gb = torch.empty(world * n * 2, dtype=torch.uint8) if rank == 0 else None
    gc = torch.empty(world * (bench.N_BACKENDS + 1), dtype=torch.int32) if rank == 0 else None
    bench.gather_results(be_t, cnt_t, gb, gc, rank, world)
    gather_ok = True
    if rank == 0:
        exp_be = np.concatenate([orc.classify(nb.make_trace(n, 0, seed=bench.shard_seed(r, 0))[0], n, lut,
                                              stride=64, fixed_len=60) for r in range(world)])
        got_be = gb.numpy().view(np.uint16)
        gather_ok = np.array_equal(got_be, exp_be) and int(gc.sum()) == world * n
    out[rank] = {"lut_ok": np.array_equal(lut, nb.build_lut(names, bench.TABLE)), "scatter_ok": scatter_ok,
                 "gather_ok": gather_ok,
                 "same_lut": len({int(d) for d in all_d}) == 1, "counts": c.numpy().tolist(),
                 "first": buf[:64].tobytes()}
    dist.destroy_process_group()


def test_two_rank_shards_gloo():
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import bench
    import netbricks_amd as nb
    import orc

    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    assert all(out[r]["lut_ok"] and out[r]["same_lut"] and out[r]["scatter_ok"] for r in range(world))
    assert out[0]["gather_ok"]
    assert out[0]["first"] != out[1]["first"]  # distinct shards
    # global reference: concatenate the shards and group once
    lut = nb.build_lut([f"backend-{i}" for i in range(bench.N_BACKENDS)], bench.TABLE)
    bufs = [nb.make_trace(4096, 0, seed=bench.shard_seed(r, 0))[0] for r in range(world)]
    allbuf = np.concatenate(bufs)
    be = orc.classify(allbuf, 4096 * world, lut, stride=64, fixed_len=60)
    _, counts = orc.group(be, bench.N_BACKENDS)
    assert out[0]["counts"] == counts.tolist() == out[1]["counts"]
