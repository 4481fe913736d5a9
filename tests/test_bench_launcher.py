"""The bench launcher (`bench.py --gpus N`) end to end on the CPU: the parent spawns N rank
processes (it never touches the GPU), each joins a gloo process group (`--selftest`: the same
rank logic with no HIP call), and rank 0's JSON line reports N ranks, one rate per rank and the
identical LUT digest on every rank (the LUT is built on rank 0 and broadcast).  Reference: one
pipeline per RX queue, framework/src/scheduler/context.rs:241-255."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n, tmp):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--selftest",
                        "--steps", "3", "--warmup", "1"], capture_output=True, text=True, timeout=300,
                       env={**{k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")},
                            "NBG_BENCH_FULL": os.path.join(str(tmp), "full.json")})
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    assert len(lines[0]) <= 8000, len(lines[0])  # the driver reads a ~8.3 KB stdout tail
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [1, 2, 4])
def test_launcher_spawns_ranks(n, tmp_path):
    line = _run(n, tmp_path)
    full = json.load(open(tmp_path / "full.json"))  # the full record beside the compact line
    assert full["n_gpus"] == n and len(full["lut_digest_per_rank"]) == n
    assert line["n_gpus"] == n
    assert line["selftest"] is True
    assert len(line["per_gpu_mpps"]) == n
    assert line["lut_digests_agree"] is True
    assert line["config"]["parallelism"] == f"shard{n}"
    assert line["scaling"] == "weak"
    # config C4: one 1M batch in n contiguous shards, one per rank; with N > 1
    # the scatter / classify / gather pass ran (gloo here) and rank 0's gathered counts summed to 1M
    c4 = line["c4"]
    assert c4["shards"] == n and c4["shard_pkts"] * n == c4["batch_pkts"] == 1 << 20
    assert len(c4["device_resident"]["per_gpu_mpps"]) == n
    if n > 1:
        assert c4["scatter_inclusive"]["checked"] is True and c4["scatter_inclusive"]["steps"] > 0
        # the communicator's own rank count (an all-reduce over it; gloo here, RCCL on GPUs)
        assert line["rccl_ranks"] == n and line["comm_backend"] == "gloo"
    else:
        assert "scatter_inclusive" not in c4
        assert "rccl_ranks" not in line


def test_rank_rejects_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--selftest"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in r.stderr
