"""CPU tests of the tools that recompute the profiled figures from profiles/: tools/kshapes.py (kernel
durations by launch shape, and the dispatches that ran alone) and tools/ring_slope.py (per-batch
ring time from completion stamps)."""
import csv
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import ring_slope  # noqa: E402


def _trace(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Grid_Size_X", "Workgroup_Size_X", "Group_Segment_Size",
                                          "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        for name, grid, wg, lds, t0, t1 in rows:
            w.writerow({"Kernel_Name": name, "Grid_Size_X": grid, "Workgroup_Size_X": wg, "Group_Segment_Size": lds,
                        "Start_Timestamp": t0, "End_Timestamp": t1})


def test_kshapes_groups_by_shape_and_finds_alone_dispatches(tmp_path):
    """Two launch shapes of one kernel land in two rows; a dispatch that overlaps another is not
    'alone' (ns timestamps -> us)."""
    k = "void nbg::(anonymous namespace)::classify_stream_kernel<true, true, 1, 0>(nbg::ClassifyArgs)"
    g = "void nbg::(anonymous namespace)::group_kernel<2, 7>(nbg::GroupMulti)"
    rows = [
        (k, 256 * 512, 512, 0, 0, 90_000),             # 4 x 1M shape, alone
        (k, 256 * 512, 512, 0, 100_000, 200_000),      # overlaps the group below
        (g, 1024 * 512, 512, 512, 150_000, 180_000),
        (k, 128 * 512, 512, 0, 300_000, 310_000),      # another shape, alone
    ]
    trace = tmp_path / "run_kernel_trace.csv"
    _trace(trace, rows)
    out = tmp_path / "shapes.csv"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "kshapes.py"), str(trace), str(out)], check=True,
                   capture_output=True)
    got = {(r["kernel"], int(r["workgroups"])): r for r in csv.DictReader(open(out))}
    big = got[("classify_stream_kernel<true, true, 1, 0>", 256)]
    assert int(big["calls"]) == 2 and float(big["mean_us"]) == 95.0
    assert int(big["alone_calls"]) == 1 and float(big["alone_mean_us"]) == 90.0
    small = got[("classify_stream_kernel<true, true, 1, 0>", 128)]
    assert int(small["alone_calls"]) == 1 and float(small["alone_mean_us"]) == 10.0
    assert int(got[("group_kernel<2, 7>", 1024)]["alone_calls"]) == 0


def test_ring_slope_recovers_the_per_batch_time(tmp_path):
    """A completion stamp series with a slow ramp and a slow drain: the slope over the middle three
    quarters is the steady per-batch time."""
    n = 800
    t = np.concatenate([np.arange(100) * 40.0, 4000.0 + np.arange(600) * 21.5, 4000.0 + 600 * 21.5 + np.arange(100) * 50.0])
    p = tmp_path / "ring_in_place.csv"
    with open(p, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["us_since_first", "completed"])
        for i in range(n):
            w.writerow([f"{t[i]:.3f}", i + 1])
    samples, us = ring_slope.slope(str(p))
    assert samples == n and abs(us - 21.5) < 0.5
