"""CPU tests of bench.py's helpers that the GPU runs depend on: the rocprofv3 --pmc CSV reader that
turns counter rows into per-launch bytes (only the classify kernels, in dispatch order, KB -> B),
and the CPU inventory used to size the CPU baseline."""
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_pmc_rows_filters_and_orders(tmp_path):
    d = tmp_path / "pass" / "host" / "1234"
    d.mkdir(parents=True)
    rows = [
        (7, "void nbg::(anonymous namespace)::classify_stream_kernel<true, true, 1>(nbg::ClassifyArgs)", "FETCH_SIZE", 3.0),
        (3, "void nbg::(anonymous namespace)::classify_stream_kernel<true, true, 1>(nbg::ClassifyArgs)", "FETCH_SIZE", 1.5),
        (5, "void nbg::(anonymous namespace)::group_kernel<2, 7>(nbg::GroupArgs)", "FETCH_SIZE", 99.0),
        (6, "void nbg::(anonymous namespace)::classify_kernel<2, true, true, false, 2, 0, 256>(nbg::ClassifyArgs)",
         "FETCH_SIZE", 2.0),
        (8, "void nbg::(anonymous namespace)::classify_stream_kernel<true, true, 1>(nbg::ClassifyArgs)", "WRITE_SIZE", 9.0),
    ]
    with open(d / "run_counter_collection.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        for r in rows:
            w.writerow(r)
    got, names = bench._pmc_rows(str(tmp_path / "pass"), "FETCH_SIZE")
    assert got == [1.5 * 1024, 2.0 * 1024, 3.0 * 1024]
    assert "classify_kernel<2" in names[1] and all("classify" in n for n in names)
    assert bench._pmc_rows(str(tmp_path / "pass"), "WRITE_SIZE")[0] == [9.0 * 1024]


def test_pmc_rows_desc_multi_kept_apart(tmp_path):
    """The descriptor multi-batch kernel (C3 / C5, several IMIX batches per launch) is its own row set:
    never mixed into the single-launch classify order, and read by desc=True alone."""
    d = tmp_path / "pass" / "host" / "1"
    d.mkdir(parents=True)
    rows = [
        (1, "void nbg::(anonymous namespace)::classify_kernel<3, false, false, false, 2, 0, 256>(nbg::ClassifyArgs)",
         "FETCH_SIZE", 1.0),
        (2, "void nbg::(anonymous namespace)::classify_desc_multi_kernel<3, false, false, false>(nbg::ClassifyArgs, "
            "nbg::DescBatches)", "FETCH_SIZE", 8.0),
        (3, "void nbg::(anonymous namespace)::classify_ring_kernel<true, 1>(nbg::ClassifyArgs, nbg::RingArgs)",
         "FETCH_SIZE", 5.0),
        (4, "void nbg::(anonymous namespace)::classify_desc_multi_kernel<2, true, true, true>(nbg::ClassifyArgs, "
            "nbg::DescBatches)", "FETCH_SIZE", 7.0),
    ]
    with open(d / "run_counter_collection.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        for r in rows:
            w.writerow(r)
    top = str(tmp_path / "pass")
    assert bench._pmc_rows(top, "FETCH_SIZE")[0] == [1.0 * 1024]
    assert bench._pmc_rows(top, "FETCH_SIZE", ring=True)[0] == [5.0 * 1024]
    assert bench._pmc_rows(top, "FETCH_SIZE", desc=True)[0] == [8.0 * 1024, 7.0 * 1024]


def test_pmc_algorithmic_bytes():
    """Per-launch algorithmic bytes of every PMC entry: a lagged launch carries the
    whole path (82 B: classify + the previous batch's perm), the others their classify bytes."""
    assert bench._pmc_algorithmic("in_place_lag") == bench.BATCH * 82
    assert bench._pmc_algorithmic("in_place") == bench.BATCH * 78
    assert bench._pmc_algorithmic("read_only") == bench.BATCH * 66
    assert bench._pmc_algorithmic("c4_shard") == 131072 * 78
    assert bench._pmc_algorithmic("c3") == bench.BATCH * 84
    assert bench._pmc_algorithmic("c5") == bench.BATCH * 78
    assert bench._pmc_algorithmic(f"read_only_multi{bench.MULTI_K}") == bench.MULTI_K * bench.BATCH * 66


def test_aggregate_frac():
    # 8 GPUs at 40 Gpps each of 82 B/pkt: 3.28 TB/s per GPU of 8 TB/s
    assert bench.aggregate_frac(8 * 40e9, 1.0, 82, 8) == round(40e9 * 82 / 1e9 / 8000.0, 4)


def test_cpu_inventory_is_sane():
    affinity, quota, model = bench.cpu_inventory()
    assert affinity >= 1
    assert quota is None or quota > 0
    assert isinstance(model, str) and model


def _full_record_n8():
    """A full-size N = 8 record: round 4's final N = 1 record (21 variants, 16 PMC blocks, the working-set
    sweep) with an 8-rank c4 block, 8 per-GPU rates and an e2e block."""
    import json

    full = json.load(open(os.path.join(ROOT, "profiles", "r04_bench_final.json")))
    for k in ("c3_multi16", "c5_multi16"):  # round 5 reports both at 16 per launch
        full["variants"].setdefault(k, dict(full["variants"]["c3_multi8"]))
    full["n_gpus"] = 8
    full["per_gpu_mpps"] = [44000.1] * 8
    full["lut_digest_per_rank"] = ["0123456789abc"] * 8
    full["rccl_ranks"], full["comm_backend"] = 8, "nccl"
    full["c4"]["device_resident"]["per_gpu_mpps"] = [5000.5] * 8
    full["c4"]["scatter_inclusive"] = {"value": 9000.1, "unit": "Mpps", "steps": 50, "ms_per_batch": 0.1165,
                                       "root_egress_GBps": 500.0, "checked": True, "what": "x" * 300}
    full["e2e"] = {"pipelined": {"mpps": 700.0}, "compact": {k: 123.4 for k in (
        "pipelined_mpps", "pipelined_h2d_gbps", "host_submit_mpps", "classify_host_mpps", "zero_copy_mpps",
        "host_submit_registered_mpps", "copies_only_mpps", "h2d_only_gbps", "d2h_only_gbps",
        "pcie_bound_gbps_per_dir", "batch_pkts", "host_batch_pkts")}}
    return full


def test_compact_line_fits_driver_tail():
    """The stdout line stays whole in the driver's ~8.3 KB tail (BENCH_r04 was 22.9 KB and unparsed):
    a full-size record compacts to <= LINE_LIMIT bytes and keeps every field the driver and judge read."""
    import json

    full = _full_record_n8()
    assert len(json.dumps(full)) > 20000
    line = bench.compact_line(full)
    s = json.dumps(line, separators=(",", ":"))
    assert len(s) <= bench.LINE_LIMIT < 8000, len(s)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "config", "dtype",
              "roofline", "cpu_baseline", "north_star", "c4", "e2e", "variants", "rccl_ranks"):
        assert k in line, k
    assert line["roofline"]["traffic"] == full["roofline"]["traffic"]
    assert line["c4"]["scatter_inclusive"]["checked"] is True and "what" not in line["c4"]["scatter_inclusive"]
    assert line["variants_fields"] == list(bench.VARIANT_FIELDS)
    row = line["variants"]["c5_multi8"]
    v = full["variants"]["c5_multi8"]
    assert row[0] == round(v["ms_per_batch"] * 1e3, 3) and row[1] == v["frac"]
    assert row[2] == full["pmc"]["c5_multi8"]["ratio"] and row[3] == v["classify_us_per_batch"]
    assert line["variants"]["ring_in_place"][2] == full["variants"]["ring_in_place"]["traffic_ratio"]
    assert "ws32_ring_in_place" in line["variants"]


def test_emit_line_fails_loudly_over_limit(tmp_path, monkeypatch, capsys):
    import json

    import pytest

    monkeypatch.setattr(bench, "FULL_RECORD", str(tmp_path / "full.json"))
    full = _full_record_n8()
    bench.emit_line(full)
    out = capsys.readouterr().out.strip()
    assert json.loads(out)["value"] == full["value"]
    assert json.load(open(tmp_path / "full.json"))["pmc"] == full["pmc"]
    full["variants"].update({f"extra_{i}": {"us_per_batch": 1.0, "frac": 0.5} for i in range(400)})
    with pytest.raises(SystemExit):
        bench.emit_line(full)


def test_completion_slope_uses_the_middle_of_the_run():
    """The ring's per-batch time (ring_pass, ring_path): the slope of (time, completed) stamps over the
    middle three quarters of the run, so a slow start (ring launch, LUT staging) and the drain at the
    stop do not enter it; None when the stamps do not span that window."""
    batches = 800
    stamps = [(0.0, 0)]
    t = 1e-3  # a 1 ms start-up before the first completion
    for c in range(1, batches + 1):
        t += 20e-6 if 100 <= c <= 700 else 50e-6  # steady 20 us per batch in the middle
        stamps.append((t, c))
    s = bench.completion_slope(stamps, batches)
    assert abs(s - 20e-6) < 1e-9
    # completions seen in bursts (the producer polls between posts): the slope is unchanged
    burst = [x for x in stamps if x[1] % 4 == 0 or x[1] in (0, batches)]
    assert abs(bench.completion_slope(burst, batches) - 20e-6) < 1e-9
    assert bench.completion_slope(stamps[:50], batches) is None
    assert bench.completion_slope([(0.0, 0)], batches) is None


def test_spread_cpus_deals_over_l3_caches(monkeypatch):
    """spread_cpus (the drop-in threads' placement, also tried for the CPU baseline): CPUs dealt
    round-robin over their L3 caches, the order within a cache kept, nothing lost or repeated."""
    l3 = {c: f"{c // 8 * 8}-{c // 8 * 8 + 7}" for c in range(32)}
    real_open = open

    def fake_open(path, *a, **k):
        if path.startswith("/sys/devices/system/cpu/cpu") and path.endswith("shared_cpu_list"):
            import io
            return io.StringIO(l3[int(path.split("/cpu")[2].split("/")[0])])
        return real_open(path, *a, **k)

    monkeypatch.setattr("builtins.open", fake_open)
    got = bench.spread_cpus(list(range(16)))
    assert got == [0, 8, 1, 9, 2, 10, 3, 11, 4, 12, 5, 13, 6, 14, 7, 15]
    assert bench.spread_cpus(list(range(32)))[:4] == [0, 8, 16, 24]


def test_cpu_baseline_reports_both_placements():
    """cpu_baseline times the reference loop with the threads on the first allowed CPUs and dealt over
    the L3 caches, and reports the faster as the baseline (a short sample over one 1M batch)."""
    import numpy as np

    import netbricks_amd as nb

    buf, _, _ = nb.make_trace(bench.BATCH, 0, seed=5)
    lut = nb.build_lut([f"backend-{i}" for i in range(bench.N_BACKENDS)], bench.TABLE)
    r = bench.cpu_baseline([buf], lut, target_cpu_s=0.2)
    assert r["packed_mpps"] > 0 and r["spread_l3_mpps"] > 0
    assert r["value"] == round(max(r["packed_mpps"], r["spread_l3_mpps"]), 1) or \
        abs(r["value"] - max(r["packed_mpps"], r["spread_l3_mpps"])) < 0.11
    assert np.isfinite(r["single_core_mpps"])


def test_idle_cpus_puts_busy_cpus_last(monkeypatch):
    """idle_cpus (the drop-in pipelines' and the CPU baseline's placement): CPUs busier than 20 % over
    the sample go last, the order otherwise kept."""
    import io

    samples = iter([
        "cpu  0 0 0 0 0 0 0 0\ncpu0 100 0 0 900 0 0 0 0\ncpu1 100 0 0 900 0 0 0 0\ncpu2 100 0 0 900 0 0 0 0\n",
        "cpu  0 0 0 0 0 0 0 0\ncpu0 105 0 0 995 0 0 0 0\ncpu1 190 0 0 910 0 0 0 0\ncpu2 110 0 0 990 0 0 0 0\n",
    ])
    real_open = open

    def fake_open(path, *a, **k):
        if path == "/proc/stat":
            return io.StringIO(next(samples))
        return real_open(path, *a, **k)

    monkeypatch.setattr("builtins.open", fake_open)
    idle, busy = bench.idle_cpus([0, 1, 2], sample_s=0.0)
    assert idle == [0, 2] and busy == [1]
