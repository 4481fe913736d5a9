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
