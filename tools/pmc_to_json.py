#!/usr/bin/env python3
"""HBM bytes per launch of the classify and group kernels from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE, separate runs of `bench.py --streams 1`), with the gfx950
correction of MI355X_MICROARCH.md's HBM section: FETCH_SIZE counts 128-B requests as 64 B
(x2); WRITE_SIZE is read as is.  Both counters are in KB.

usage: pmc_to_json.py <pmc_FETCH_SIZE dir> <pmc_WRITE_SIZE dir> <round> > profiles/pmc_rNN.json
"""
import csv
import json
import os
import sys
from collections import defaultdict


def per_kernel(d, counter):
    acc = defaultdict(list)
    for row in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if row["Counter_Name"] != counter:
            continue
        name = row["Kernel_Name"]
        key = ("classify" if ("classify_kernel" in name or "classify_stream_kernel" in name)
               else ("group" if "group_kernel" in name else None))
        if key:
            acc[key].append(float(row["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def main():
    fdir, wdir, rnd = sys.argv[1], sys.argv[2], int(sys.argv[3])
    f, nf = per_kernel(fdir, "FETCH_SIZE")
    w, nw = per_kernel(wdir, "WRITE_SIZE")
    pkts = 1 << 20
    out = {
        "round": rnd,
        "command": "rocprofv3 --pmc {FETCH_SIZE|WRITE_SIZE} --kernel-trace -- python bench.py --streams 1 "
                   "--steps 50 --warmup 10 --no-cpu-baseline",
        "kernel": "classify_kernel<GlobalU8, F4, HIST> (in-place MAC swap, C2)",
        "pkts_per_launch": pkts,
        "launches": {"fetch": nf, "write": nw},
        "correction": "FETCH_SIZE x2 (gfx950 tallies 128-B requests as 64 B); WRITE_SIZE as read; KB = 1024 B",
        "classify_read_bytes_per_launch": 2 * f.get("classify", 0.0),
        "classify_write_bytes_per_launch": w.get("classify", 0.0),
        "classify_hbm_bytes_per_launch": 2 * f.get("classify", 0.0) + w.get("classify", 0.0),
        "algorithmic_bytes_per_launch": pkts * 78,
        "group_kernel_read_bytes": 2 * f.get("group", 0.0),
        "group_kernel_write_bytes": w.get("group", 0.0),
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
