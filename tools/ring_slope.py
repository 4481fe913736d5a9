#!/usr/bin/env python3
"""Per-batch ring time from the completion stamps `bench.py` dumps (NBG_BENCH_DUMP=<dir>).

Each CSV holds (us_since_first, completed) samples of the relay's completion count during one ring
pass; the ring figure in the bench line is the least-squares slope of time over `completed` across the
middle three quarters of the samples (the ramp and the drain excluded).  Committed stamps:
profiles/r04_ring_stamps/.

Usage: ring_slope.py <csv or directory>...
"""
import csv
import glob
import os
import sys

import numpy as np


def slope(path):
    rows = np.array([[float(r["us_since_first"]), float(r["completed"])] for r in csv.DictReader(open(path))])
    n = len(rows)
    a, b = n // 8, n - n // 8
    return n, float(np.polyfit(rows[a:b, 1], rows[a:b, 0], 1)[0])


def main():
    files = []
    for p in sys.argv[1:] or ["profiles/r04_ring_stamps"]:
        files += sorted(glob.glob(os.path.join(p, "*.csv"))) if os.path.isdir(p) else [p]
    for f in files:
        n, us = slope(f)
        print(f"{os.path.basename(f):48s} samples {n:6d}  {us:8.3f} us per batch")


if __name__ == "__main__":
    main()
