#!/usr/bin/env python3
"""Average duration of the LAST n dispatches of every kernel in a rocprofv3 kernel-trace CSV.
bench.py --multi-only runs each variant's multi-stream value pass first and its single-stream
kernel pass (the one the roofline uses) last, so the last n = its launches."""
import csv
import sys
from collections import defaultdict


def main():
    path, n = sys.argv[1], int(sys.argv[2])
    d = defaultdict(list)
    for r in csv.DictReader(open(path)):
        d[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    for k, v in sorted(d.items()):
        v.sort()
        last = [(e - s) / 1e3 for s, e in v[-n:]]
        print(f"{k[:70]:70s} last {len(last):4d} avg {sum(last) / len(last):9.2f} us  min {min(last):9.2f}")


if __name__ == "__main__":
    main()
