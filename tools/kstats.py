#!/usr/bin/env python3
"""Print a rocprofv3 kernel_stats.csv compactly (kernel names contain commas)."""
import csv
import sys

for row in csv.DictReader(open(sys.argv[1])):
    name = row["Name"]
    name = name.replace("void nbg::(anonymous namespace)::", "").replace("(nbg::ClassifyArgs)", "")
    print(f"{name[:70]:70s} calls {int(row['Calls']):6d} avg {float(row['AverageNs']) / 1e3:9.2f} us"
          f"  min {float(row['MinNs']) / 1e3:8.2f}  max {float(row['MaxNs']) / 1e3:8.2f}")
