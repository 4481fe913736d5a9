#!/usr/bin/env python3
"""Summarise a rocprofv3 --pmc counter_collection.csv: mean of each counter per kernel name."""
import collections
import csv
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for row in csv.DictReader(open(sys.argv[1])):
    name = row.get("Kernel_Name", row.get("Kernel-Name", "?"))
    name = name.replace("void nbg::(anonymous namespace)::", "").replace("(nbg::ClassifyArgs)", "")[:60]
    acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
for name, cs in acc.items():
    print(name)
    for c, v in sorted(cs.items()):
        print(f"   {c:34s} {sum(v) / len(v):16.1f}  (n={len(v)})")
