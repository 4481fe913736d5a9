#!/usr/bin/env python3
"""Mean counter values per dispatch, per kernel, from a rocprofv3 --pmc run directory."""
import csv
import os
import sys
from collections import defaultdict


def _name(n):
    """Kernel name with its template arguments, without the parameter list."""
    n = n[:n.rfind("(")] if n.endswith(")") else n
    return n.replace("void nbg::(anonymous namespace)::", "")


def main():
    d = sys.argv[1]
    path = None
    for dp, _, files in os.walk(d):
        for f in files:
            if f.endswith("counter_collection.csv"):
                path = os.path.join(dp, f)
    acc = defaultdict(lambda: defaultdict(list))
    for row in csv.DictReader(open(path)):
        acc[_name(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in sorted(acc.items()):
        print(f"{k:72s} " + "  ".join(f"{c} {sum(v) / len(v):14.0f} (n={len(v)})" for c, v in sorted(cs.items())))


if __name__ == "__main__":
    main()
