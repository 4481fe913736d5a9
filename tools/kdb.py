#!/usr/bin/env python3
"""Per-kernel, per-launch-shape duration summary from a rocprofv3 SQLite database (run_results.db).

  python tools/kdb.py <dir-or-db> [name-substring ...]

rocprofv3 of ROCm 7.2 writes its kernel trace to a rocpd SQLite database unless --output-format csv
is given; this reads its `kernels` view: one row per (kernel, grid, workgroup) with calls, mean and
median duration in microseconds, VGPRs, SGPRs and LDS bytes."""
import glob
import os
import re
import sqlite3
import statistics
import sys


def short(n):
    n = n.replace("void ", "").replace("nbg::(anonymous namespace)::", "")
    i = n.rfind("(")
    return n[:i] if n.endswith(")") and i > 0 else n


def main():
    p = sys.argv[1]
    dbs = [p] if p.endswith(".db") else glob.glob(os.path.join(p, "**", "*.db"), recursive=True)
    keys = sys.argv[2:]
    for db in dbs:
        c = sqlite3.connect(db)
        acc = {}
        for name, gx, wx, dur, vg, sg, lds in c.execute(
                "select name, grid_x, workgroup_x, duration, vgpr_count, sgpr_count, lds_size from kernels"):
            k = (short(name), gx // max(wx, 1), wx, vg, sg, lds)
            acc.setdefault(k, []).append(dur / 1000.0)
        print(f"# {db}")
        for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
            if keys and not any(s in k[0] for s in keys):
                continue
            print(f"{k[0][:64]:64s} wg {k[1]:6d}x{k[2]:4d} vgpr {k[3]:3d} sgpr {k[4]:3d} lds {k[5]:6d} "
                  f"n {len(v):5d} mean {statistics.mean(v):9.2f} med {statistics.median(v):9.2f} us")


if __name__ == "__main__":
    main()
