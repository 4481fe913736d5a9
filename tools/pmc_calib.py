#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE calibration from two rocprofv3 --pmc passes of tools/membench.

Every membench dispatch moves a known byte count (64 MiB buffers; IMIX windows: 1M x 64 B at scattered
64-B-aligned offsets + 4-B offsets): this divides each counter (KB, x 1024) by that count per access
shape, so that the bench's PMC traffic figures (FETCH_SIZE x 2 + WRITE_SIZE, MI355X_MICROARCH.md's HBM
section) are checked on the shapes the classify kernels use — 16-B-per-lane streaming reads (the tile
loads), whole-line rewrites (in place, nt or sc1 stores) and the IMIX window gathers.

Usage: pmc_calib.py <fetch dir> <write dir> [out.json]
"""
import csv
import json
import os
import re
import sys

B = 64 << 20          # one membench buffer
N_WIN = 1 << 20       # IMIX windows per dispatch


def rows(d, counter):
    for dp, _, files in os.walk(d):
        for f in files:
            if f.endswith("counter_collection.csv"):
                for r in csv.DictReader(open(os.path.join(dp, f))):
                    if r.get("Counter_Name") == counter:
                        yield r


def expected(name, grid):
    """(read bytes, write bytes, shape) of one dispatch, from the kernel's template arguments."""
    m = re.search(r"pattern(_p)?<(\d+), (\d+)(?:, (true|false))?>", name)
    if m:
        persistent, u, mode = bool(m.group(1)), int(m.group(2)), int(m.group(3))
        nt = m.group(4) == "true"
        blocks = grid // 256
        rd = B if persistent else blocks * 256 * u * 16
        wr = {0: 0, 1: rd, 2: rd / 4, 3: rd, 4: rd / 4, 5: rd, 6: rd / 4, 7: rd}[mode]
        shape = {0: "read", 1: "rw full line", 2: "rw 16 B per 64 B", 3: "copy", 4: "read + dense 16 B/pkt",
                 5: "rw full line, nt stores", 6: "rw 16 B per 64 B, nt stores", 7: "rw full line, sc1 stores (ring)"}[mode]
        return rd, wr, f"{'persistent ' if persistent else ''}{shape}, U{u}{', nt loads' if nt else ''}"
    m = re.search(r"windows<(\d+)(?:, (true|false))?>", name)
    if m:
        mode, nt = int(m.group(1)), m.group(2) == "true"
        rd = 64 * N_WIN + 4 * N_WIN
        wr = {0: 0, 1: 64 * N_WIN, 2: 12 * N_WIN}[mode]
        shape = {0: "IMIX windows read", 1: "IMIX windows rewrite (nt)", 2: "IMIX windows + 12 B/pkt out"}[mode]
        return rd, wr, shape + (", nt loads" if nt else "")
    return None


def main():
    fetch, write = sys.argv[1], sys.argv[2]
    acc = {}
    for counter, d in (("FETCH_SIZE", fetch), ("WRITE_SIZE", write)):
        for r in rows(d, counter):
            name, grid = r["Kernel_Name"], int(r.get("Grid_Size", 0))
            e = expected(name, grid)
            if e is None:
                continue
            a = acc.setdefault((name, grid), {"exp": e, "FETCH_SIZE": [], "WRITE_SIZE": []})
            a[counter].append(float(r["Counter_Value"]) * 1024.0)
    out = []
    for (name, grid), a in acc.items():
        rd, wr, shape = a["exp"]
        f = sum(a["FETCH_SIZE"]) / max(len(a["FETCH_SIZE"]), 1)
        w = sum(a["WRITE_SIZE"]) / max(len(a["WRITE_SIZE"]), 1)
        out.append({"shape": shape, "grid": grid, "dispatches": len(a["FETCH_SIZE"]),
                    "read_bytes": rd, "fetch_size_bytes": round(f), "fetch_ratio": round(f / rd, 4) if rd else None,
                    "write_bytes": wr, "write_size_bytes": round(w),
                    "write_ratio": round(w / wr, 4) if wr else None})
    for o in out:
        print(f"{o['shape'][:52]:52s} FETCH/read {o['fetch_ratio']!s:8s} WRITE/write {o['write_ratio']!s:8s} "
              f"({o['dispatches']} dispatches)")
    if len(sys.argv) > 3:
        json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
