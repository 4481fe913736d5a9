#!/usr/bin/env python3
"""Kernel durations by launch shape from a rocprofv3 kernel trace (`--kernel-trace --output-format csv`).

rocprofv3's --stats summary keys kernels by name only, so launches of one kernel with different
shapes (a 1M batch, 4 x 1M batches in one multi-batch launch, a 131,072-packet shard) land in one
row.  This groups the dispatches of the trace by (kernel, grid, workgroup, LDS bytes) and, when the
bench's run is split by `--multi-only`, by template instantiation; it prints and writes a CSV with
calls, mean / median / min / max microseconds per shape, so that every `avg_launch_us` and `frac` of
the bench line can be recomputed from a committed file.  `alone_*` covers only the dispatches that
overlapped no other dispatch in time: the bench times its `roofline` / `avg_launch_us` figures with
the kernel alone on one stream, while its multi-stream passes co-run classify and grouping.

Usage: kshapes.py <dir or kernel_trace.csv> [out.csv]
"""
import csv
import os
import statistics
import sys


def find_trace(p):
    if os.path.isfile(p):
        return p
    for dp, _, files in os.walk(p):
        for f in files:
            if f.endswith("kernel_trace.csv"):
                return os.path.join(dp, f)
    raise SystemExit(f"no kernel_trace.csv under {p}")


def short(name):
    name = name.replace("void nbg::(anonymous namespace)::", "").replace("void nbg::", "")
    return name.split("(nbg::")[0].split("(unsigned")[0].strip()


def main():
    path = find_trace(sys.argv[1])
    rows = list(csv.DictReader(open(path)))
    # a dispatch is "alone" when no other dispatch's [start, end) intersects its own
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), i) for i, r in enumerate(rows))
    alone = set()
    max_end = -1
    for k, (s0, e0, i) in enumerate(iv):
        nxt = iv[k + 1][0] if k + 1 < len(iv) else None
        if max_end <= s0 and (nxt is None or nxt >= e0):
            alone.add(i)
        max_end = max(max_end, e0)
    shapes = {}
    lone = {}
    for i, r in enumerate(rows):
        name = short(r.get("Kernel_Name", ""))
        grid = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
        wg = int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 0)) or 0)
        lds = int(r.get("Group_Segment_Size", r.get("LDS_Block_Size", 0)) or 0)
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        key = (name, grid // max(wg, 1), wg, lds)
        shapes.setdefault(key, []).append(dur)
        if i in alone:
            lone.setdefault(key, []).append(dur)
    out = []
    for (name, blocks, wg, lds), d in sorted(shapes.items(), key=lambda kv: -sum(kv[1])):
        out.append({"kernel": name, "workgroups": blocks, "workgroup_size": wg, "lds_bytes": lds, "calls": len(d),
                    "mean_us": round(statistics.fmean(d), 3), "median_us": round(statistics.median(d), 3),
                    "min_us": round(min(d), 3), "max_us": round(max(d), 3), "total_us": round(sum(d), 1),
                    "alone_calls": len(lone.get((name, blocks, wg, lds), [])),
                    "alone_mean_us": round(statistics.fmean(lone[(name, blocks, wg, lds)]), 3)
                    if lone.get((name, blocks, wg, lds)) else None})
    for o in out:
        print(f"{o['kernel'][:64]:64s} wg {o['workgroups']:6d}x{o['workgroup_size']:4d} lds {o['lds_bytes']:6d} "
              f"calls {o['calls']:6d} mean {o['mean_us']:10.3f} med {o['median_us']:10.3f} us"
              + (f"  alone {o['alone_calls']:5d} mean {o['alone_mean_us']:9.3f}" if o["alone_calls"] else ""))
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(out[0].keys()))
            w.writeheader()
            w.writerows(out)


if __name__ == "__main__":
    main()
