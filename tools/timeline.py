"""Kernel timeline from a rocprofv3 --kernel-trace CSV: per-kernel start/end/queue for the last
`--last` kernels, and how long each kernel kind runs alone vs. next to others.

usage: python tools/timeline.py <run_kernel_trace.csv> [--last 40]"""
import argparse
import csv


def short(name):
    for k in ("classify_stream_desc_kernel", "classify_stream_kernel", "classify_kernel", "group_kernel",
              "scan_kernel", "hist_kernel"):
        if k in name:
            return "classify" if k.startswith("classify") else k.replace("_kernel", "")
    return name[:24]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last", type=int, default=40)
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.csv)))
    ks = []
    for r in rows:
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                   r.get("Stream_Id", r.get("Queue_Id", "?")), r.get("Queue_Id", "?")))
    ks = [k for k in ks if k[2] in ("classify", "group", "scan", "hist")]
    ks.sort()
    ks = ks[-args.last:]
    t0 = ks[0][0]
    for s, e, n, st, q in ks:
        print(f"{n:9s} stream {st:>3s} queue {q:>3s}  start {(s - t0) / 1e3:9.2f}  end {(e - t0) / 1e3:9.2f}  dur {(e - s) / 1e3:7.2f} us")
    # concurrency: sweep events
    ev = []
    for s, e, n, _, _ in ks:
        ev.append((s, 1, n))
        ev.append((e, -1, n))
    ev.sort()
    cur = {}
    last = ev[0][0]
    acc = {}
    for t, d, n in ev:
        key = tuple(sorted((k, v) for k, v in cur.items() if v))
        acc[key] = acc.get(key, 0) + (t - last)
        cur[n] = cur.get(n, 0) + d
        last = t
    tot = sum(acc.values())
    print(f"span {tot / 1e3:.1f} us over {len(ks)} kernels")
    for key, v in sorted(acc.items(), key=lambda x: -x[1])[:12]:
        print(f"  {v / tot * 100:5.1f} %  {dict(key)}")


if __name__ == "__main__":
    main()
