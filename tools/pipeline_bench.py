"""Throughput of the C++ operator mirror (netbricks_amd/host/nb_maglev: ReceiveBatch -> parse ->
swap -> group_by(maglev) -> merge -> send) on a large synthetic pcap, with the group_by batches
gathered into staging buffers or read in place from the registered mempool (--zero-copy 1).

    python tools/pipeline_bench.py --packets 1000000 --out gpurun_out/pipeline.json

The pcap is written to a temporary directory; the timed region is the scheduler loop only (the
capture is already in memory; no tx pcap is written).  One JSON object per (batch, zero_copy, rep).
"""
import argparse
import json
import os
import struct
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
NB = os.path.join(ROOT, "netbricks_amd", "host", "nb_maglev")


def write_pcap(path, buf, off, ln):
    n = off.size
    hdr = np.zeros((n, 4), dtype="<u4")
    hdr[:, 0] = np.arange(n, dtype=np.uint32)
    hdr[:, 2] = ln
    hdr[:, 3] = ln
    with open(path, "wb") as f:
        f.write(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 1))
        step = 65536
        for s in range(0, n, step):
            parts = []
            for i in range(s, min(n, s + step)):
                parts.append(hdr[i].tobytes())
                parts.append(buf[off[i]:off[i] + ln[i]].tobytes())
            f.write(b"".join(parts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=1000000)
    ap.add_argument("--imix", type=int, default=1)
    ap.add_argument("--backends", type=int, default=65)
    ap.add_argument("--batches", default="4096,32768")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from netbricks_amd import make_trace

    buf, off, ln = make_trace(args.packets, args.imix, seed=11)
    off = off.astype(np.int64)
    rows = []
    with tempfile.TemporaryDirectory() as td:
        rx = os.path.join(td, "in.pcap")
        write_pcap(rx, buf, off, ln)
        print(f"pcap {os.path.getsize(rx) / 1e6:.1f} MB, {args.packets} frames", flush=True)
        for batch in [int(b) for b in args.batches.split(",")]:
            for zc in (0, 1):
                for rep in range(args.reps):
                    cmd = [NB, "--rx", rx, "--batch", str(batch), "--backends", str(args.backends), "--zero-copy", str(zc)]
                    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
                    if r.returncode != 0:
                        print(r.stderr, file=sys.stderr)
                        sys.exit(r.returncode)
                    d = json.loads(r.stdout.strip().splitlines()[-1])
                    d.pop("groups", None)
                    d.update(batch=batch, rep=rep, imix=bool(args.imix))
                    rows.append(d)
                    print(json.dumps(d), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
