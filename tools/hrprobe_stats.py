#!/usr/bin/env python3
"""Summarise a host-batch server probe dump (tools/runs/mk_hrprobe.sh): per ticket the GPU wall clock
(100 MHz) at claim, descriptor seen, body start, body end and completion word.  Prints the median and
90th percentile of each interval (us) and the tickets completed per second."""
import json
import sys

import numpy as np


def main(path):
    a = np.fromfile(path, dtype=np.uint64).reshape(-1, 5).astype(np.int64)
    a = a[(a > 0).all(axis=1)]
    a = a[len(a) // 10:]  # past the start
    us = lambda x: np.percentile(x / 100.0, [50, 90]).round(2).tolist()  # noqa: E731
    out = {"tickets": int(len(a)),
           "wait_for_post_us": us(a[:, 1] - a[:, 0]),
           "descriptor_us": us(a[:, 2] - a[:, 1]),
           "body_us": us(a[:, 3] - a[:, 2]),
           "fence_and_flag_us": us(a[:, 4] - a[:, 3]),
           "busy_us": us(a[:, 4] - a[:, 1]),
           "batches_per_s": round(len(a) / ((a[:, 4].max() - a[:, 1].min()) / 1e8), 0)}
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1])
