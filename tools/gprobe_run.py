#!/usr/bin/env python3
"""Group-kernel phase timestamps (diagnostic build with -DNBG_GPROBE via NBG_LIB_OVERRIDE): a few
single-stream full-path launches; the kernel printf()s the phase durations of three blocks."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import netbricks_amd as nb

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    nb_ = int(sys.argv[2]) if len(sys.argv) > 2 else 65
    m = int(sys.argv[3]) if len(sys.argv) > 3 else 65537
    kind = int(sys.argv[4]) if len(sys.argv) > 4 else 0  # 0: 64-B C2 slots, 1: IMIX with descriptors
    mg = nb.Maglev([f"backend-{i}" for i in range(nb_)], m)
    buf, off, ln = nb.make_trace(n, kind, seed=3)
    buf = torch.from_numpy(buf).cuda()
    kw = {}
    if kind:
        kw = dict(offsets=torch.from_numpy(off.astype(np.uint32)).cuda(), lens=torch.from_numpy(ln).cuda())
    for _ in range(3):
        mg.group_by(buf, n, **kw)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
