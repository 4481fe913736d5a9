#!/usr/bin/env python3
"""Group-kernel phase timestamps (diagnostic build with -DNBG_GPROBE via NBG_LIB_OVERRIDE): a few
single-stream full-path launches; the kernel printf()s the phase durations of three blocks."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import netbricks_amd as nb

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    mg = nb.Maglev([f"backend-{i}" for i in range(65)], 65537)
    buf = torch.from_numpy(nb.make_trace(n, 0, seed=3)[0]).cuda()
    for _ in range(3):
        mg.group_by(buf, n)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
