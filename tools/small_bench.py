"""Small device-resident batches: per-call latency (synchronised) and back-to-back throughput on
one stream, full path (classify + grouping), 65 backends / 65537."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import netbricks_amd as nb

    mg = nb.Maglev([f"backend-{i}" for i in range(65)], 65537)
    out = {}
    for n in (32, 256, 1024, 4096, 16384, 65536):
        buf = torch.from_numpy(nb.make_trace(n, 0, seed=n)[0]).cuda()
        be = torch.empty(n, dtype=torch.uint16, device="cuda")
        pm = torch.empty(n, dtype=torch.uint32, device="cuda")
        ct = torch.empty(66, dtype=torch.uint32, device="cuda")
        for _ in range(20):
            mg.group_by(buf, n, backend=be, perm=pm, counts=ct)
        torch.cuda.synchronize()
        lat = []
        for _ in range(200):
            t = time.perf_counter()
            mg.group_by(buf, n, backend=be, perm=pm, counts=ct)
            torch.cuda.synchronize()
            lat.append(time.perf_counter() - t)
        lat.sort()
        k = 1000
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(k):
            mg.group_by(buf, n, backend=be, perm=pm, counts=ct)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / k
        out[n] = {"latency_us_median": round(lat[len(lat) // 2] * 1e6, 1), "back_to_back_us": round(dt * 1e6, 2),
                  "mpps_back_to_back": round(n / dt / 1e6, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
