#!/usr/bin/env python3
"""Phase timeline of the group kernel (measurement only; the product source is never modified).

  python tools/gprobe.py build          # patched copy of csrc -> tools/ab/lib_gprobe.so (CPU, hipcc)
  python tools/gprobe.py run [--n N]    # on the GPU: C2 (65 bins) and C3 (1000 bins) group launches

`build` copies netbricks_amd/csrc + include into tools/ab/gprobe_src, inserts timestamp stores at the
phase boundaries of group_kernel (lane 0 of every wave of every 32nd block: the shader clock at each
boundary; thread 0 of every block: the 100 MHz wall clock at entry and exit) and a readout entry point,
and builds it.  `run` loads that library through NBG_LIB_OVERRIDE, groups a 1M batch (one stream,
synchronised, the last of several launches is the one read back) and prints per-phase medians.
"""
import os
import re
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tools", "ab", "gprobe_src")
LIB = os.path.join(ROOT, "tools", "ab", "lib_gprobe.so")

PHASES = ["entry", "loads_issued", "ranked", "B1", "sums_scan1", "B2", "bases_scan2", "B3", "sorted", "B4",
          "stores", "end"]

PROBE_DEFS = r"""
__device__ unsigned long long g_gprobe[64 * 8 * 12];  // inside nbg::(anonymous)
__device__ unsigned long long g_gwall[4096 * 2];
#define NBG_GP(k) do { if (blockIdx.x % 32u == 0u && blockIdx.x / 32u < 64u && (threadIdx.x & 63u) == 0u) \
  g_gprobe[((blockIdx.x / 32u) * 8u + (threadIdx.x >> 6)) * 12u + (k)] = __builtin_readcyclecounter(); } while (0)
#define NBG_GW(k) do { if (threadIdx.x == 0u && blockIdx.x < 4096u) g_gwall[blockIdx.x * 2u + (k)] = wall_clock64(); } while (0)
"""

READOUT = r"""
extern "C" int nbg_debug_gprobe(unsigned long long* phase, unsigned long long* wall) {
  if (hipMemcpyFromSymbol(phase, HIP_SYMBOL(nbg::g_gprobe), sizeof(nbg::g_gprobe)) != hipSuccess) return -5;
  if (hipMemcpyFromSymbol(wall, HIP_SYMBOL(nbg::g_gwall), sizeof(nbg::g_gwall)) != hipSuccess) return -5;
  return 0;
}
"""


def _insert(text, anchor, line, before=True, count=1):
    i = text.find(anchor)
    if i < 0:
        raise SystemExit(f"gprobe: anchor not found: {anchor!r}")
    if count == 1 and text.find(anchor, i + 1) >= 0:
        raise SystemExit(f"gprobe: anchor not unique in the group kernel: {anchor!r}")
    j = i if before else i + len(anchor)
    return text[:j] + line + text[j:]


def patch(src):
    beg = src.index("void group_kernel(GroupMulti gm) {")
    end = src.index("// group_direct_kernel:")
    g = src[beg:end]
    g = _insert(g, "  const uint32_t c = blockIdx.x - bj * gm.per;  // partition of batch bj\n",
                "  NBG_GW(0);\n  NBG_GP(0);\n", before=False)
    g = _insert(g, "  const unsigned long long lt = (lane == 0)", "  NBG_GP(1);\n")
    g = _insert(g, "  if (perm) rank_chunk(pbeg);\n", "  NBG_GP(2);\n", before=False)
    g = _insert(g, "  lds_sync();  // (B1) base / tot zeroed, every wave's counts of the first chunk in LDS\n",
                "  NBG_GP(3);\n", before=False)
    g = _insert(g, "  lds_sync();  // (B2)\n", "  NBG_GP(4);\n")
    g = _insert(g, "  lds_sync();  // (B2)\n", "  NBG_GP(5);\n", before=False)
    g = _insert(g, "  uint32_t ctotal = chunk_scan_end();", "  NBG_GP(6);\n")
    g = _insert(g, "    lds_sync();  // (B3)\n", "    NBG_GP(7);\n", before=False)
    g = _insert(g, "    lds_sync();  // (B4)\n", "    NBG_GP(8);\n")
    g = _insert(g, "    lds_sync();  // (B4)\n", "    NBG_GP(9);\n", before=False)
    tail = g.rindex("  zero_next();\n}")
    g = g[:tail] + "  NBG_GP(10);\n  zero_next();\n  NBG_GP(11);\n  NBG_GW(1);\n}" + g[tail + len("  zero_next();\n}"):]
    out = src[:beg] + g + src[end:]
    # definitions after the anonymous-namespace helpers (wall_clock64 must be declared first)
    k = out.index("template <int SCAN, int BITS>\n// Blocks [j * gm.per")
    out = out[:k] + PROBE_DEFS + out[k:]
    return out + READOUT


def build():
    if os.path.isdir(SRC):
        shutil.rmtree(SRC)
    os.makedirs(os.path.join(SRC, "netbricks_amd"))
    shutil.copytree(os.path.join(ROOT, "netbricks_amd", "csrc"), os.path.join(SRC, "netbricks_amd", "csrc"),
                    ignore=shutil.ignore_patterns("*.o", "*.s"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(SRC, "include"))
    kf = os.path.join(SRC, "netbricks_amd", "csrc", "maglev_kernels.hip")
    with open(kf) as f:
        s = f.read()
    with open(kf, "w") as f:
        f.write(patch(s))
    subprocess.check_call(["make", "-s", "-C", os.path.join(SRC, "netbricks_amd", "csrc"), f"OUT={LIB}",
                           "EXTRA=-Wno-undef"])
    print("built", LIB)


def run(n):
    import ctypes as C

    import numpy as np
    os.environ["NBG_LIB_OVERRIDE"] = LIB
    sys.path.insert(0, ROOT)
    import torch

    import netbricks_amd as nb
    from netbricks_amd import _lib
    lib = _lib._load()
    fn = lib.nbg_debug_gprobe
    fn.argtypes = [C.c_void_p, C.c_void_p]
    dev = torch.device("cuda:0")
    for label, nbk, m, mode in (("C2 65 backends", 65, 65537, 0), ("C3 1000 backends", 1000, 655373, 1)):
        mg = nb.Maglev([f"backend-{i}" for i in range(nbk)], m)
        mg.reserve(n)
        buf, off, ln = nb.make_trace(n, mode, seed=7)
        pk = torch.from_numpy(buf).to(dev)
        backend = torch.empty(n, dtype=torch.uint16, device=dev)
        perm = torch.empty(n, dtype=torch.uint32, device=dev)
        counts = torch.empty(nbk + 1, dtype=torch.uint32, device=dev)
        kw = {} if mode == 0 else dict(offsets=torch.from_numpy(off.view(np.int32)).to(dev).view(torch.uint32),
                                       lens=torch.from_numpy(ln.view(np.int16)).to(dev).view(torch.uint16),
                                       owned_windows=True)
        for _ in range(6):
            mg.group_by(pk, n, backend=backend, perm=perm, counts=counts, swap_macs=False, **kw)
            torch.cuda.synchronize()
        ph = np.zeros(64 * 8 * 12, dtype=np.uint64)
        wall = np.zeros(4096 * 2, dtype=np.uint64)
        assert fn(ph.ctypes.data, wall.ctypes.data) == 0
        nparts = (n + 4095) // 4096
        ph = ph.reshape(64, 8, 12)[: (nparts + 31) // 32].astype(np.int64)
        d = np.diff(ph[:, :, :len(PHASES)], axis=2)  # cycles between consecutive phase points
        print(f"# {label}, {n} packets, {nparts} blocks; shader cycles per phase (median over sampled waves; "
              f"max over waves in brackets)")
        for k in range(len(PHASES) - 1):
            v = d[:, :, k].ravel()
            print(f"  {PHASES[k]:>10s} -> {PHASES[k + 1]:<10s} {int(np.median(v)):8d}  [{int(v.max()):8d}]")
        tot = (ph[:, :, len(PHASES) - 1] - ph[:, :, 0]).ravel()
        print(f"  {'total':>24s} {int(np.median(tot)):8d}  [{int(tot.max()):8d}]")
        w = wall.reshape(4096, 2)[:nparts].astype(np.int64)
        t0 = w[:, 0].min()
        print(f"  wall (10 ns ticks from the first entry): entries {int(np.median(w[:, 0] - t0))} median, "
              f"{int((w[:, 0] - t0).max())} last; exits {int(np.median(w[:, 1] - t0))} median, "
              f"{int((w[:, 1] - t0).max())} last; block life median {int(np.median(w[:, 1] - w[:, 0]))}")
        mg.close()


if __name__ == "__main__":
    if len(sys.argv) < 2 or sys.argv[1] not in ("build", "run"):
        raise SystemExit(__doc__)
    if sys.argv[1] == "build":
        build()
    else:
        n = int(sys.argv[sys.argv.index("--n") + 1]) if "--n" in sys.argv else 1 << 20
        run(n)
