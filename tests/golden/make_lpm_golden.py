#!/usr/bin/env python3
"""Generate the committed LPM / chain golden fixtures from the Python oracle (oracle/maglev_ref.py).

Run once here (no GPU):
  lpm_routes.json   the 105 routes test/lpm installs (test/lpm/src/nf.rs:106-210, extracted from the
                    reference source text as data), plus the seeded synthetic "mixed" route set
  lpm_golden.json   table digests (tbl24, used tbl_long) and lookup vectors for both route sets
  lpm_chain.npz     ~3k frames whose source addresses fall in the mixed routes, with the expected
                    lpm gate and Maglev backend (65 backends, M = 65537) of lpm() -> maglev()

The reference has no known-answer test for the LPM either: these vectors come from the
restatement (parity unpinned by reference outputs).
"""
from __future__ import annotations

import hashlib
import json
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
sys.path.insert(0, HERE)
import maglev_ref as ref  # noqa: E402
from make_golden import frame  # noqa: E402

REF_NF = "/root/reference/test/lpm/src/nf.rs"


def reference_routes():
    txt = open(REF_NF).read()
    pat = re.compile(r"insert_ipv4\(&Ipv4Addr::new\((\d+), (\d+), (\d+), (\d+)\), (\d+), (\d+)\)")
    out = []
    for m in pat.finditer(txt):
        a, b, c, d, plen, gate = map(int, m.groups())
        out.append([f"{a}.{b}.{c}.{d}", plen, gate])
    assert len(out) == 105, len(out)
    return out


def mixed_routes():
    """Masked prefixes of every length 8..32 under 10.0.0.0/8 and 172.16.0.0/12, gates 0..3
    (gate 3 >= the 3 lpm groups: the reference would panic in group_by), with /25-/32 routes
    nested in /24s that already carry a shorter route."""
    rng = np.random.default_rng(0x1F3)
    routes = [["10.0.0.0", 8, 1], ["172.16.0.0", 12, 2]]
    for plen in range(9, 33):
        for _ in range(24 if plen < 24 else 60):
            base = 0x0A000000 if rng.integers(0, 4) else 0xAC100000
            span = 24 if base == 0x0A000000 else 20
            ip = base | int(rng.integers(0, 1 << span))
            ip &= (0xFFFFFFFF << (32 - plen)) & 0xFFFFFFFF
            routes.append([f"{ip >> 24}.{(ip >> 16) & 255}.{(ip >> 8) & 255}.{ip & 255}", plen,
                           int(rng.integers(0, 4))])
    return routes


def table_of(routes):
    t = ref.IPLookup()
    for ip, plen, gate in routes:
        a = [int(x) for x in ip.split(".")]
        t.insert((a[0] << 24) | (a[1] << 16) | (a[2] << 8) | a[3], plen, gate)
    t.construct_table()
    return t


def probe_ips(routes, rng):
    ips = set()
    for ip, plen, _ in routes:
        a = [int(x) for x in ip.split(".")]
        v = (a[0] << 24) | (a[1] << 16) | (a[2] << 8) | a[3]
        span = 1 << (32 - plen)
        for x in (v, v - 1, v + 1, v + span - 1, v + span, v + int(rng.integers(0, span))):
            ips.add(x & 0xFFFFFFFF)
    ips.update(int(x) for x in rng.integers(0, 1 << 32, 2000, dtype=np.uint64))
    return np.array(sorted(ips), dtype=np.uint32)


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).astype("<u2").tobytes()).hexdigest()


def main():
    rng = np.random.default_rng(0x17A)
    sets = {"reference": reference_routes(), "mixed": mixed_routes()}
    with open(os.path.join(HERE, "lpm_routes.json"), "w") as fh:
        json.dump({"reference_source": "test/lpm/src/nf.rs:106-210", **sets}, fh, indent=0)
    golden, tables = {}, {}
    for key, routes in sets.items():
        t = table_of(routes)
        tables[key] = t
        ips = probe_ips(routes, rng)
        gates = np.array([t.lookup_entry(int(x)) for x in ips], dtype=np.uint16)
        golden[key] = {"n_routes": len(routes), "long_used": t.current_tbl_long,
                       "tbl24_sha256": digest(t.tbl24), "tbl_long_sha256": digest(t.tbl_long[:t.current_tbl_long]),
                       "ips": ips.tolist(), "gates": gates.tolist()}
        print(f"{key}: {len(routes)} routes, tbl_long {t.current_tbl_long}, {ips.size} probes, "
              f"gate hist {np.bincount(gates).tolist()}")
    with open(os.path.join(HERE, "lpm_golden.json"), "w") as fh:
        json.dump(golden, fh)

    # chain frames: sources drawn from the mixed routes (plus runts / IHL edge cases)
    t = tables["mixed"]
    lut = ref.generate_lut([f"backend-{i}" for i in range(65)], 65537)
    mixed = sets["mixed"]
    frames = []
    for i in range(3000):
        ln = int(rng.choice([60, 60, 64, 96, 128]))
        f = frame(rng, ln, proto=int(rng.choice([17, 6])))
        ip, plen, _ = mixed[int(rng.integers(0, len(mixed)))]
        a = [int(x) for x in ip.split(".")]
        v = ((a[0] << 24) | (a[1] << 16) | (a[2] << 8) | a[3]) + int(rng.integers(0, 1 << (32 - plen)))
        f[26:30] = int(v & 0xFFFFFFFF).to_bytes(4, "big")
        frames.append(f)
    for ihl in (0, 4, 5, 6, 15):
        for ln in (0, 13, 14, 33, 34, 37, 38, 47, 48, 60, 78, 79):
            f = frame(rng, ln, ihl=ihl)
            if ln >= 30:
                f[26:30] = bytes([10, 1, 2, 3])
            frames.append(f)
    n = len(frames)
    off = np.zeros(n, dtype=np.uint32)
    lens = np.array([len(f) for f in frames], dtype=np.uint16)
    pos = 0
    for i, f in enumerate(frames):
        off[i] = pos
        pos += (len(f) + 63) // 64 * 64 + 64
    buf = np.zeros(pos, dtype=np.uint8)
    gate = np.zeros(n, dtype=np.uint16)
    backend = np.zeros(n, dtype=np.uint16)
    for i, f in enumerate(frames):
        if len(f):
            buf[off[i]:off[i] + len(f)] = np.frombuffer(bytes(f), dtype=np.uint8)
        gate[i], backend[i] = ref.process_chain(bytes(f), t, lut, 3)
    perm, counts = ref.group_perm(backend.tolist(), 65)
    np.savez_compressed(os.path.join(HERE, "lpm_chain.npz"), buf=buf, off=off, len=lens, gate=gate,
                        backend=backend, perm=np.array(perm, dtype=np.uint32),
                        counts=np.array(counts, dtype=np.uint32))
    print(f"chain: {n} frames, gate hist {np.bincount(gate[gate != 0xFFFF]).tolist()}, "
          f"sentinel backends {(backend == 0xFFFF).sum()}")


if __name__ == "__main__":
    main()
