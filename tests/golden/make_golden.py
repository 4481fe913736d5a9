#!/usr/bin/env python3
"""Generate the committed golden fixtures from the Python oracle (oracle/maglev_ref.py).

Run once here (no GPU); the outputs are small data files:
  lut_golden.json   Maglev LUT digests/heads/counts + per-name (offset, skip) for three backend sets
  packets.npz       ~4.4k packets (synthetic UDP/TCP + hand-built edge cases) with expected
                    flow hashes, backends (3- and 65-backend LUTs) and MAC-swapped first 12 bytes
  lemmy.json        the reference's macswap fixture (http_lemmy.pcap) through the oracle

The reference itself cannot be built here, so these vectors come from the
independent restatement; http_lemmy.pcap + macswap_expect.out are the reference's own data
(test/macswap/data/) and pin the MAC swap.
"""
from __future__ import annotations

import hashlib
import json
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import maglev_ref as ref  # noqa: E402

NAMESETS = {
    "stooges_65537": (["Larry", "Curly", "Moe"], 65537),       # test/maglev/src/main.rs:36, nf.rs:90
    "backend65_65537": ([f"backend-{i}" for i in range(65)], 65537),   # BASELINE C1/C2
    "be1000_655373": ([f"be{i}" for i in range(1000)], 655373),        # BASELINE C3
}


def lut_entry(names, m):
    lut = ref.generate_lut(names, m)
    arr = np.array(lut, dtype=np.uint16)
    counts = np.bincount(arr, minlength=len(names))
    return lut, {
        "n": len(names),
        "m": m,
        "names_head": names[:8],
        "offset_skip_head": [list(ref.offset_skip_for_name(n, m)) for n in names[:8]],
        "head": arr[:64].tolist(),
        "tail": arr[-16:].tolist(),
        "counts_min": int(counts.min()),
        "counts_max": int(counts.max()),
        "counts_head": counts[:8].tolist(),
        "sha256_u16le": hashlib.sha256(arr.astype("<u2").tobytes()).hexdigest(),
    }


def ipv4_csum(h: bytes) -> int:
    s = sum(struct.unpack("!10H", h))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF


def frame(rng, length, ihl=5, proto=17, ethertype=0x0800):
    f = bytearray(rng.integers(0, 256, max(length, 1), dtype=np.uint8).tobytes())[:length]
    if length >= 14:
        f[12:14] = struct.pack("!H", ethertype)
    if length >= 34 and ethertype == 0x0800:
        ip = bytearray(f[14:34])
        ip[0] = 0x40 | ihl
        ip[9] = proto
        ip[10:12] = b"\0\0"
        ip[10:12] = struct.pack("!H", ipv4_csum(bytes(ip)))
        f[14:34] = ip
    elif length > 14:
        f[14] = (0x40 | ihl) if ethertype == 0x0800 else f[14]
    return f


def make_packets():
    rng = np.random.default_rng(0x5EED)
    frames = []
    # synthetic UDP/TCP with a few hundred repeating flows, 60..1514 B
    flows = [rng.integers(0, 256, 12, dtype=np.uint8).tobytes() for _ in range(300)]
    for i in range(4096):
        ln = int(rng.choice([60, 60, 60, 64, 96, 128, 200]))
        f = frame(rng, ln, proto=int(rng.choice([17, 6])))
        fl = flows[int(rng.integers(0, len(flows)))]
        f[26:34] = fl[:8]       # src, dst
        f[34:38] = fl[8:12]     # ports (IHL 5)
        frames.append(f)
    # edge cases: every IHL, runts, boundary lengths, non-IPv4, empty
    for ihl in range(16):
        for ln in (0, 1, 13, 14, 15, 33, 34, 37, 38, 47, 48, 49, 60, 63, 64, 65, 77, 78, 79, 100):
            frames.append(frame(rng, ln, ihl=ihl))
    for et in (0x86DD, 0x0806, 0x8100, 0x88A8):
        for ln in (60, 64, 100):
            frames.append(frame(rng, ln, ethertype=et))
    return frames


def main():
    golden = {}
    luts = {}
    for key, (names, m) in NAMESETS.items():
        print(f"LUT {key} ...", flush=True)
        luts[key], golden[key] = lut_entry(names, m)
    with open(os.path.join(HERE, "lut_golden.json"), "w") as fh:
        json.dump(golden, fh, indent=1)

    frames = make_packets()
    n = len(frames)
    off = np.zeros(n, dtype=np.uint32)
    lens = np.array([len(f) for f in frames], dtype=np.uint16)
    pos = 0
    for i, f in enumerate(frames):
        off[i] = pos
        pos += (len(f) + 63) // 64 * 64 + 64
    buf = np.zeros(pos, dtype=np.uint8)
    for i, f in enumerate(frames):
        buf[off[i]:off[i] + len(f)] = np.frombuffer(bytes(f), dtype=np.uint8) if len(f) else []
    hashes = np.zeros(n, dtype=np.uint64)
    hash_ok = np.zeros(n, dtype=np.uint8)
    be3 = np.zeros(n, dtype=np.uint16)
    be65 = np.zeros(n, dtype=np.uint16)
    mac12 = np.zeros((n, 12), dtype=np.uint8)
    for i, f in enumerate(frames):
        flow = ref.extract_flow(bytes(f[14:])) if len(f) >= 14 else None
        if flow is not None:
            hashes[i] = ref.flow_hash(flow)
            hash_ok[i] = 1
        g3 = bytearray(f)
        be3[i] = ref.process_packet(g3, luts["stooges_65537"])
        g65 = bytearray(f)
        be65[i] = ref.process_packet(g65, luts["backend65_65537"])
        mac12[i, :min(12, len(g65))] = np.frombuffer(bytes(g65[:12]), dtype=np.uint8)
    perm65, counts65 = ref.group_perm(be65.tolist(), 65)
    np.savez_compressed(os.path.join(HERE, "packets.npz"), buf=buf, off=off, len=lens, flow_hash=hashes,
                        flow_ok=hash_ok, backend3=be3, backend65=be65, mac12=mac12,
                        perm65=np.array(perm65, dtype=np.uint32), counts65=np.array(counts65, dtype=np.uint32))

    # the reference's own macswap fixture through the oracle
    data = open(os.path.join(HERE, "http_lemmy.pcap"), "rb").read()
    pos, out = 24, []
    while pos + 16 <= len(data):
        _, _, incl, _ = struct.unpack("<IIII", data[pos:pos + 16])
        f = bytearray(data[pos + 16:pos + 16 + incl])
        pos += 16 + incl
        flow = ref.extract_flow(bytes(f[14:]))
        g = bytearray(f)
        b3 = ref.process_packet(g, luts["stooges_65537"])
        out.append({"len": len(f), "flow_hash": f"{ref.flow_hash(flow):016x}", "backend3": b3,
                    "backend65": ref.process_packet(bytearray(f), luts["backend65_65537"]),
                    "swapped_head12": g[:12].hex()})
    with open(os.path.join(HERE, "lemmy.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(f"wrote {n} packets, {len(out)} lemmy frames")


if __name__ == "__main__":
    main()
