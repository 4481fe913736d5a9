"""TEST INFRASTRUCTURE ONLY — CPU oracle for the Maglev flow-steering path.

Pure-Python restatement of NetBricks' `test/maglev` hot path, written from the
Rust source (study only; nothing is imported or executed from the reference).
Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may
use anything under `oracle/`; the product path (`netbricks_amd`) never does.

Restated reference items (paths relative to the NetBricks repo root):

* `Maglev::offset_skip_for_name`  test/maglev/src/nf.rs:21-31
* `Maglev::generate_permutations` test/maglev/src/nf.rs:33-42
* `Maglev::generate_lut`          test/maglev/src/nf.rs:44-68
* `Maglev::lookup`                test/maglev/src/nf.rs:78-81
* `maglev()` per-packet closures  test/maglev/src/nf.rs:94-105
* `ipv4_extract_flow`             framework/src/utils/flow.rs:53-62
* `Flow` (repr(C, packed), LE)    framework/src/utils/flow.rs:10-18
* `flow_hash` / `ipv4_flow_hash`  framework/src/utils/flow.rs:96-110
* `MacHeader::swap_addresses`     framework/src/headers/mac.rs:140-145
* `MacHeader::offset` (feature `performance` => 14)  framework/src/headers/mac.rs:96-106
* `Packet::parse_header` / `get_payload` / `payload_size`
                                  framework/src/interface/packet.rs:258-260,392-399,467-472
* GroupBy producer FIFO semantics framework/src/operators/group_by.rs:43-55
* `IPLookup` (DIR-24-8) insert / construct_table / lookup_entry
                                  test/lpm/src/nf.rs:12-99
* `lpm()` pipeline (parse, swap, parse::<IpHeader>, group_by(3, lookup(src)))
                                  test/lpm/src/nf.rs:212-228; IpHeader size 20 headers/ip.rs:53-56

Third-party arithmetic (un-vendored crates, unpinned `"*"` in the reference):
* `fnv` crate `FnvHasher`: FNV-1a 64, offset 0xcbf29ce484222325, prime 0x100000001b3.
  Restated here from the published algorithm; pinned by the FNV spec vectors in tests.
* `twox-hash` 1.x `XxHash` (seed 0) = XXH64.  Computed here with the Python
  `xxhash` package 3.8.1 (upstream C library), which is the published algorithm.
* Rust `impl Hash for str` = `write(bytes); write_u8(0xff)`.

Parity status: the reference has no test that pins the hash, the LUT or the grouping
(SURVEY.md §4, §8c), and the reference cannot be built here.  This oracle is pinned by
(a) the FNV-1a / XXH64 published vectors, (b) the reference's own macswap golden output
(`test/macswap/data/expect.out`) for the MAC swap, and (c) agreement with the independent
C restatement in `oracle/maglev_oracle.c`.  Backend assignment itself is "parity
unpinned" by reference-produced outputs.
"""
from __future__ import annotations

import struct

import xxhash

FNV_OFFSET = 0xCBF29CE484222325
FNV_PRIME = 0x100000001B3
MASK64 = (1 << 64) - 1
ETH_HDR = 14            # MacHeader::offset() under feature "performance" (mac.rs:96-106)
LUT_EMPTY = 0x8000      # generate_lut's fill sentinel (nf.rs:46)
SENTINEL = 0xFFFF       # this build's "reference would panic" backend value


def fnv1a64(data: bytes) -> int:
    """FNV-1a 64 as the `fnv` crate's FnvHasher::write + finish."""
    h = FNV_OFFSET
    for b in data:
        h ^= b
        h = (h * FNV_PRIME) & MASK64
    return h


def rust_str_hash_bytes(name: str) -> bytes:
    """Bytes fed to a Hasher by Rust's `impl Hash for str` (write + write_u8(0xff))."""
    return name.encode("utf-8") + b"\xff"


def offset_skip_for_name(name: str, lsize: int) -> tuple[int, int]:
    """nf.rs:21-31: offset = XXH64 % M, skip = FNV % (M-1) + 1."""
    b = rust_str_hash_bytes(name)
    hash1 = fnv1a64(b)
    hash2 = xxhash.xxh64_intdigest(b, seed=0)
    return hash2 % lsize, hash1 % (lsize - 1) + 1


def generate_lut(names: list[str], lsize: int) -> list[int]:
    """nf.rs:33-68 (permutation rows computed on the fly instead of materialised)."""
    params = [offset_skip_for_name(n, lsize) for n in names]
    nxt = [0] * len(names)
    entry = [LUT_EMPTY] * lsize
    n = 0
    while n < lsize:
        for i, (off, skip) in enumerate(params):
            c = (off + nxt[i] * skip) % lsize
            while entry[c] != LUT_EMPTY:
                nxt[i] += 1
                if nxt[i] >= lsize:  # permutations[i][lsize] is out of bounds: the reference panics
                    raise IndexError("maglev: permutation exhausted (table size not coprime to skip)")
                c = (off + nxt[i] * skip) % lsize
            if entry[c] == LUT_EMPTY:
                entry[c] = i
                nxt[i] += 1
                n += 1
            if n >= lsize:
                break
    return entry


def extract_flow(payload: bytes):
    """flow.rs:53-62. Returns (src, dst, sport, dport, proto) or None where Rust panics."""
    if len(payload) < 1:
        return None
    port_start = (payload[0] & 0xF) * 4
    if len(payload) < 20 or len(payload) < port_start + 4:
        return None
    proto = payload[9]
    src = struct.unpack(">I", payload[12:16])[0]
    dst = struct.unpack(">I", payload[16:20])[0]
    sport = struct.unpack(">H", payload[port_start:port_start + 2])[0]
    dport = struct.unpack(">H", payload[port_start + 2:port_start + 4])[0]
    return src, dst, sport, dport, proto


def flow_bytes(flow) -> bytes:
    """`Flow` is #[repr(C, packed)] on little-endian x86-64 (flow.rs:10-18)."""
    src, dst, sport, dport, proto = flow
    return struct.pack("<IIHHB", src, dst, sport, dport, proto)


def flow_hash(flow) -> int:
    return fnv1a64(flow_bytes(flow))


def process_packet(frame: bytearray, lut: list[int], swap: bool = True) -> int:
    """One packet through parse -> transform(swap) -> group_fn. Mutates `frame`.

    data_len < 14: `parse_header` asserts (packet.rs:392-399) -> no swap, sentinel.
    Otherwise the MAC swap is applied (transform runs before group_by over the batch,
    transform_batch.rs:70-81), then the flow slice may panic -> sentinel.
    """
    if len(frame) < ETH_HDR:
        return SENTINEL
    if swap:
        dst = bytes(frame[0:6])
        frame[0:6] = frame[6:12]
        frame[6:12] = dst
    flow = extract_flow(bytes(frame[ETH_HDR:]))
    if flow is None:
        return SENTINEL
    h = flow_hash(flow)
    return lut[h % len(lut)]


def group_perm(backends: list[int], n_backends: int):
    """Per-group FIFO order (group_by.rs:46-51 + mpsc enqueue order): stable partition.

    Returns (perm, counts) with groups 0..n_backends-1 then the sentinel group.
    """
    bins = [n_backends if b == SENTINEL else b for b in backends]
    counts = [0] * (n_backends + 1)
    for b in bins:
        counts[b] += 1
    perm = sorted(range(len(bins)), key=lambda i: (bins[i], i))
    return perm, counts


# ---- test/lpm (chained before test/maglev in BASELINE config C5) -------------------------

TBL24_SIZE = (1 << 24) + 1   # nf.rs:19
RAW_SIZE = 33                # nf.rs:20
OVERFLOW_MASK = 0x8000       # nf.rs:21
IP_HDR = 20                  # IpHeader::size() (headers/ip.rs:53-56)


class IPLookup:
    """test/lpm/src/nf.rs:12-99.  raw_entries[len] maps prefix -> gate (HashMap::insert
    replaces).  construct_table visits one length's routes in ascending prefix order: the
    reference iterates a HashMap, whose order only matters when routes of one length overlap
    with different gates (never for masked prefixes) — the product uses the same rule."""

    def __init__(self):
        import numpy as np
        self.tbl24 = np.zeros(TBL24_SIZE, dtype=np.uint16)
        self.tbl_long = np.zeros(TBL24_SIZE, dtype=np.uint16)
        self.current_tbl_long = 0
        self.raw_entries = [dict() for _ in range(RAW_SIZE)]

    def insert(self, ip: int, plen: int, gate: int) -> None:
        if plen >= RAW_SIZE:
            raise IndexError("prefix length > 32 (the reference panics)")
        self.raw_entries[plen][ip & 0xFFFFFFFF] = gate & 0xFFFF

    def construct_table(self) -> None:
        for i in range(25):
            for k in sorted(self.raw_entries[i]):
                v = self.raw_entries[i][k]
                start = k >> 8
                end = start + (1 << (24 - i))
                if end > TBL24_SIZE:
                    raise IndexError("tbl24 fill past its end (the reference panics)")
                self.tbl24[start:end] = v
        for i in range(25, RAW_SIZE):
            for k in sorted(self.raw_entries[i]):
                v = self.raw_entries[i][k]
                addr = k
                t24entry = int(self.tbl24[addr >> 8])
                if t24entry & OVERFLOW_MASK == 0:
                    ctlb = self.current_tbl_long
                    if ctlb + 256 > TBL24_SIZE:
                        raise IndexError("tbl_long exhausted (the reference panics)")
                    start = ctlb + (addr & 0xFF)
                    end = start + (1 << (32 - i))
                    for j in range(ctlb, ctlb + 256):
                        self.tbl_long[j] = t24entry if (j < start or j >= end) else v
                    self.tbl24[addr >> 8] = ((ctlb >> 8) & 0xFFFF) | OVERFLOW_MASK   # `as u16`
                    self.current_tbl_long += 256
                else:
                    start = ((t24entry & ~OVERFLOW_MASK & 0xFFFF) << 8) + (addr & 0xFF)
                    end = start + (1 << (32 - i))
                    if end > TBL24_SIZE:
                        raise IndexError("tbl_long fill past its end (the reference panics)")
                    self.tbl_long[start:end] = v

    def lookup_entry(self, ip: int) -> int:
        t24entry = int(self.tbl24[ip >> 8])
        if t24entry & OVERFLOW_MASK:
            return int(self.tbl_long[((t24entry & ~OVERFLOW_MASK & 0xFFFF) << 8) + (ip & 0xFF)])
        return t24entry


def process_chain(frame: bytes, table: IPLookup, lut: list[int], lpm_groups: int = 3):
    """One packet through lpm() then maglev() (frames are not modified: the swaps cancel).

    Returns (gate, backend): gate = SENTINEL where lpm cannot parse the packet (data_len <
    14 + 20: parse::<MacHeader>/parse::<IpHeader> asserts); backend = SENTINEL where either
    NF would panic (also gate >= lpm_groups: group index out of range in group_by.rs:48).
    """
    if len(frame) < ETH_HDR + IP_HDR:
        return SENTINEL, SENTINEL
    src = struct.unpack(">I", bytes(frame[ETH_HDR + 12:ETH_HDR + 16]))[0]   # IpHeader::src (ip.rs:101-103)
    gate = table.lookup_entry(src)
    if gate >= lpm_groups:
        return gate, SENTINEL
    flow = extract_flow(bytes(frame[ETH_HDR:]))
    if flow is None:
        return gate, SENTINEL
    return gate, lut[flow_hash(flow) % len(lut)]
