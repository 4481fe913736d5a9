"""CPU tests (no GPU): pin the oracle, check the product's host-side pieces and the C-ABI.

* FNV-1a 64 / XXH64 published vectors (the two hashes of nf.rs:21-31 and flow.rs:105-110).
* The reference's own macswap golden output (test/macswap/data/expect.out, tcpdump -ter of the
  swapped http_lemmy.pcap) against the oracle's MAC swap (headers/mac.rs:140-145).
* Python oracle == C oracle == committed golden vectors (LUTs, flow hashes, backends, swaps, perm).
* The product's host LUT builder (nbg_lut_build_host, what nbg_maglev_create uploads) == golden.
* libnbgpu.so loads and exports every symbol include/nbgpu.h declares; device entry points fail
  loudly (-ENODEV) without a GPU: there is no CPU fallback.
"""
import ctypes as C
import hashlib
import json
import os
import re
import struct

import numpy as np
import pytest
import xxhash

import maglev_ref as ref
import orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
LUT_GOLD = json.load(open(os.path.join(GOLD, "lut_golden.json")))
NAMESETS = {
    "stooges_65537": (["Larry", "Curly", "Moe"], 65537),
    "backend65_65537": ([f"backend-{i}" for i in range(65)], 65537),
    "be1000_655373": ([f"be{i}" for i in range(1000)], 655373),
}


def _digest(arr):
    return hashlib.sha256(np.asarray(arr, dtype="<u2").tobytes()).hexdigest()


# ---- published hash vectors ------------------------------------------------------------
FNV_VECTORS = [(b"", 0xCBF29CE484222325), (b"a", 0xAF63DC4C8601EC8C), (b"foobar", 0x85944171F73967E8)]


@pytest.mark.parametrize("data,h", FNV_VECTORS)
def test_fnv1a64_vectors(data, h):
    assert ref.fnv1a64(data) == h
    buf = (C.c_uint8 * max(len(data), 1)).from_buffer_copy(data or b"\0")
    assert orc.lib().orc_fnv1a64(buf, len(data)) == h


@pytest.mark.parametrize("data", [b"", b"a", b"Larry\xff", b"backend-17\xff", bytes(range(100))])
def test_xxh64_c_oracle_matches_upstream(data):
    buf = (C.c_uint8 * max(len(data), 1)).from_buffer_copy(data or b"\0")
    assert orc.lib().orc_xxh64(buf, len(data), 0) == xxhash.xxh64_intdigest(data, seed=0)
    assert xxhash.xxh64_intdigest(b"", seed=0) == 0xEF46DB3751D8E999


def test_offset_skip_python_vs_c():
    for name in ["Larry", "Curly", "Moe", "backend-0", "be999", "ünïcode"]:
        off, skip = C.c_uint64(), C.c_uint64()
        b = name.encode()
        orc.lib().orc_offset_skip(b, len(b), 65537, C.byref(off), C.byref(skip))
        assert (off.value, skip.value) == ref.offset_skip_for_name(name, 65537)


# ---- the reference's own golden output: macswap expect.out ------------------------------
def _pcap_frames(path):
    data = open(path, "rb").read()
    magic = struct.unpack("<I", data[:4])[0]
    assert magic == 0xA1B2C3D4
    pos, frames = 24, []
    while pos + 16 <= len(data):
        _, _, incl, _ = struct.unpack("<IIII", data[pos:pos + 16])
        frames.append(bytearray(data[pos + 16:pos + 16 + incl]))
        pos += 16 + incl
    return frames


def _mac(b):
    return ":".join(f"{x:02x}" for x in b)


def test_macswap_expect_out():
    """tcpdump -ter prints 'SRC (oui) > DST (oui), ..., length L' for each swapped frame."""
    frames = _pcap_frames(os.path.join(GOLD, "http_lemmy.pcap"))
    lines = open(os.path.join(GOLD, "macswap_expect.out")).read().splitlines()
    assert len(frames) == len(lines) == 15
    lut = ref.generate_lut(["Larry", "Curly", "Moe"], 65537)
    for f, line in zip(frames, lines):
        ref.process_packet(f, lut)
        m = re.match(r"(\S+) \(oui \w+\) > (\S+) \(oui \w+\), ethertype IPv4 \(0x0800\), length (\d+):", line)
        assert m, line
        assert _mac(f[6:12]) == m.group(1)   # new source = old destination
        assert _mac(f[0:6]) == m.group(2)
        assert len(f) == int(m.group(3))


def test_lemmy_golden_python_and_c():
    frames = _pcap_frames(os.path.join(GOLD, "http_lemmy.pcap"))
    gold = json.load(open(os.path.join(GOLD, "lemmy.json")))
    lut3 = orc.lut_build(["Larry", "Curly", "Moe"], 65537)
    for f, g in zip(frames, gold):
        assert orc.flow_hash(bytes(f)) == int(g["flow_hash"], 16)
        buf = np.frombuffer(bytes(f), dtype=np.uint8).copy()
        be = orc.classify(buf, 1, lut3, offs=np.array([0]), lens=np.array([len(f)]))
        assert be[0] == g["backend3"]
        assert buf[:12].tobytes().hex() == g["swapped_head12"]
    # survey §8c prototype: frames 0,2,3,6,8,10,11,14 -> backend 0, the rest -> 1
    assert [g["backend3"] for g in gold] == [0, 1, 0, 0, 1, 1, 0, 1, 0, 1, 0, 0, 1, 1, 0]


# ---- LUTs: Python oracle / C oracle / product host builder vs golden ---------------------
@pytest.mark.parametrize("key", list(NAMESETS))
def test_lut_c_oracle_golden(key):
    names, m = NAMESETS[key]
    g = LUT_GOLD[key]
    lut = orc.lut_build(names, m)
    assert _digest(lut) == g["sha256_u16le"]
    assert lut[:64].tolist() == g["head"]
    counts = np.bincount(lut, minlength=len(names))
    assert (int(counts.min()), int(counts.max())) == (g["counts_min"], g["counts_max"])


@pytest.mark.parametrize("key", ["stooges_65537", "backend65_65537"])
def test_lut_python_oracle_golden(key):
    names, m = NAMESETS[key]
    assert _digest(ref.generate_lut(names, m)) == LUT_GOLD[key]["sha256_u16le"]
    for n, os_ in zip(names, LUT_GOLD[key]["offset_skip_head"]):
        assert list(ref.offset_skip_for_name(n, m)) == os_


@pytest.mark.parametrize("key", list(NAMESETS))
def test_lut_product_host_builder_golden(key):
    import netbricks_amd as nb

    names, m = NAMESETS[key]
    assert _digest(nb.build_lut(names, m)) == LUT_GOLD[key]["sha256_u16le"]


def test_lut_small_tables_match():
    """Small and odd tables through all three builders; a non-coprime permutation that the
    reference would index past its end (nf.rs:52-54 panic) is an error in every builder."""
    import netbricks_amd as nb

    for names, m in [(["a"], 2), (["a", "b"], 7), (["x", "y", "z", "w"], 11), ([f"n{i}" for i in range(20)], 97),
                     (["dup", "dup"], 13)]:
        p = np.array(ref.generate_lut(names, m), dtype=np.uint16)
        assert np.array_equal(orc.lut_build(names, m).astype(np.uint16), p)
        assert np.array_equal(nb.build_lut(names, m), p)
    # M = 10: find a name set whose skip shares a factor with 10 and exhausts a permutation
    bad = None
    for k in range(200):
        names = [f"x{k}", f"y{k}"]
        try:
            ref.generate_lut(names, 10)
        except IndexError:
            bad = names
            break
    assert bad is not None
    with pytest.raises(nb.NbgError):
        nb.build_lut(bad, 10)


# ---- per-packet golden vectors ------------------------------------------------------------
@pytest.fixture(scope="module")
def pk():
    return dict(np.load(os.path.join(GOLD, "packets.npz")))


def test_packets_c_oracle_golden(pk):
    n = pk["off"].size
    lut65 = orc.lut_build(NAMESETS["backend65_65537"][0], 65537)
    lut3 = orc.lut_build(NAMESETS["stooges_65537"][0], 65537)
    buf = pk["buf"].copy()
    be65 = orc.classify(buf, n, lut65, offs=pk["off"], lens=pk["len"])
    np.testing.assert_array_equal(be65, pk["backend65"])
    for i in range(n):
        ln = min(12, int(pk["len"][i]))
        assert buf[pk["off"][i]:pk["off"][i] + ln].tobytes() == pk["mac12"][i, :ln].tobytes()
    be3 = orc.classify(pk["buf"].copy(), n, lut3, offs=pk["off"], lens=pk["len"])
    np.testing.assert_array_equal(be3, pk["backend3"])
    perm, counts = orc.group(be65, 65)
    np.testing.assert_array_equal(perm, pk["perm65"])
    np.testing.assert_array_equal(counts, pk["counts65"])
    for i in range(n):
        f = pk["buf"][pk["off"][i]:pk["off"][i] + pk["len"][i]].tobytes()
        h = orc.flow_hash(f)
        assert (h is not None) == bool(pk["flow_ok"][i])
        if h is not None:
            assert h == int(pk["flow_hash"][i])


def test_packets_python_oracle_subset(pk):
    lut65 = ref.generate_lut(NAMESETS["backend65_65537"][0], 65537)
    idx = list(range(0, 4096, 37)) + list(range(4096, pk["off"].size))
    for i in idx:
        f = bytearray(pk["buf"][pk["off"][i]:pk["off"][i] + pk["len"][i]].tobytes())
        assert ref.process_packet(f, lut65) == pk["backend65"][i]


def test_sentinel_rules():
    """Would-panic packets (packet.rs:392-399 assert, flow.rs:53-62 slice OOB) -> 0xFFFF."""
    lut = [0] * 7
    assert ref.process_packet(bytearray(13), lut) == ref.SENTINEL
    f = bytearray(33)  # payload 19 < 20
    f[14] = 0x45
    assert ref.process_packet(f, lut) == ref.SENTINEL
    f = bytearray(14 + 63)  # IHL 15 -> needs 64 payload bytes
    f[14] = 0x4F
    assert ref.process_packet(f, lut) == ref.SENTINEL
    f = bytearray(14 + 64)
    f[14] = 0x4F
    assert ref.process_packet(f, lut) == 0


# ---- product host-side pieces --------------------------------------------------------------
def test_trace_generator_deterministic_and_wellformed():
    import netbricks_amd as nb

    a = nb.make_trace(2000, 1, seed=99)
    b = nb.make_trace(2000, 1, seed=99)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    buf, off, ln = a
    assert set(np.unique(ln).tolist()) <= {60, 572, 1496}
    assert np.all(off % 64 == 0)
    for i in range(0, 2000, 97):
        f = buf[off[i]:off[i] + ln[i]].tobytes()
        assert f[12:14] == b"\x08\x00" and f[14] == 0x45 and f[23] == 17
        assert struct.unpack("!H", f[16:18])[0] == ln[i] - 14
        s = sum(struct.unpack("!10H", f[14:34]))
        while s >> 16:
            s = (s & 0xFFFF) + (s >> 16)
        assert s == 0xFFFF  # valid IPv4 header checksum
    buf0, off0, ln0 = nb.make_trace(100, 0)
    assert np.all(ln0 == 60) and np.array_equal(off0, np.arange(100) * 64)


@pytest.mark.parametrize("cfg", ["c2", "c3", "c5"])
def test_cpu_baseline_loop_matches_oracle(cfg):
    """The CPU baseline (the reference's producer loop restated: bursts, memo map, rings; for C5
    test/lpm's stage and its group rings first) computes the oracle's backends, on 2 threads, with
    and without the memo map."""
    import netbricks_amd as nb

    n = 3000
    if cfg == "c2":
        names, m, mode = [f"backend-{i}" for i in range(65)], 65537, 0
    elif cfg == "c3":
        names, m, mode = [f"be{i}" for i in range(1000)], 655373, 1
    else:
        names, m, mode = [f"backend-{i}" for i in range(65)], 65537, 1
    lut = orc.lut_build(names, m)
    buf, off, ln = nb.make_trace(n, mode, seed=5)
    kw = dict(stride=64, fixed_len=60) if mode == 0 else dict(offs=off, lens=ln)
    if cfg == "c5":
        routes = json.load(open(os.path.join(GOLD, "lpm_routes.json")))
        rc, t24, tl = orc.lpm_build(routes["reference"] + routes["mixed"])
        assert rc == 0
        _, exp = orc.chain_classify(buf, n, t24, tl, lut, **kw)
        chain = (t24, tl)
    else:
        exp = orc.classify(buf.copy(), n, lut, **kw)
        chain = None
    for cache in (True, False):
        work = buf.copy()
        t, got = orc.cpu_baseline(work, n, lut, len(names), chain=chain, cache=cache, threads=2, **kw)
        assert t > 0
        np.testing.assert_array_equal(got, exp)
        if cfg == "c5":
            np.testing.assert_array_equal(work, buf)  # lpm's and maglev's swaps cancel
    assert (exp != 0xFFFF).any()


def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "nbgpu.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(nbg_[a-z0-9_]+)\s*\(", txt)))


def test_c_abi_exports_every_header_symbol():
    import netbricks_amd._lib as L

    lib = C.CDLL(L.LIB_PATH)
    syms = _header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(L.SIGNATURES), set(syms) ^ set(L.SIGNATURES)


def test_no_cpu_fallback_without_gpu():
    import torch

    import netbricks_amd as nb

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(nb.NbgError) as e:
        nb.Maglev(["a", "b"])
    assert e.value.code == -19
    import ctypes as C

    from netbricks_amd._lib import lib

    n = C.c_uint32(7)
    assert lib.nbg_device_local_cpus(0, None, 0, C.byref(n)) == -19 and n.value == 0


def test_oracle_is_test_infrastructure_only():
    """The product package never imports or links the oracle."""
    for dirpath, _, files in os.walk(os.path.join(ROOT, "netbricks_amd")):
        for f in files:
            if f.endswith((".py", ".hip", ".cpp", ".h", ".hpp", "Makefile")):
                txt = open(os.path.join(dirpath, f), errors="ignore").read()
                assert "maglev_ref" not in txt and "liborc" not in txt and "orc_" not in txt, f


def test_host_operator_selftest():
    """C++ operator mirror pieces that need no GPU: MPSC ring semantics and the pcap port."""
    import subprocess

    exe = os.path.join(ROOT, "netbricks_amd", "host", "nb_host_selftest")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.dirname(exe)], check=True, capture_output=True)
    r = subprocess.run([exe, os.path.join(GOLD, "http_lemmy.pcap"), "/tmp/nb_selftest_out.pcap"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
