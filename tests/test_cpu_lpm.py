"""CPU tests (no GPU) of the chained test/lpm stage (BASELINE config C5).

* Python oracle (golden generator) == C oracle == the product's host DIR-24-8 builder
  (nbg_lpm_build_host, what nbg_lpm_create uploads), by table digest, on the reference's own
  105 routes (test/lpm/src/nf.rs:106-210) and on a mixed route set of every length 8..32.
* lookup_entry vectors (test/lpm/src/nf.rs:88-98) and lpm() -> maglev() per-packet vectors.
* The reference's panics (fills past a table's end, length > 32) are errors in every builder.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import maglev_ref as ref
import orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
ROUTES = json.load(open(os.path.join(GOLD, "lpm_routes.json")))
LPM_GOLD = json.load(open(os.path.join(GOLD, "lpm_golden.json")))


def _digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).astype("<u2").tobytes()).hexdigest()


@pytest.mark.parametrize("key", ["reference", "mixed"])
def test_lpm_c_oracle_tables_and_lookups(key):
    rc, t24, tl = orc.lpm_build(ROUTES[key])
    g = LPM_GOLD[key]
    assert rc == 0
    assert tl.size == g["long_used"]
    assert _digest(t24) == g["tbl24_sha256"]
    assert _digest(tl) == g["tbl_long_sha256"]
    assert np.array_equal(orc.lpm_lookup(t24, tl, g["ips"]), np.array(g["gates"], dtype=np.uint16))


@pytest.mark.parametrize("key", ["reference", "mixed"])
def test_lpm_product_host_builder_golden(key):
    import netbricks_amd as nb

    t24, tl = nb.build_lpm(ROUTES[key])
    g = LPM_GOLD[key]
    assert tl.size == g["long_used"]
    assert _digest(t24) == g["tbl24_sha256"]
    assert _digest(tl) == g["tbl_long_sha256"]


def test_reference_routes_all_gate_one():
    """Every address test/lpm installs maps to gate 1; its /24 neighbours fall back to 0."""
    rc, t24, tl = orc.lpm_build(ROUTES["reference"])
    assert rc == 0
    ips = []
    for ip, plen, gate in ROUTES["reference"]:
        assert plen == 32 and gate == 1
        a = [int(x) for x in ip.split(".")]
        ips.append((a[0] << 24) | (a[1] << 16) | (a[2] << 8) | a[3])
    ips = np.array(ips, dtype=np.uint32)
    assert (orc.lpm_lookup(t24, tl, ips) == 1).all()
    others = np.setdiff1d(ips ^ np.uint32(1), ips)
    assert (orc.lpm_lookup(t24, tl, others) == 0).all()


def test_lpm_small_tables_python_c_product():
    """Hand-built tables: nesting, duplicates (last insert wins), overflow blocks, /0, /32."""
    import netbricks_amd as nb

    cases = [
        [],
        [("0.0.0.0", 0, 2)],
        [("10.0.0.0", 8, 1), ("10.1.0.0", 16, 2), ("10.1.2.0", 24, 1), ("10.1.2.128", 25, 2), ("10.1.2.3", 32, 0)],
        [("10.0.0.0", 8, 1), ("10.0.0.0", 8, 2)],                 # duplicate: last wins
        [("192.168.1.7", 32, 1), ("192.168.1.9", 32, 2), ("192.168.1.0", 30, 2)],  # shared /24 block
        [("1.2.3.4", 32, 0x8001)],                                 # gate with the overflow bit set
    ]
    rng = np.random.default_rng(7)
    for routes in cases:
        rc, t24, tl = orc.lpm_build(routes)
        assert rc == 0
        p24, ptl = nb.build_lpm(routes)
        assert np.array_equal(p24, t24) and np.array_equal(ptl, tl)
        py = ref.IPLookup()
        for ip, plen, gate in routes:
            a = [int(x) for x in ip.split(".")]
            py.insert((a[0] << 24) | (a[1] << 16) | (a[2] << 8) | a[3], plen, gate)
        py.construct_table()
        assert np.array_equal(py.tbl24, t24)
        assert np.array_equal(py.tbl_long[:py.current_tbl_long], tl)
        ips = rng.integers(0, 1 << 32, 500, dtype=np.uint64).astype(np.uint32)
        ips = np.concatenate([ips, np.array([0x0A010203, 0x0A010280, 0x0A0102FF, 0xC0A80107, 0xC0A80109,
                                             0xC0A80100, 0x01020304], dtype=np.uint32)])
        assert np.array_equal(orc.lpm_lookup(t24, tl, ips),
                              np.array([py.lookup_entry(int(x)) for x in ips], dtype=np.uint16))


@pytest.mark.parametrize("routes", [
    [("10.0.0.0", 33, 1)],          # raw_entries[33]: index out of bounds
    [("1.0.0.0", 0, 1)],            # /0 with a non-zero key: tbl24[(k >> 8) ..] past the end
])
def test_lpm_reference_panics_are_errors(routes):
    import netbricks_amd as nb

    rc, _, _ = orc.lpm_build(routes)
    assert rc == -34
    with pytest.raises(nb.NbgError) as e:
        nb.build_lpm(routes)
    assert e.value.code == -22


def test_chain_c_oracle_golden():
    g = np.load(os.path.join(GOLD, "lpm_chain.npz"))
    rc, t24, tl = orc.lpm_build(ROUTES["mixed"])
    assert rc == 0
    lut = orc.lut_build([f"backend-{i}" for i in range(65)], 65537)
    buf = g["buf"].copy()
    n = g["off"].size
    gate, be = orc.chain_classify(buf, n, t24, tl, lut, offs=g["off"], lens=g["len"])
    assert np.array_equal(gate, g["gate"])
    assert np.array_equal(be, g["backend"])
    assert np.array_equal(buf, g["buf"]), "the chain must not modify packet bytes (the two swaps cancel)"
    perm, counts = orc.group(be, 65)
    assert np.array_equal(perm, g["perm"]) and np.array_equal(counts, g["counts"])
    # every path is exercised: all three gates, gate >= 3 rejections, unparseable frames
    assert set(np.unique(gate).tolist()) >= {0, 1, 2, 3, 0xFFFF}
