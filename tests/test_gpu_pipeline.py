"""GPU: the C++ operator mirror (netbricks_amd/host) running test/maglev end to end on pcaps.

nb_maglev = ReceiveBatch(pcap port) -> parse::<MacHeader> -> transform(swap) -> group_by(ct,
maglev) -> get_group(i) -> merge -> send(pcap port), i.e. test/maglev/src/main.rs:23-42 with the
group_by producer on the MI355X.  Config C1: 65 backends / 65537 slots, 10k-packet UDP pcap.
Checks: every packet transmitted exactly once, bytes == oracle (MAC swapped), the group of
each packet == oracle backend, and per-group FIFO order (group_by.rs:46-51 + MPSC FIFO).
"""
import os
import struct
import subprocess

import numpy as np
import pytest

import orc

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NB = os.path.join(ROOT, "netbricks_amd", "host", "nb_maglev")


def write_pcap(path, frames):
    with open(path, "wb") as f:
        f.write(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 1))
        for i, fr in enumerate(frames):
            f.write(struct.pack("<IIII", i, 0, len(fr), len(fr)))
            f.write(bytes(fr))


def read_pcap(path):
    data = open(path, "rb").read()
    pos, out = 24, []
    while pos + 16 <= len(data):
        incl = struct.unpack("<IIII", data[pos:pos + 16])[2]
        out.append(data[pos + 16:pos + 16 + incl])
        pos += 16 + incl
    return out


def run_pipeline(tmp_path, frames, names, batch=992, zero_copy=False, drop_on_full=False, depth=3, server=-1):
    rx, tx, order = tmp_path / "in.pcap", tmp_path / "out.pcap", tmp_path / "order.txt"
    write_pcap(rx, frames)
    args = [NB, "--rx", str(rx), "--tx", str(tx), "--order", str(order), "--batch", str(batch), "--depth", str(depth),
            "--host-ring", str(server)]
    args += ["--zero-copy", "1" if zero_copy else "0", "--drop-on-full", "1" if drop_on_full else "0"]
    args += ["--names", ",".join(names)]
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return read_pcap(tx), [int(x) for x in open(order).read().split()], r.stdout


def check(frames, names, out, idx):
    n = len(frames)
    assert sorted(idx) == list(range(n))  # every packet exactly once, none dropped
    lut = orc.lut_build(names, 65537)
    offs = np.zeros(n, dtype=np.uint64)
    lens = np.array([len(f) for f in frames], dtype=np.uint16)
    pos = 0
    for i, f in enumerate(frames):
        offs[i] = pos
        pos += len(f) + 64
    buf = np.zeros(pos + 64, dtype=np.uint8)
    for i, f in enumerate(frames):
        buf[offs[i]:offs[i] + len(f)] = np.frombuffer(bytes(f), dtype=np.uint8)
    be = orc.classify(buf, n, lut, offs=offs, lens=lens)
    bad = [(k, i) for k, (o, i) in enumerate(zip(out, idx)) if o != buf[offs[i]:offs[i] + lens[i]].tobytes()]
    assert not bad, (f"{len(bad)} of {n} transmitted frames differ; first (tx position, rx index): {bad[:8]}; "
                     f"tx {out[bad[0][0]][:14].hex()} expected {buf[offs[bad[0][1]]:offs[bad[0][1]] + 14].tobytes().hex()}")
    # per-group FIFO: within each backend the transmit order is the arrival order
    last = {}
    for i in idx:
        g = int(be[i])
        assert last.get(g, -1) < i
        last[g] = i


@pytest.mark.parametrize("zero_copy", [False, True])
def test_lemmy_pcap_through_pipeline(torch_cuda, tmp_path, zero_copy):
    data = open(os.path.join(ROOT, "tests", "golden", "http_lemmy.pcap"), "rb").read()
    pos, frames = 24, []
    while pos + 16 <= len(data):
        incl = struct.unpack("<IIII", data[pos:pos + 16])[2]
        frames.append(data[pos + 16:pos + 16 + incl])
        pos += 16 + incl
    names = ["Larry", "Curly", "Moe"]
    out, idx, stdout = run_pipeline(tmp_path, frames, names, zero_copy=zero_copy)
    check(frames, names, out, idx)
    assert (f'"zero_copy": {"true" if zero_copy else "false"}') in stdout


@pytest.mark.parametrize("batch,zero_copy,depth,server", [(32, False, 3, -1), (4096, False, 4, -1), (4096, True, 4, -1),
                                                        (320, False, 3, -1), (320, True, 2, -1), (992, False, 1, -1),
                                                        (992, False, 4, 32), (992, True, 4, 8), (32, False, 4, 2)])
def test_c1_10k_udp_pcap_65_backends(torch_cuda, tmp_path, batch, zero_copy, depth, server):
    """BASELINE config C1: 65 backends / 65537-slot table, 10k-packet UDP pcap.  The group queues
    keep the reference's 1024 slots; --batch 4096 is capped at 992 packets (whole bursts, <= 1023);
    up to `depth` batches are on the GPU at once, delivered in submit order, and the producer waits
    while a queue could not take every packet in flight plus a whole batch: nothing is dropped."""
    from netbricks_amd import make_trace

    buf, off, ln = make_trace(10000, 0, seed=2024)
    frames = [buf[o:o + l].tobytes() for o, l in zip(off, ln)]
    names = [f"backend-{i}" for i in range(65)]
    out, idx, stdout = run_pipeline(tmp_path, frames, names, batch=batch, zero_copy=zero_copy, depth=depth,
                                    server=server)
    check(frames, names, out, idx)
    assert '"dropped": 0' in stdout
    assert f'"max_batch": {min(batch, 992)}' in stdout
    assert f'"depth": {depth}' in stdout


@pytest.mark.parametrize("zero_copy,drop_on_full,server", [(False, False, -1), (True, False, -1), (False, True, -1),
                                                         (False, False, 32), (True, False, 32)])
def test_loop_pipelines_account_for_every_packet(torch_cuda, tmp_path, zero_copy, drop_on_full, server):
    """nb_maglev --loop (the throughput mode: LoopPort replay ports, one pipeline per thread with its
    own handle and stream; with and without the host-batch server): 3 pipelines x 300k packets of a
    C1-style capture through 992-packet batches, several in flight; every received packet is sent,
    dropped or would-panic, and nothing is dropped with backpressure."""
    import json

    from netbricks_amd import make_trace

    buf, off, ln = make_trace(10000, 0, seed=2026)
    rx = tmp_path / "c1.pcap"
    write_pcap(rx, [buf[o:o + l].tobytes() for o, l in zip(off, ln)])
    args = [NB, "--rx", str(rx), "--backends", "65", "--batch", "992", "--loop", "300000", "--pipelines", "3",
            "--zero-copy", "1" if zero_copy else "0", "--drop-on-full", "1" if drop_on_full else "0",
            "--host-ring", str(server)]
    r = subprocess.run(args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    st = json.loads(r.stdout)
    assert st["rx"] == 900000 and st["tx"] + st["dropped"] + st["would_panic"] == st["rx"]
    assert st["would_panic"] == 0 and len(st["per_pipeline_mpps"]) == 3 and st["aggregate_mpps"] > 0
    if not drop_on_full:
        assert st["dropped"] == 0 and st["tx"] == 900000
    # one mempool of 10,000 mbufs per port (the capture, once), threads on CPUs the process may use
    assert st["pool_mbufs"] == 10000
    cpus = [int(c) for c in st["cpus"].split(",")]
    assert len(cpus) == 3 and set(cpus) <= os.sched_getaffinity(0)


def test_device_local_cpus(torch_cuda):
    """nbg_device_local_cpus: the CPUs of the GPU's socket from sysfs (nb_maglev pins its pipelines to
    them): a non-empty list of distinct CPUs of this machine; a short buffer still reports the count."""
    import ctypes as C

    from netbricks_amd._lib import lib

    from netbricks_amd._lib import NBG_EIO

    buf = (C.c_int32 * 4096)()
    n = C.c_uint32()
    rc = lib.nbg_device_local_cpus(0, buf, 4096, C.byref(n))
    if rc == NBG_EIO:  # the documented answer where sysfs has no local_cpulist for the device
        pytest.skip("no local_cpulist for the GPU's PCI function on this host")
    assert rc == 0
    cpus = list(buf[:n.value])
    assert 0 < n.value <= os.cpu_count() and len(set(cpus)) == n.value
    assert all(0 <= c < os.cpu_count() for c in cpus)
    m = C.c_uint32()
    assert lib.nbg_device_local_cpus(0, buf, 1, C.byref(m)) == 0 and m.value == n.value and buf[0] == cpus[0]
    assert lib.nbg_device_local_cpus(99, buf, 4096, C.byref(m)) != 0


def test_c1_drop_on_full_keeps_reference_semantics(torch_cuda, tmp_path):
    """--drop-on-full: the producer pulls a batch every round, as the reference's does, and a full
    1024-slot queue loses the packet (group_by.rs:50, mpsc_mbuf_queue.rs:91-115).  With 3 groups and
    the consumer draining one 32-packet burst per round, 10k packets overflow: what is sent is a
    subset, each frame at most once, still in per-group FIFO order, and sent + dropped = received."""
    import json

    from netbricks_amd import make_trace

    buf, off, ln = make_trace(10000, 0, seed=2025)
    frames = [buf[o:o + l].tobytes() for o, l in zip(off, ln)]
    names = ["Larry", "Curly", "Moe"]
    out, idx, stdout = run_pipeline(tmp_path, frames, names, batch=992, drop_on_full=True)
    st = json.loads(stdout)
    assert st["dropped"] > 0 and st["tx"] + st["dropped"] + st["would_panic"] == st["rx"] == 10000
    assert len(set(idx)) == len(idx) == st["tx"]
    lut = orc.lut_build(names, 65537)
    be = orc.classify(buf.copy(), 10000, lut, offs=off.astype(np.uint64), lens=ln)
    last = {}
    for i in idx:
        g = int(be[i])
        assert last.get(g, -1) < i
        last[g] = i
