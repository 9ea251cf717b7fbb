"""The drop-in service (VERDICT r3 "do this" 6; one per device since round 5):
a resident workgroup serves every thread's (b1) drop-ins and small host
bursts from its mailbox slot instead of one queue dispatch per call.  Its
lifetime rules are what these tests exercise: the idle exit and the relaunch
by the next call (including a request posted just as the service leaves), a
large host burst dispatched on the same queue while the service runs beside
it, staging buffer growth (the slot's header follows it), slots across thread
churn, and the breakdown stamps.  Every result is
checked against the reference's known answers or the oracle.
"""
import ctypes as C
import random
import threading
import time

import numpy as np
import pytest
import torch

import libunsod_amd as mi
from libunsod_amd import synth
from libunsod_amd._lib import load
from oracle.pyoracle import Oracle


@pytest.fixture(autouse=True)
def _gpu_mode(gpu_dropins):
    """These tests are about the GPU drop-in path (MI_DROPIN_GPU); the host
    fold, the default, is tests/test_dropin_host.py."""
    yield


pytestmark = pytest.mark.gpu
ORC = Oracle("port")

KAT_HDR = bytes.fromhex("450000730000400040110000c0a80001c0a800c7")
KAT_WANT = {0: 0x61B8, 2: 0x61B8, 1: 0xB861, 3: 0xB861}
PAT = bytes(i & 0xFF for i in range(1 << 18))


@pytest.fixture
def lib():
    lib = load()
    lib.mi__set_dropin_service.restype = C.c_int
    lib.mi__set_dropin_service.argtypes = [C.c_int]
    lib.mi__dropin_service_live.restype = C.c_int
    lib.mi__dropin_trace.argtypes = [C.c_int]
    lib.mi__dropin_trace_read.argtypes = [C.POINTER(C.c_double), C.c_int]
    was = lib.mi__set_dropin_service(1)
    yield lib
    lib.mi__set_dropin_service(was)


def _skip_want(n, skip=0):
    return ORC.chain_skip([(PAT[:n], 3)], n - skip, skip)


def test_service_runs_and_answers(lib):
    torch.cuda.init()
    for j in range(200):
        mod = j % 4
        assert mi.in_cksum_hdr(KAT_HDR, addr_mod=mod) == KAT_WANT[mod]
    assert lib.mi__dropin_service_live() == 1
    m = mi.MbufChain([(PAT[:1500], 3)])
    assert mi.in_cksum_skip(m, 1500, 0) == 0x4E39  # KAT7
    assert mi.in_cksum_skip(m, 1480, 20) == _skip_want(1500, 20)


def test_service_inline_and_staged_spans(lib):
    """Spans up to 2048 staging bytes travel inline in the mailbox and are
    folded by wave 0; longer ones stay in the staging buffer: both sides of
    the cut, odd lengths and starts, skips, pseudo headers, odd chains."""
    lib.mi__dropin_mailbox.restype = C.c_int
    rnd = random.Random(11)
    for n in list(range(1, 40)) + [200, 255, 256, 257, 511, 1500, 2000, 2044, 2045, 2047, 2048, 2049, 2100, 4000]:
        k = rnd.randrange(0, 4)
        segs = [(PAT[7:7 + n // 3], 1), (PAT[100:100 + n - n // 3 - k], 3), (PAT[900:900 + k], 2)]
        m = mi.MbufChain(segs)
        for skip in (0, 1, min(3, n)):
            got = mi.in_cksum_skip(m, n - skip, skip)
            assert got == ORC.chain_skip(segs, n - skip, skip), (n, skip)
        got = mi.in_cksum_pseudo_header(m, n, 0, 0x0101A8C0, 0x0201A8C0, 17)
        assert got == ORC.chain_pseudo(segs, n, 0, 0x0101A8C0, 0x0201A8C0, 17), n
    assert lib.mi__dropin_mailbox() in (1, 2)
    print("drop-in service mailbox:", {1: "host memory", 2: "device memory (BAR)"}[lib.mi__dropin_mailbox()])


def test_service_idle_exit_and_relaunch(lib):
    """Calls spaced around the 1 ms idle exit: some find the service gone and
    launch another, some post just as it leaves; all answers right."""
    rnd = random.Random(7)
    for j in range(120):
        mod = j % 4
        assert mi.in_cksum_hdr(KAT_HDR, addr_mod=mod) == KAT_WANT[mod], j
        time.sleep(rnd.choice([0.0, 0.0002, 0.0008, 0.001, 0.0012, 0.003]))
    assert mi.in_cksum_hdr(KAT_HDR, addr_mod=0) == 0x61B8


def test_service_runs_beside_host_burst(lib):
    """A host burst too large for the service (> 64 datagrams) is a dispatch
    on the device's drop-in queue, not the service's (a packet behind a
    running kernel on one queue waits for it): it runs beside the resident
    service and the service stays up.  (The first burst is a warm-up: its
    first-use costs outlast the service's 1 ms idle exit.)"""
    n, L, stride, first = 200, 1500, 2176, 142
    b = synth.build_ipv4_batch(n, L, stride=stride, first_off=first, seed=3)
    buf = mi.page_buffer(b["buf"].size)  # registrable: pages of its own
    buf[:] = b["buf"]
    raw = buf
    ORC.ipv4_finalize_batch(buf, n, stride=stride, first_off=first, fixed_flen=L)
    buf[first + 5 * stride + 99] ^= 0x11
    want = ORC.ipv4_verify_batch(buf, n, stride=stride, first_off=first, fixed_flen=L)
    mi.host_register(raw)
    try:
        mi.ipv4_verify_host(buf, n, stride=stride, first_off=first, fixed_len=L)
        for k in range(6):
            assert mi.in_cksum_hdr(KAT_HDR, addr_mod=k % 4) == KAT_WANT[k % 4]
            assert lib.mi__dropin_service_live() == 1
            ip, l4, st, bad = mi.ipv4_verify_host(buf, n, stride=stride, first_off=first, fixed_len=L)
            assert lib.mi__dropin_service_live() == 1
            assert np.array_equal(st, want[2]) and np.array_equal(l4, want[1])
            assert bad == int((want[2] != 0).sum()) >= 1
    finally:
        mi.host_unregister(raw)


def test_service_staging_growth(lib):
    """A larger chain than the staging buffer holds: the buffer is
    reallocated between calls and the slot's header points the service at the
    new one."""
    sizes = [20, 1500, 65536, 100, 200000, 40, 262144, 64]
    for n in sizes:
        m = mi.MbufChain([(PAT[:n // 2], 1), (PAT[n // 2:n], 2)])
        assert mi.in_cksum_skip(m, n, 0) == ORC.chain_skip([(PAT[:n // 2], 1), (PAT[n // 2:n], 2)], n, 0), n
        assert mi.in_cksum_hdr(KAT_HDR, addr_mod=0) == 0x61B8


def test_service_thread_churn(lib):
    """16 threads at a time, each with a slot of the one service; after they
    exit the library's queue count is back and nothing was leaked."""
    lib.mi_cksum_hsa_queues.restype = C.c_int
    lib.mi__hsa_queues_leaked.restype = C.c_int
    assert mi.in_cksum_hdr(KAT_HDR, addr_mod=0) == 0x61B8
    base = lib.mi_cksum_hsa_queues()
    leaked0 = lib.mi__hsa_queues_leaked()
    for rnd in range(3):
        errors = []

        def work(k):
            try:
                torch.cuda.set_device(0)
                for j in range(40):
                    mod = (k + j) % 4
                    got = mi.in_cksum_hdr(KAT_HDR, addr_mod=mod)
                    if got != KAT_WANT[mod]:
                        errors.append((k, j, hex(got)))
                m = mi.MbufChain([(PAT[:1500], k % 64)])
                if mi.in_cksum_skip(m, 1500, 0) != 0x4E39:
                    errors.append((k, "skip"))
            except Exception as e:  # noqa: BLE001
                errors.append((k, repr(e)))

        ts = [threading.Thread(target=work, args=(k,)) for k in range(16)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=60)
        assert not any(t.is_alive() for t in ts)
        assert not errors, errors[:5]
        # (Python's join returns before the OS thread has run its key destructors)
        deadline = time.monotonic() + 5.0
        while lib.mi_cksum_hsa_queues() != base and time.monotonic() < deadline:
            time.sleep(0.01)
        assert lib.mi_cksum_hsa_queues() == base, (rnd, lib.mi_cksum_hsa_queues(), base)
    assert lib.mi__hsa_queues_leaked() == leaked0


def test_process_exit_with_live_service():
    """A process that exits right after its last drop-in (the service still
    polling its mailbox) stops the service at exit -- the exit handler waits
    for its token -- so nothing faults while the runtime tears the process
    down; this process's GPU work is unaffected afterwards."""
    import os
    import subprocess
    import sys
    code = ("import libunsod_amd as mi, torch; torch.cuda.init()\n"
            "h = bytes.fromhex('450000730000400040110000c0a80001c0a800c7')\n"
            "assert all(mi.in_cksum_hdr(h, addr_mod=0) == 0x61B8 for _ in range(50))\n"
            "print('ok')\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for _ in range(3):
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=root,
                           env=dict(os.environ, MI_CKSUM_DROPIN="gpu"))
        assert r.returncode == 0 and r.stdout.strip() == "ok", (r.returncode, r.stderr[-2000:])
    x = torch.arange(1 << 20, device="cuda", dtype=torch.int64)
    assert int(x.sum().item()) == (1 << 20) * ((1 << 20) - 1) // 2
    torch.cuda.synchronize()


@pytest.mark.parametrize("service", [0, 1])
def test_breakdown_stamps(lib, service):
    """The breakdown's figures are consistent: request posted before the
    result is seen, and the kernel's own time (GPU clock) inside that span."""
    lib.mi__set_dropin_service(service)
    out = (C.c_double * 4)()
    assert lib.mi__dropin_trace(1) == 0
    try:
        rows = []
        for j in range(50):
            assert mi.in_cksum_hdr(KAT_HDR, addr_mod=j % 4) == KAT_WANT[j % 4]
            assert lib.mi__dropin_trace_read(out, 4) == 0
            rows.append(list(out))
    finally:
        lib.mi__dropin_trace(0)
    r = np.median(np.array(rows), axis=0)
    assert 0 <= r[0] <= r[2], r
    assert 0 < r[1] <= r[2] - r[0], r


def test_small_host_bursts_through_the_service(lib, demux_golden):
    """Host-memory bursts of at most 64 datagrams go to the device's service
    (arguments and descriptors in the thread's mailbox slot), larger ones to a dispatch:
    the reference-generated demux golden (TCP / UDP / ICMP / IGMP / CARP,
    options, fragments, bad sums, malformed headers) in bursts of 1-128 must
    give the golden ip / l4 / status and the same RX offload flags as one
    720-datagram launch, with u64 and u32 offsets."""
    g = demux_golden
    buf = mi.page_buffer(g["ver_in"].size)  # registrable: pages of its own
    buf[:] = g["ver_in"]
    offs, flen = g["offs"].astype(np.int64), g["flen"].astype(np.int32)
    n = len(offs)
    mi.host_register(buf)
    try:
        fl_all, cd_all, _ = mi.rx_offload_host(buf, n, offs=offs, lens=flen, demux=True)  # 720 > 128: a launch
        for size in (1, 7, 32, 100, 128):
            for offs32 in (False, True):
                ip = np.zeros(n, np.uint16); l4 = np.zeros(n, np.uint16); st = np.zeros(n, np.uint8)
                fl = np.zeros(n, np.uint32); cd = np.zeros(n, np.uint32)
                for i0 in range(0, n, size):
                    i1 = min(n, i0 + size)
                    ip[i0:i1], l4[i0:i1], st[i0:i1], _ = mi.ipv4_verify_host(
                        buf, i1 - i0, offs=offs[i0:i1], lens=flen[i0:i1], demux=True, offs32=offs32)
                    if i1 - i0 <= 64:
                        assert lib.mi__dropin_service_live() == 1
                    fl[i0:i1], cd[i0:i1], _ = mi.rx_offload_host(buf, i1 - i0, offs=offs[i0:i1], lens=flen[i0:i1],
                                                                demux=True, offs32=offs32)
                assert np.array_equal(st, g["st"]), (size, offs32)
                assert np.array_equal(ip, g["ip"]) and np.array_equal(l4, g["l4"]), (size, offs32)
                assert np.array_equal(fl, fl_all) and np.array_equal(cd, cd_all), (size, offs32)
    finally:
        mi.host_unregister(buf)


def test_service_stands_aside_for_the_batch_path(lib):
    """With a quiet time set, a batch submission stops the running service
    (the safety net for a queue placement other queue creations defeat:
    DESIGN.md 5.6), drop-ins within the quiet time dispatch instead -- still
    right -- and the first drop-in after it brings the service back."""
    torch.cuda.init()
    lib.mi__set_service_quiet_us.restype = C.c_long
    lib.mi__set_service_quiet_us.argtypes = [C.c_long]
    was = lib.mi__set_service_quiet_us(500)  # (off by default: DESIGN.md 5.6)
    try:
        _stand_aside(lib)
    finally:
        lib.mi__set_service_quiet_us(was)


def _stand_aside(lib):
    n, L = 4096, 1500
    buf = torch.zeros(synth.IP_OFF + (n - 1) * synth.STRIDE_1500 + L + 64, dtype=torch.uint8, device="cuda")
    b = mi.PktBatch(buf, n, stride=synth.STRIDE_1500, first_off=synth.IP_OFF, fixed_len=L)
    mi.synth_ipv4(b, seed=5)
    mi.ipv4_finalize(b)
    torch.cuda.synchronize()
    for _ in range(3):
        time.sleep(0.002)  # past the quiet time of the last batch submission
        assert mi.in_cksum_hdr(KAT_HDR, addr_mod=0) == 0x61B8
        assert lib.mi__dropin_service_live() == 1
        mi.ipv4_finalize(b)  # a batch submission
        assert mi.in_cksum_hdr(KAT_HDR, addr_mod=1) == 0xB861  # inside the quiet time: a dispatch
        deadline = time.monotonic() + 2.0
        while lib.mi__dropin_service_live() and time.monotonic() < deadline:
            time.sleep(0.0005)
        assert lib.mi__dropin_service_live() == 0
        torch.cuda.synchronize()
        time.sleep(0.002)
    assert mi.in_cksum_hdr(KAT_HDR, addr_mod=2) == 0x61B8
    assert lib.mi__dropin_service_live() == 1


def test_dropin_queues_avoid_the_batch_queues_pipes():
    """Queue placement: in a fresh process, a prepared batch
    handle's two queues, then a foreign queue (a HIP stream's), then the
    drop-in queues -- which must land in HSA queue-id classes (mod 4) the
    batch queues do not use, spacers taking the rejected ids."""
    import os
    import subprocess
    import sys
    code = r"""
import ctypes as C, json, torch
import libunsod_amd as mi
from libunsod_amd import synth
lib = mi.load()
for f in ("mi__repeat_queue_id", "mi__dropin_queue_id"):
    getattr(lib, f).restype = C.c_longlong
lib.mi__repeat_queue_id.argtypes = [C.c_void_p, C.c_int]
lib.mi__dropin_queue_id.argtypes = [C.c_int]
n, L = 1024, 1500
buf = torch.zeros(synth.IP_OFF + (n - 1) * synth.STRIDE_1500 + L + 64, dtype=torch.uint8, device="cuda")
b = mi.PktBatch(buf, n, stride=synth.STRIDE_1500, first_off=synth.IP_OFF, fixed_len=L)
mi.synth_ipv4(b, seed=1); mi.ipv4_finalize(b); torch.cuda.synchronize()
rep = mi.VerifyRepeat([b], [dict(status=torch.empty(n, dtype=torch.uint8, device="cuda"))], nstreams=2, engine="aql")
rep.run(4)
s = torch.cuda.Stream(); x = torch.ones(16, device="cuda")
with torch.cuda.stream(s): x.add_(1)
torch.cuda.synchronize()
assert mi.in_cksum_hdr(bytes.fromhex("450000730000400040110000c0a80001c0a800c7")) == 0x61B8
print(json.dumps(dict(batch=[lib.mi__repeat_queue_id(rep._h, i) for i in (0, 1)],
                      dropin=[lib.mi__dropin_queue_id(0), lib.mi__dropin_queue_id(1)],
                      spacers=lib.mi__placement_spacers())))
rep.close()
"""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=root,
                       env=dict(os.environ, MI_CKSUM_DROPIN="gpu"))
    assert r.returncode == 0, r.stderr[-2000:]
    import json
    got = json.loads(r.stdout.strip().splitlines()[-1])
    batch = {q % 4 for q in got["batch"]}
    dq, sq = got["dropin"]
    assert min(got["batch"]) >= 0 and dq >= 0 and sq >= 0, got
    assert dq % 4 not in batch and sq % 4 not in batch, got
    print("queue ids:", got)
