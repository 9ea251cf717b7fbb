"""Round 5: what keeps a wrong index from faulting the GPU, on the GPU.

Every array a kernel reads or writes is reached through a buffer resource
carrying its extent (cksum_device.h `Arr`; tests/test_isa_audit.py checks the
code object on the CPU).  Here: an index past an array's extent reads zeros
instead of faulting (a chain batch whose segment tables are declared shorter
than the chains reference: the walk sees zero-length mbufs, exactly the
reference's silent truncation, in_cksum.c:214-229); outputs are never written
past their n elements, whichever kernel and submission path wrote them; the
GPU memory-fault reporter is registered; the AQL engine leaks rather than
frees under passes whose wait failed; a drop-in tag wraps past 0; the
drop-in service slots are capped; and the MI_DEBUG_BOUNDS build names an
out-of-range access.
"""
import ctypes as C
import os
import subprocess
import sys
import threading
import time

import numpy as np
import pytest
import torch

import libunsod_amd as mi
from libunsod_amd import synth
from libunsod_amd._lib import ChainBatchC, LIB_DIR, MI_CHAIN_SKIP, check, load
from oracle.pyoracle import Oracle


@pytest.fixture(autouse=True)
def _gpu_mode(gpu_dropins):
    """These tests are about the GPU drop-in path (MI_DROPIN_GPU); the host
    fold, the default, is tests/test_dropin_host.py."""
    yield


pytestmark = pytest.mark.gpu
ORC = Oracle("port")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KAT_HDR = bytes.fromhex("450000730000400040110000c0a80001c0a800c7")


def _lib():
    lib = load()
    lib.mi__fault_reporter.restype = C.c_int
    lib.mi__hsa_queues_leaked.restype = C.c_int
    lib.mi__journal_events.restype = C.c_ulonglong
    lib.mi__set_dropin_tag.argtypes = [C.c_uint32]
    lib.mi__dropin_service_owners.restype = C.c_int
    lib.mi__set_dropin_service.restype = C.c_int
    lib.mi__set_dropin_service.argtypes = [C.c_int]
    return lib


def _chains(seed=5, n=300):
    rng = np.random.default_rng(seed)
    chains = []
    for i in range(n):
        k = int(rng.integers(1, 6))
        chains.append([(rng.integers(0, 256, int(rng.integers(0, 700)), dtype=np.uint8).tobytes(),
                        int(rng.integers(0, 4))) for _ in range(k)])
    return chains


def _chain_call(cb, length, skip, nseg):
    out = torch.empty(cb.n, dtype=torch.uint16, device="cuda")
    ln = torch.as_tensor(length, dtype=torch.int32, device="cuda")
    sk = torch.as_tensor(skip, dtype=torch.int32, device="cuda")
    c = ChainBatchC(cb.buf.data_ptr(), cb.buf.numel(), cb.seg_off.data_ptr(), cb.seg_len.data_ptr(),
                    cb.pkt_seg.data_ptr(), cb.n, MI_CHAIN_SKIP, ln.data_ptr(), sk.data_ptr(), None, None, None,
                    cb.max_seg, nseg)
    check("mi_cksum_chain_batch", load().mi_cksum_chain_batch(C.byref(c), out.data_ptr(), None))
    torch.cuda.synchronize()
    return out.cpu().numpy().astype(np.int64)


def test_fault_reporter_registered():
    lib = _lib()
    assert mi.in_cksum_hdr(KAT_HDR) == 0x61B8
    state = lib.mi__fault_reporter()
    print("GPU memory-fault reporter:", {1: "registered", -1: "refused by the HSA runtime"}.get(state, state))
    assert state == 1
    assert lib.mi__journal_events() > 0


def test_segment_table_extent_bounds_the_walk():
    """nseg declared at half the segments the chains reference: every index at
    or past it reads (m_data 0, m_len 0) -- skipped, the chain truncated --
    instead of reaching memory past the tables."""
    chains = _chains()
    cb = mi.ChainBatch(chains)
    total = cb.seg_len.numel()
    length = [sum(len(s) for s, _ in ch) for ch in chains]
    skip = [min(3, ln) for ln in length]
    full = _chain_call(cb, length, skip, total)
    want_full = np.array([ORC.chain_skip(ch, ln, sk) for ch, ln, sk in zip(chains, length, skip)], np.int64)
    assert np.array_equal(full, want_full)
    cut = total // 2
    got = _chain_call(cb, length, skip, cut)
    want, k = [], 0
    for ch, ln, sk in zip(chains, length, skip):
        kept = [(s if k + j < cut else b"", m) for j, (s, m) in enumerate(ch)]
        k += len(ch)
        want.append(ORC.chain_skip(kept, ln, sk))
    assert np.array_equal(got, np.array(want, np.int64))
    assert not np.array_equal(got, full)


def test_huge_segment_index_reads_nothing():
    """a segment index of 2^30 used to wrap the 32-bit byte offsets
    of both tables (4 * i, 8 * i) to 0 and read segment 0's m_len / m_data --
    a plausible wrong checksum.  Offsets now clamp to the out-of-range value
    and read (m_data 0, m_len 0): the last chain, pointed at segments 2^30 and
    2^30 + 1, is an empty chain (in_cksum_skip of nothing: 0xffff) and every
    other chain is unchanged."""
    chains = _chains(seed=9, n=64)
    cb = mi.ChainBatch(chains)
    length = [sum(len(s) for s, _ in ch) for ch in chains]
    skip = [0] * len(chains)
    want = np.array([ORC.chain_skip(ch, ln, 0) for ch, ln in zip(chains, length)], np.int64)
    n = cb.n
    cb.pkt_seg[n - 1] = 1 << 30
    cb.pkt_seg[n] = (1 << 30) + 2
    got = _chain_call(cb, length, skip, 1 << 30)
    assert np.array_equal(got[:n - 1], want[:n - 1])
    assert got[n - 1] == 0xFFFF


@pytest.mark.parametrize("kind", ["1500", "64", "pareto", "pareto-dma"])
def test_outputs_never_written_past_n(kind):
    """Outputs sit at the front of larger poisoned tensors: nothing past n
    changes, through the direct call and the AQL engine."""
    if kind.startswith("pareto"):
        n = 3000
        lens = synth.pareto_lengths(n, seed=4)
        offs = synth.packed_offsets(lens, first_off=2)
        buf = torch.zeros(int(offs[-1] + lens[-1]) + 256, dtype=torch.uint8, device="cuda")
        b = mi.PktBatch(buf, n, offs=torch.from_numpy(offs.astype(np.int64)).cuda(),
                        lens=torch.from_numpy(lens.astype(np.int32)).cuda(), packed=True)
    else:
        n, L, stride, first = {"1500": (1000, 1500, synth.STRIDE_1500, synth.IP_OFF),
                               "64": (5000, synth.MIN_FRAME_IP_LEN, synth.STRIDE_64, synth.ETH_HLEN)}[kind]
        buf = torch.zeros(first + (n - 1) * stride + L + 64, dtype=torch.uint8, device="cuda")
        b = mi.PktBatch(buf, n, stride=stride, first_off=first, fixed_len=L)
    mi.synth_ipv4(b, seed=3)
    mi.ipv4_finalize(b)
    if kind == "pareto-dma":
        mi.set_run_kernel(4, 3)
    try:
        for engine in ("direct", "aql"):
            pad = 4096
            out = dict(ip=torch.full((n + pad,), 0xABAB, dtype=torch.int32, device="cuda").to(torch.uint16),
                       l4=torch.full((n + pad,), 0xCDCD, dtype=torch.int32, device="cuda").to(torch.uint16),
                       status=torch.full((n + pad,), 0xEE, dtype=torch.uint8, device="cuda"))
            views = {k: v[:n] for k, v in out.items()}
            if engine == "direct":
                mi.ipv4_verify(b, out=views)
            else:
                rep = mi.VerifyRepeat([b], [views], nstreams=1, engine="aql")
                try:
                    rep.run(3)
                finally:
                    rep.close()
            torch.cuda.synchronize()
            assert (out["status"][:n] == 0).all().item(), (kind, engine)
            assert (out["ip"][n:].to(torch.int32) == 0xABAB).all().item(), (kind, engine)
            assert (out["l4"][n:].to(torch.int32) == 0xCDCD).all().item(), (kind, engine)
            assert (out["status"][n:] == 0xEE).all().item(), (kind, engine)
    finally:
        mi.set_run_kernel(0, 0)


def test_repeat_destroy_leaks_when_the_wait_fails():
    """repeat_free after a failed AQL wait keeps the run's queues, signals and
    kernel arguments (the passes may still be reading them) and counts the
    queues as leaked."""
    lib = _lib()
    n, L, stride, first = 2048, 1500, synth.STRIDE_1500, synth.IP_OFF
    buf = torch.zeros(first + (n - 1) * stride + L + 64, dtype=torch.uint8, device="cuda")
    b = mi.PktBatch(buf, n, stride=stride, first_off=first, fixed_len=L)
    mi.synth_ipv4(b, seed=9)
    mi.ipv4_finalize(b)
    st = torch.empty(n, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    live0, leaked0 = lib.mi_cksum_hsa_queues(), lib.mi__hsa_queues_leaked()
    rep = mi.VerifyRepeat([b], [dict(status=st)], nstreams=2, engine="aql")
    assert lib.mi_cksum_hsa_queues() == live0 + 2
    rep.run(8, wait=False)
    lib.mi__aql_fail_next_wait()
    rep.close()
    assert lib.mi__hsa_queues_leaked() == leaked0 + 2
    assert lib.mi_cksum_hsa_queues() == live0
    time.sleep(0.2)  # the passes finish on their own; the tensors outlive them
    assert (st == 0).all().item()


def test_dropin_tag_wraps_past_zero():
    """A thread whose first service call would carry tag 0 (the tag after
    0xffff) on a fresh mailbox: the tag skips 0, the call answers at once."""
    lib = _lib()
    res = {}

    def work():
        was = lib.mi__set_dropin_service(0)
        try:
            assert mi.in_cksum_hdr(KAT_HDR) == 0x61B8  # dispatch mode: the thread's context, no mailbox
            lib.mi__set_dropin_tag(0xFFFF)
            lib.mi__set_dropin_service(1)
            t0 = time.time()
            res["v"] = [mi.in_cksum_hdr(KAT_HDR, addr_mod=k % 4) for k in range(4)]
            res["dt"] = time.time() - t0
        finally:
            lib.mi__set_dropin_service(was)

    t = threading.Thread(target=work)
    t.start()
    t.join(30)
    assert res["v"] == [0x61B8, 0xB861, 0x61B8, 0xB861]
    assert res["dt"] < 2.0, res["dt"]


def test_dropin_threads_share_one_service():
    """16 threads calling drop-ins at once: each holds a mailbox slot of the
    device's ONE service (no queue per thread: the process's queue count does
    not move), every answer right, and the slots come back when the threads
    exit."""
    lib = _lib()
    was = lib.mi__set_dropin_service(1)
    assert mi.in_cksum_hdr(KAT_HDR) == 0x61B8  # the main thread's slot, the device's queue
    q0 = lib.mi_cksum_hsa_queues()
    bar = threading.Barrier(16)
    peak, queues, bad = [], [], []

    def work(k):
        for j in range(50):
            v = mi.in_cksum_hdr(KAT_HDR, addr_mod=(k + j) % 4)
            if v != (0x61B8 if (k + j) % 2 == 0 else 0xB861):
                bad.append((k, j, v))
            if j == 10:
                bar.wait(30)
                peak.append(lib.mi__dropin_service_owners())
                queues.append(lib.mi_cksum_hsa_queues())
                bar.wait(30)

    try:
        ts = [threading.Thread(target=work, args=(k,)) for k in range(16)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(60)
    finally:
        lib.mi__set_dropin_service(was)
    assert not bad, bad[:5]
    assert max(peak) == 17, peak
    assert set(queues) == {q0}, (queues, q0)
    deadline = time.monotonic() + 5.0
    while lib.mi__dropin_service_owners() != 1 and time.monotonic() < deadline:
        time.sleep(0.01)
    assert lib.mi__dropin_service_owners() == 1  # the main thread's


def test_reused_slot_with_the_same_first_word():
    """A slot's next owner whose first request would carry exactly the word
    the previous owner's last one did (same tag, same inline size): the word
    is changed, the service sees it, the call answers at once."""
    lib = _lib()
    was = lib.mi__set_dropin_service(1)
    res = []

    def work():
        lib.mi__set_dropin_tag(0x1233)
        t0 = time.time()
        res.append((mi.in_cksum_hdr(KAT_HDR, addr_mod=0), time.time() - t0))

    try:
        for _ in range(3):
            t = threading.Thread(target=work)
            t.start()
            t.join(30)
            time.sleep(0.05)  # (the thread's key destructor gives its slot back)
    finally:
        lib.mi__set_dropin_service(was)
    assert [v for v, _ in res] == [0x61B8] * 3
    assert max(dt for _, dt in res) < 2.0, res


DEBUG_LIB = os.path.join(LIB_DIR, "debug", "libmicksum.so")
DEBUG_PROG = r"""
import ctypes as C, sys
sys.path.insert(0, sys.argv[1])
import numpy as np, torch
import libunsod_amd as mi
from libunsod_amd._lib import ChainBatchC, MI_CHAIN_SKIP, check, load
chains = [[(bytes(range(200)), 0), (bytes(300), 1), (bytes(50), 2)] for _ in range(64)]
cb = mi.ChainBatch(chains)
ln = torch.full((64,), 550, dtype=torch.int32, device="cuda")
sk = torch.zeros(64, dtype=torch.int32, device="cuda")
out = torch.empty(64, dtype=torch.uint16, device="cuda")
c = ChainBatchC(cb.buf.data_ptr(), cb.buf.numel(), cb.seg_off.data_ptr(), cb.seg_len.data_ptr(),
                cb.pkt_seg.data_ptr(), 64, MI_CHAIN_SKIP, ln.data_ptr(), sk.data_ptr(), None, None, None,
                cb.max_seg, 100)
check("chain", load().mi_cksum_chain_batch(C.byref(c), out.data_ptr(), None))
torch.cuda.synchronize()
print("done", int(out[0].item()))
"""


@pytest.mark.skipif(not os.path.exists(DEBUG_LIB), reason="the MI_DEBUG_BOUNDS build (make -C libunsod_amd/csrc debug)")
def test_debug_build_names_the_out_of_range_access():
    env = dict(os.environ, MI_CKSUM_LIB=DEBUG_LIB)
    p = subprocess.run([sys.executable, "-c", DEBUG_PROG, ROOT], env=env, capture_output=True, text=True, timeout=100)
    print(p.stdout[-2000:], p.stderr[-2000:])
    assert p.returncode == 0
    assert "done" in p.stdout
    assert "libmicksum: out-of-range access in" in p.stdout + p.stderr
