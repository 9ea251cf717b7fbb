"""Per-thread resources across thread churn ("do this" 8).

The (b1) drop-ins and the host-burst path run on whatever thread calls them
-- the dpdk_rx kthread, application threads in ud_send, the callout thread
(SURVEY.md 8(b1) "Threading").  Each calling thread gets its own completion
signal, kernel-argument slots, mailbox slot, staging and streams (the HSA
queue is the device's one drop-in queue, shared); a pthread-key destructor
gives them back when the thread exits.  This test creates and joins 64
threads at a time, several rounds, each thread making drop-in calls (every
eighth a zero-copy host burst through the service or the drop-in queue, every
eighth a staged one through its own HIP streams), checks every result against the
reference's known answers / the oracle, and checks that the library's HSA
queue count is back where it started after every round.  The kernel driver's
per-process queue list (where readable) must stay flat from the second round
on: HIP keeps a small pool of hardware queues for its streams."""
import os
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

# the IPv4 header, in_cksum_hdr at 4-aligned / 2 mod 4 / odd
KAT_HDR = bytes.fromhex("450000730000400040110000c0a80001c0a800c7")
KAT_WANT = {0: 0x61B8, 2: 0x61B8, 1: 0xB861, 3: 0xB861}


def kfd_queues():
    """Queues the kernel driver lists for this process (None if not readable)."""
    try:
        return len(os.listdir(f"/sys/class/kfd/kfd/proc/{os.getpid()}/queues"))
    except OSError:
        return None


def _burst(seed):
    n, L, stride, first = 64, 1500, 2176, 142
    b = synth.build_ipv4_batch(n, L, stride=stride, first_off=first, seed=seed)
    buf = mi.page_buffer(b["buf"].size)  # registrable: pages of its own
    buf[:] = b["buf"]
    raw = buf
    ORC.ipv4_finalize_batch(buf, n, stride=stride, first_off=first, fixed_flen=L)
    return raw, buf, n, stride, first, L


def test_thread_churn_keeps_queue_count_flat():
    torch.cuda.init()
    lib = load()
    # warm the main thread (the device's drop-in queue stays for the process's life)
    assert mi.in_cksum_hdr(KAT_HDR, addr_mod=0) == 0x61B8
    base = lib.mi_cksum_hsa_queues()
    kfd = []
    for rnd in range(3):
        errors = []

        def work(k):
            try:
                torch.cuda.set_device(0)
                for j in range(6):
                    mod = (k + j) % 4
                    got = mi.in_cksum_hdr(KAT_HDR, addr_mod=mod)
                    if got != KAT_WANT[mod]:
                        errors.append((k, j, mod, hex(got)))
                m = mi.MbufChain([(bytes(i & 0xFF for i in range(1500)), k % 64)])
                if mi.in_cksum_skip(m, 1500, 0) != 0x4E39:  # KAT7, 1500 B
                    errors.append((k, "skip"))
                if k % 4 == 0:
                    raw, buf, n, stride, first, L = _burst(k)
                    zero_copy = k % 8 == 0
                    if zero_copy:
                        mi.host_register(raw)
                    try:
                        ip, l4, st, bad = mi.ipv4_verify_host(buf, n, stride=stride, first_off=first,
                                                              fixed_len=L, staged=not zero_copy)
                    finally:
                        if zero_copy:
                            mi.host_unregister(raw)
                    if bad or st.any() or ip.any() or l4.any():
                        errors.append((k, "burst", zero_copy, bad))
            except Exception as e:  # noqa: BLE001 -- reported below
                errors.append((k, repr(e)))

        ts = [threading.Thread(target=work, args=(k,)) for k in range(64)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=120)
        assert not any(t.is_alive() for t in ts), "a worker thread hung"
        assert not errors, errors[:5]
        # Thread.join returns when the Python side of a thread is done; the
        # OS thread runs its pthread-key destructors just after -- poll briefly
        deadline = time.monotonic() + 5.0
        while lib.mi_cksum_hsa_queues() != base and time.monotonic() < deadline:
            time.sleep(0.01)
        assert lib.mi_cksum_hsa_queues() == base, (rnd, lib.mi_cksum_hsa_queues(), base)
        kfd.append(kfd_queues())
    print("library queues", base, "kfd queues per round", kfd)
    if kfd[0] is not None:
        assert kfd[2] <= kfd[1] <= kfd[0] + 8, kfd
