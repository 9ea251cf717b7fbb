#!/usr/bin/env python3
"""Does the NUMBER of HSA queues a process holds slow its batch path down?

tools/service_interference.py showed the 1500 B batch rate falling to
0.27-0.51x while 4-16 drop-in threads each kept their own HSA queue.  Here the
batch side (the bench's AQL submission, 2 queues) runs alone while the process
holds N extra queues that are (a) idle -- created, never given a packet -- or
(b) busy with a trivial dispatch loop from one thread each; nothing else
differs.  One JSON line per N.

    python tools/queue_probe.py > queue_probe.jsonl
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import libunsod_amd as mi  # noqa: E402
from libunsod_amd import synth  # noqa: E402

KAT_HDR = bytes.fromhex("450000730000400040110000c0a80001c0a800c7")


class Agent(C.Structure):
    _fields_ = [("handle", C.c_uint64)]


def main():
    hsa = C.CDLL("libhsa-runtime64.so.1")
    assert hsa.hsa_init() == 0
    agents = []
    CB = C.CFUNCTYPE(C.c_int, Agent, C.c_void_p)

    def cb(a, _):
        t = C.c_uint32(0)
        hsa.hsa_agent_get_info(a, 17, C.byref(t))  # HSA_AGENT_INFO_DEVICE
        if t.value == 1:  # HSA_DEVICE_TYPE_GPU
            agents.append(Agent(a.handle))
        return 0

    hsa.hsa_iterate_agents(CB(cb), None)
    gpu = agents[0]
    n, L, stride, first = 65536, 1500, synth.STRIDE_1500, synth.IP_OFF
    bs, outs = [], []
    for r in range(23):
        buf = torch.empty(first + (n - 1) * stride + L + 64, dtype=torch.uint8, device="cuda")
        b = mi.PktBatch(buf, n, stride=stride, first_off=first, fixed_len=L)
        mi.synth_ipv4(b, seed=0x5EED + r)
        mi.ipv4_finalize(b)
        bs.append(b)
        outs.append(dict(status=torch.empty(n, dtype=torch.uint8, device="cuda")))
    torch.cuda.synchronize()
    rep = mi.VerifyRepeat(bs, outs, nstreams=2, engine="aql")
    rep.run(400)

    def rate(seconds=1.5):
        t0, passes = time.perf_counter(), 0
        while time.perf_counter() - t0 < seconds:
            rep.run(200)
            passes += 200
        return round(float(n) * L * passes / (time.perf_counter() - t0) / 2**30, 1)

    base = rate()
    print(json.dumps(dict(extra_queues=0, kind="none", batch_gib_s=base)), flush=True)
    lib = mi.load()
    lib.mi__set_dropin_service.argtypes = [C.c_int]
    lib.mi__set_dropin_service(0)  # drop-in threads: one dispatch per call
    hraw = np.zeros(256, np.uint8)
    off = (-hraw.ctypes.data) % 64
    hraw[off:off + 20] = np.frombuffer(KAT_HDR, np.uint8)
    addr = C.c_void_p(hraw.ctypes.data + off)
    lib.in_cksum_hdr.restype = C.c_uint
    lib.in_cksum_hdr.argtypes = [C.c_void_p]
    for k in (1, 2, 4, 8, 16):
        qs = []
        for _ in range(k):
            q = C.c_void_p()
            st = hsa.hsa_queue_create(gpu, 64, 0, None, None, C.c_uint32(0xFFFFFFFF), C.c_uint32(0xFFFFFFFF),
                                      C.byref(q))
            assert st == 0, st
            qs.append(q)
        idle = rate()
        for q in qs:
            hsa.hsa_queue_destroy(q)
        # k threads with a queue each, calling a drop-in in a loop
        stop = threading.Event()

        def caller():
            while not stop.is_set():
                lib.in_cksum_hdr(addr)

        ts = [threading.Thread(target=caller) for _ in range(k)]
        for t in ts:
            t.start()
        time.sleep(0.3)
        busy = rate()
        stop.set()
        for t in ts:
            t.join()
        print(json.dumps(dict(extra_queues=k, idle_queues_batch_gib_s=idle, idle_vs_none=round(idle / base, 3),
                              dropin_threads_batch_gib_s=busy, busy_vs_none=round(busy / base, 3))), flush=True)
    rep.close()


if __name__ == "__main__":
    main()
