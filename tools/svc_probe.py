#!/usr/bin/env python3
"""Does a dispatch wait behind the resident drop-in service on the same HSA
queue?  (It did, round 5: a 200-datagram host burst dispatched into the
service's queue took the service's 1 ms idle exit, with no barrier bit set;
the service now has a queue of its own.)  Per mode (service on / off / on):
the service's liveness before and after a 200 x 1500 B zero-copy host burst
(> 64 datagrams: a dispatch), and the burst's wall time.  One JSON line each.

    python tools/svc_probe.py
"""
import ctypes as C, json, time, sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np, torch
import libunsod_amd as mi
from libunsod_amd import synth
from libunsod_amd._lib import load
lib = load()
lib.mi__dropin_service_live.restype = C.c_int
lib.mi__set_dropin_service.argtypes = [C.c_int]
KAT_HDR = bytes.fromhex("450000730000400040110000c0a80001c0a800c7")
n, L, stride, first = 200, 1500, 2176, 142
b = synth.build_ipv4_batch(n, L, stride=stride, first_off=first, seed=3)
raw = np.zeros(b["buf"].size + 4096, np.uint8)
s = (-raw.ctypes.data) % 4096
buf = raw[s:s + b["buf"].size]
buf[:] = b["buf"]
mi.host_register(raw)
torch.cuda.init()
for svc in (1, 0, 1):
    lib.mi__set_dropin_service(svc)
    for k in range(4):
        mi.in_cksum_hdr(KAT_HDR)
        l0 = lib.mi__dropin_service_live()
        t0 = time.perf_counter()
        mi.ipv4_verify_host(buf, n, stride=stride, first_off=first, fixed_len=L)
        dt = time.perf_counter() - t0
        l1 = lib.mi__dropin_service_live()
        print(json.dumps(dict(svc=svc, k=k, live_before=l0, live_after=l1, burst_us=round(dt * 1e6, 1))), flush=True)
mi.host_unregister(raw)
