#!/usr/bin/env python3
"""Where the ~8 us of a (b1) drop-in call goes (VERDICT r3 "do this" 6).

With mi__dropin_trace(1) the drop-in kernel stores its start and end on the
GPU's 100 MHz clock next to the result (the drop-in service: the moment it saw
the request, and its result store); every call then records, on the host's
clock from the fold's entry, the doorbell rung (the service: the request
posted) and the moment the host sees the result word, and the kernel's own
time from the GPU clock's difference.  Median over N calls of each (b1) function on real
mbuf chains, next to the untraced per-call time, for one dispatch per call and
for the resident drop-in service.

    python tools/dropin_breakdown.py [--calls 400] > dropin_breakdown.jsonl
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (one HIP runtime per process: torch's)

import libunsod_amd as mi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=400)
    a = ap.parse_args()
    lib = mi.load()
    lib.mi__dropin_trace.argtypes = [C.c_int]
    lib.mi__dropin_trace_read.argtypes = [C.POINTER(C.c_double), C.c_int]
    lib.mi__dropin_mailbox.restype = C.c_int
    lib.mi__set_dropin_service.restype = C.c_int
    lib.mi__set_dropin_service.argtypes = [C.c_int]
    pat = bytes(i & 0xFF for i in range(65536))
    m64 = mi.MbufChain([pat])
    ip_hdr = bytes.fromhex("450005dc0000400040060000c0a80101c0a80102")
    m1500 = mi.MbufChain([ip_hdr + pat[:1480]])
    hraw = np.zeros(256, np.uint8)
    hoff = 64 + ((2 - (hraw.ctypes.data + 64)) % 64)
    hraw[hoff:hoff + 20] = np.frombuffer(ip_hdr, np.uint8)
    haddr = hraw.ctypes.data + hoff
    src, dst = 0x0101A8C0, 0x0201A8C0
    cases = {
        "in_cksum_hdr_20B": (lib.in_cksum_hdr, (C.c_void_p(haddr),)),
        "in_cksum_pseudo_header_1480B": (lib.in_cksum_pseudo_header, (C.c_void_p(m1500.ptr), 1480, 20, src, dst, 6)),
        "in_cksum_skip_65536B": (lib.in_cksum_skip, (C.c_void_p(m64.ptr), 65536, 0)),
    }
    out = (C.c_double * 4)()
    for (name, (fn, args)), mode in [(c, m) for m in ("dispatch", "service") for c in cases.items()]:
        lib.mi__set_dropin_service(1 if mode == "service" else 0)
        fn(*args)
        plain = []
        for _ in range(a.calls):
            t0 = time.perf_counter()
            fn(*args)
            plain.append(time.perf_counter() - t0)
        assert lib.mi__dropin_trace(1) == 0
        fn(*args)
        rows, tot = [], []
        for _ in range(a.calls):
            t0 = time.perf_counter()
            fn(*args)
            tot.append(time.perf_counter() - t0)
            lib.mi__dropin_trace_read(out, 4)
            rows.append(list(out))
        assert lib.mi__dropin_trace(0) == 0
        r = np.array(rows)
        med = lambda x: round(float(np.median(x)), 3)  # noqa: E731
        print(json.dumps(dict(
            call=name, mode=mode, calls=a.calls,
            mailbox={0: None, 1: "host", 2: "device"}[lib.mi__dropin_mailbox()] if mode == "service" else None, untraced_call_us=med(np.array(plain) * 1e6),
            traced_call_us=med(np.array(tot) * 1e6),
            entry_to_posted_us=med(r[:, 0]),
            posted_to_result_seen_us=med(r[:, 2] - r[:, 0]),
            kernel_own_us=med(r[:, 1]),
            outside_kernel_us=med(r[:, 2] - r[:, 0] - r[:, 1]),
            note="host clock from the fold's entry (after the mbuf walk and staging copy); kernel_own_us on the "
                 "GPU's 100 MHz clock (dispatch: kernel start to result store; service: request seen to result "
                 "store); outside_kernel_us = doorbell/posting to result seen minus the kernel's own time = queue "
                 "dispatch + wave launch (dispatch) or mailbox poll (service) + result visibility; call_us = the "
                 "whole ctypes call measured in Python")), flush=True)
    lib.mi__set_dropin_service(0)


if __name__ == "__main__":
    main()
