#!/usr/bin/env python3
"""What a resident drop-in service costs the batch path while it is idle.

tools/service_interference.py (round 5) measured the 1500 B batch rate at
0.64-0.65x while drop-in threads used the service, against 0.90-0.96x with a
dispatch per call.  Here the service is alive but gets no request (its idle
exit pushed out to 5 s) while the batch side runs alone, for several poll
periods of its polling wave (s_sleep units of 64 clocks between polls of the
slots); then one thread's in_cksum_hdr latency with that poll period, without
the batch.  One JSON line per case.

    python tools/service_idle_probe.py
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys
import time

# (the service must stay up beside the batch here: no standing aside)
os.environ["MI_CKSUM_SERVICE_QUIET_US"] = "0"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import libunsod_amd as mi  # noqa: E402
from libunsod_amd import synth  # noqa: E402

KAT_HDR = bytes.fromhex("450000730000400040110000c0a80001c0a800c7")


def rate_of(rep, n, L, seconds=1.5):
    t0, passes = time.perf_counter(), 0
    while time.perf_counter() - t0 < seconds:
        rep.run(200)
        passes += 200
    return round(float(n) * L * passes / (time.perf_counter() - t0) / 2**30, 1)


def main():
    lib = mi.load()
    lib.mi__set_dropin_service.argtypes = [C.c_int]
    lib.mi__set_dropin_service_params.argtypes = [C.c_uint32, C.c_uint32]
    lib.mi__dropin_service_live.restype = C.c_int
    lib.in_cksum_hdr.restype = C.c_uint
    lib.in_cksum_hdr.argtypes = [C.c_void_p]
    hraw = np.zeros(256, np.uint8)
    off = (-hraw.ctypes.data) % 64
    hraw[off:off + 20] = np.frombuffer(KAT_HDR, np.uint8)
    addr = C.c_void_p(hraw.ctypes.data + off)
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

    lib.mi__set_dropin_service(0)
    lib.mi__spin.argtypes = [C.c_uint32, C.c_int]
    base = rate()
    print(json.dumps(dict(case="no service", batch_gib_s=base)), flush=True)
    # any resident wave, no memory traffic: via a HIP stream, the service's
    # queue, the drop-in dispatch queue
    lib.mi__dropin_queue_id.restype = C.c_longlong
    lib.mi__dropin_queue_id.argtypes = [C.c_int]
    lib.mi__repeat_queue_id.restype = C.c_longlong
    lib.mi__repeat_queue_id.argtypes = [C.c_void_p, C.c_int]
    for via, name in ((0, "HIP stream"), (1, "service queue"), (2, "dispatch queue")):
        assert lib.mi__spin(2_500_000, via) == 0
        time.sleep(0.1)
        r = rate()
        print(json.dumps(dict(case="resident spin wave", via=name, batch_gib_s=r, batch_vs_none=round(r / base, 3),
                              batch_queue_ids=[lib.mi__repeat_queue_id(rep._h, i) for i in (0, 1)],
                              dropin_queue_ids=[lib.mi__dropin_queue_id(0), lib.mi__dropin_queue_id(1)],
                              spacers=lib.mi__placement_spacers())), flush=True)
        time.sleep(1.0)  # (the spin ends)
    # one queue for the batch side, with and without the service
    rep1 = mi.VerifyRepeat(bs, outs, nstreams=1, engine="aql")
    rep1.run(200)
    r1 = rate_of(rep1, n, L)
    lib.mi__set_dropin_service_params(5_000_000, 1)
    lib.mi__set_dropin_service(1)
    assert lib.in_cksum_hdr(addr) == 0x61B8
    r1s = rate_of(rep1, n, L)
    print(json.dumps(dict(case="batch on one queue", batch_gib_s=r1, with_service_gib_s=r1s,
                          ratio=round(r1s / r1, 3), live=lib.mi__dropin_service_live())), flush=True)
    lib.mi__set_dropin_service(0)
    rep1.close()
    for poll in (1, 4, 16, 64, 255):
        lib.mi__set_dropin_service_params(5_000_000, poll)
        lib.mi__set_dropin_service(0)  # stops the running one: the next call launches with the new params
        lib.mi__set_dropin_service(1)
        assert lib.in_cksum_hdr(addr) == 0x61B8
        live0 = lib.mi__dropin_service_live()
        r = rate()
        live1 = lib.mi__dropin_service_live()
        lat = []
        for _ in range(2000):
            t0 = time.perf_counter()
            lib.in_cksum_hdr(addr)
            lat.append(time.perf_counter() - t0)
        lat = np.array(lat) * 1e6
        print(json.dumps(dict(case="service alive, idle", poll_sleep_units=poll, live=[live0, live1], batch_gib_s=r,
                              batch_vs_none=round(r / base, 3),
                              in_cksum_hdr_us_p50=round(float(np.median(lat)), 2),
                              in_cksum_hdr_us_p99=round(float(np.percentile(lat, 99)), 2))), flush=True)
    lib.mi__set_dropin_service_params(0, 1)
    lib.mi__set_dropin_service(0)
    lib.mi__set_dropin_service(1)
    rep.close()


if __name__ == "__main__":
    main()
