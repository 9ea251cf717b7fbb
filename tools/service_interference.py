#!/usr/bin/env python3
"""The drop-in service beside the batch path (VERDICT r4 "do this" 7).

A libuinet process has both at once: the rx kthread's batch offload
(ip_input.c:459-467 on the dpdk_rx thread, here VerifyRepeat over 65536 x
1500 B batches, the bench's AQL submission) and application threads calling
the (b1) drop-ins (ip_output.c:649-672 on the sending threads, here
in_cksum_hdr on a 20-byte header in a loop).  Each side is measured alone and
then with the other running, for 1, 4 and 16 drop-in threads, with the
drop-in service (one per device since round 5: every thread holds a mailbox
slot of it) and with one dispatch per call for every thread (on the device's
one drop-in queue since round 5; a queue per thread before):

  batch_gib_s        the batch side's rate (GiB/s of datagram bytes)
  calls_per_s        all drop-in threads together
  call_us_p50 / p99  one drop-in call's latency, over all threads' calls

Round 5: the library can keep the service out of the way while its own batch
path is busy (MI_CKSUM_SERVICE_QUIET_US, off by default since the library
places its queues): --quiet-us 500 measures that.

    python tools/service_interference.py [--seconds 2] [--quiet-us 0] > service_interference.jsonl
"""
from __future__ import annotations

import argparse
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


def make_batches(rotate: int):
    n, L, stride, first = 65536, 1500, synth.STRIDE_1500, synth.IP_OFF
    bs, outs = [], []
    for r in range(rotate):
        buf = torch.empty(first + (n - 1) * stride + L + 64, dtype=torch.uint8, device="cuda")
        b = mi.PktBatch(buf, n, stride=stride, first_off=first, fixed_len=L)
        mi.synth_ipv4(b, seed=0x5EED + r)
        mi.ipv4_finalize(b)
        bs.append(b)
        outs.append(dict(status=torch.empty(n, dtype=torch.uint8, device="cuda")))
    torch.cuda.synchronize()
    return bs, outs, float(n) * L


def batch_side(rep, bytes_per_pass: float, seconds: float, res: dict, start: threading.Event):
    start.wait()
    t0, passes = time.perf_counter(), 0
    while time.perf_counter() - t0 < seconds:
        rep.run(200)
        passes += 200
    dt = time.perf_counter() - t0
    res["batch_gib_s"] = round(bytes_per_pass * passes / dt / 2**30, 1)
    res["batch_us_per_pass"] = round(dt / passes * 1e6, 3)


def dropin_side(lib, seconds: float, lat: list, start: threading.Event, addr: int):
    fn = lib.in_cksum_hdr
    p = C.c_void_p(addr)
    fn(p)  # the thread's context (and its service, if it gets one)
    start.wait()
    mine = []
    pc = time.perf_counter
    t_end = pc() + seconds
    while True:
        t0 = pc()
        if fn(p) != 0x61B8:
            raise SystemExit("wrong in_cksum_hdr result")
        t1 = pc()
        mine.append(t1 - t0)
        if t1 > t_end:
            break
    lat.append(mine)


def run_case(lib, rep, bytes_per_pass, seconds, threads, with_batch, addr):
    start = threading.Event()
    res, lat = {}, []
    ts = []
    if with_batch:
        ts.append(threading.Thread(target=batch_side, args=(rep, bytes_per_pass, seconds, res, start)))
    for _ in range(threads):
        ts.append(threading.Thread(target=dropin_side, args=(lib, seconds, lat, start, addr)))
    for t in ts:
        t.start()
    time.sleep(0.3)  # every drop-in thread has made its first call
    start.set()
    for t in ts:
        t.join()
    if lat:
        allv = np.concatenate([np.array(x) for x in lat]) * 1e6
        res["calls_per_s"] = round(sum(len(x) for x in lat) / seconds, 0)
        res["call_us_p50"] = round(float(np.percentile(allv, 50)), 2)
        res["call_us_p99"] = round(float(np.percentile(allv, 99)), 2)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--threads", default="1,4,16")
    ap.add_argument("--rotate", type=int, default=23)
    ap.add_argument("--quiet-us", type=int, default=-1)
    a = ap.parse_args()
    if a.quiet_us >= 0:
        os.environ["MI_CKSUM_SERVICE_QUIET_US"] = str(a.quiet_us)
    lib = mi.load()
    lib.in_cksum_hdr.restype = C.c_uint
    lib.in_cksum_hdr.argtypes = [C.c_void_p]
    lib.mi__set_dropin_service.restype = C.c_int
    lib.mi__set_dropin_service.argtypes = [C.c_int]
    lib.mi__dropin_service_owners.restype = C.c_int
    hraw = np.zeros(256, np.uint8)
    off = (-hraw.ctypes.data) % 64
    hraw[off:off + 20] = np.frombuffer(KAT_HDR, np.uint8)
    addr = hraw.ctypes.data + off
    bs, outs, bytes_per_pass = make_batches(a.rotate)
    rep = mi.VerifyRepeat(bs, outs, nstreams=2, engine="aql")
    rep.run(400)
    alone = run_case(lib, rep, bytes_per_pass, a.seconds, 0, True, addr)
    print(json.dumps(dict(case="batch alone", **alone)), flush=True)
    for mode in ("service", "dispatch"):
        lib.mi__set_dropin_service(1 if mode == "service" else 0)
        for k in [int(x) for x in a.threads.split(",")]:
            solo = run_case(lib, rep, bytes_per_pass, a.seconds, k, False, addr)
            both = run_case(lib, rep, bytes_per_pass, a.seconds, k, True, addr)
            row = dict(mode=mode, dropin_threads=k, dropin_alone=solo, together=both,
                       batch_rate_vs_alone=round(both["batch_gib_s"] / alone["batch_gib_s"], 3),
                       dropin_calls_vs_alone=round(both["calls_per_s"] / solo["calls_per_s"], 3),
                       service_slots_held=lib.mi__dropin_service_owners(),
                       quiet_us=os.environ.get("MI_CKSUM_SERVICE_QUIET_US", "default"))
            print(json.dumps(row), flush=True)
    rep.close()


if __name__ == "__main__":
    main()
