#!/usr/bin/env python3
"""Where a small host RX burst's time goes (VERDICT r4 "do this" 6).

Bursts of n x 1500 B datagrams in registered host rte_mbuf slots (2176 B
apart, IP at +142) through mi_cksum_rx_offload_host, served by the device's
drop-in service.  With the drop-in trace on, each call records: request
posted (host clock, from entry), and on the GPU's 100 MHz clock from the
moment the service saw the request: acquire done, burst verified (all waves),
release done, result stored; then the result seen by the host.  Medians of
--iters calls per n and per fence mode (MI_CKSUM_BURST_FENCES is read once per
process, so each mode runs in a child process): round 5's product, 0, reads
and writes system-coherent with no fences (a wait for the stores' acks before
the result word); 1 adds a system-scope acquire before the burst, 2 a release
after it, 3 both (round 4's fences, now redundant).  profiles/r05/
burst_breakdown_r05a.jsonl is the earlier build (default-policy loads and
stores: 0 = both fences, 1 = no acquire).

    python tools/burst_breakdown.py [--sizes 1,8,32,64] [--modes 0,1,2,3]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

STRIDE, FIRST, L = 2176, 142, 1500


def child(sizes, iters, mode):
    import numpy as np
    import torch
    import libunsod_amd as mi
    from libunsod_amd._lib import PktBatchC, load
    torch.cuda.set_device(0)
    mi.set_busy_wait(True)
    lib = load()
    lib.mi__dropin_trace.argtypes = [C.c_int]
    lib.mi__dropin_trace_read.argtypes = [C.POINTER(C.c_double), C.c_int]
    nmax = max(sizes)
    size = (FIRST + (nmax - 1) * STRIDE + L + 64 + 4095) & ~4095
    dbuf = torch.empty(size, dtype=torch.uint8, device="cuda")
    db = mi.PktBatch(dbuf, nmax, stride=STRIDE, first_off=FIRST, fixed_len=L)
    mi.synth_ipv4(db, seed=0xB0057)
    mi.ipv4_finalize(db)
    raw = np.zeros(size + 8192, np.uint8)
    s = (-raw.ctypes.data) % 4096
    host = raw[s:s + size]
    host[:] = dbuf.cpu().numpy()
    mi.host_register(host)
    fl = np.zeros(nmax, np.uint32)
    cd = np.zeros(nmax, np.uint32)
    bad = C.c_uint32(0)
    out = (C.c_double * 7)()
    try:
        for n in sizes:
            bytes_n = FIRST + (n - 1) * STRIDE + L + 64
            zc = PktBatchC(host.ctypes.data, bytes_n, None, STRIDE, FIRST, None, L, n, L, 0)
            ref = C.byref(zc)
            fn = lib.mi_cksum_rx_offload_host
            for _ in range(20):
                assert fn(ref, fl.ctypes.data, cd.ctypes.data, C.addressof(bad)) == 0
            walls = []
            for _ in range(iters):
                t0 = time.perf_counter()
                rc = fn(ref, fl.ctypes.data, cd.ctypes.data, C.addressof(bad))
                walls.append(time.perf_counter() - t0)
                assert rc == 0 and bad.value == 0
            assert np.all(fl[:n] == 0xF00)
            rows = []
            assert lib.mi__dropin_trace(1) == 0
            try:
                for _ in range(iters):
                    assert fn(ref, fl.ctypes.data, cd.ctypes.data, C.addressof(bad)) == 0 and bad.value == 0
                    assert lib.mi__dropin_trace_read(out, 7) == 0
                    rows.append(list(out))
            finally:
                lib.mi__dropin_trace(0)
            m = np.median(np.array(rows), axis=0)
            print(json.dumps(dict(
                burst=n, fence_mode=mode, us_per_burst_p50=round(float(np.median(walls)) * 1e6, 2),
                us_per_burst_p90=round(float(np.percentile(walls, 90)) * 1e6, 2),
                traced=dict(posted=round(m[0], 2), seen_by_host=round(m[2], 2), gpu_request_to_result=round(m[1], 2),
                            gpu_acquire_done=round(m[4], 2), gpu_burst_done=round(m[5], 2),
                            gpu_release_done=round(m[6], 2)),
                mailbox=lib.mi__dropin_mailbox())), flush=True)
    finally:
        mi.host_unregister(host)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,8,32,64")
    ap.add_argument("--modes", default="0,1,2,3")
    ap.add_argument("--iters", type=int, default=400)
    ap.add_argument("--child", type=int, default=-1)
    a = ap.parse_args()
    sizes = [int(x) for x in a.sizes.split(",")]
    if a.child >= 0:
        child(sizes, a.iters, a.child)
        return
    for mode in [int(x) for x in a.modes.split(",")]:
        env = dict(os.environ, MI_CKSUM_BURST_FENCES=str(mode))
        r = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "--sizes", a.sizes, "--iters",
                            str(a.iters), "--child", str(mode)], env=env, timeout=300)
        if r.returncode:
            raise SystemExit(r.returncode)


if __name__ == "__main__":
    main()
