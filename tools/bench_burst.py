#!/usr/bin/env python3
"""Per-burst latency at the reference's batch point.

The offload hook sits in if_dpdk_batch_receive (uinet_if_dpdk.c:854-879),
after rte_eth_rx_burst hands over at most 512 packets (MAX_BURST_SIZE,
src/lib/libdpdk_helper/dpdk_helper.h:20; dh_recv_pkts dpdk_helper.c:204-221)
out of a ring of rx_batch_size = 4096 descriptors (uinet_api.c:1983).  The
burst lies in host memory (hugepage rte_mbufs, 2176 B slots, IP at +142).
Per burst size n this times, median over many bursts, through the C ABI with
everything prepared beforehand (one ctypes call per burst):

  gpu_zero_copy   mi_cksum_rx_offload_host on registered (mapped) slots: the
                  kernel reads the datagrams over PCIe in place, csum_flags /
                  csum_data come back to host arrays -- the hook's real call;
  gpu_staged      the same through the staged copy ring;
  gpu_device      the burst already in HBM: mi_cksum_rx_offload on a stream +
                  the flags' D2H copy into pinned memory + synchronize;
  cpu_reference   the reference's own in_cksum.c (oracle/_ref) doing what
                  ip_input + tcp_input do per packet, one thread.

One JSON line per n.

    python tools/bench_burst.py [--sizes 32,64,128,256,512,1024,4096]
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
import torch  # noqa: E402

import libunsod_amd as mi  # noqa: E402
from libunsod_amd._lib import MI_BATCH_HOST_STAGED, PktBatchC, load  # noqa: E402
from oracle.pyoracle import Oracle, available  # noqa: E402

STRIDE, FIRST, L = 2176, 142, 1500


def med_us(fn, iters):
    fn()
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(float(np.median(ts)) * 1e6, 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="32,64,128,256,512,1024,4096")
    ap.add_argument("--iters", type=int, default=300)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    mi.set_busy_wait(True)  # a polling RX thread, like the reference's dpdk_rx
    lib = load()
    sizes = [int(x) for x in a.sizes.split(",")]
    nmax = max(sizes)
    # the ring of host slots, valid packets (device synth + finalize, then host)
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
    ref = Oracle("reference" if available("reference") else "port")
    fl = np.zeros(nmax, np.uint32)
    cd = np.zeros(nmax, np.uint32)
    bad = C.c_uint32(0)
    pin_fl = torch.empty(nmax, dtype=torch.int32).pin_memory()
    pin_cd = torch.empty(nmax, dtype=torch.int32).pin_memory()
    stream = torch.cuda.Stream()
    try:
        for n in sizes:
            bytes_n = FIRST + (n - 1) * STRIDE + L + 64
            zc = PktBatchC(host.ctypes.data, bytes_n, None, STRIDE, FIRST, None, L, n, L, 0)
            st = PktBatchC(host.ctypes.data, bytes_n, None, STRIDE, FIRST, None, L, n, L, MI_BATCH_HOST_STAGED)
            f_ptr, c_ptr, b_ptr = fl.ctypes.data, cd.ctypes.data, C.addressof(bad)
            zc_ref, st_ref = C.byref(zc), C.byref(st)
            rx_host = lib.mi_cksum_rx_offload_host

            def gpu_zc():
                rc = rx_host(zc_ref, f_ptr, c_ptr, b_ptr)
                assert rc == 0 and bad.value == 0

            def gpu_staged():
                rc = rx_host(st_ref, f_ptr, c_ptr, b_ptr)
                assert rc == 0 and bad.value == 0

            sub = mi.PktBatch(dbuf[:bytes_n], n, stride=STRIDE, first_off=FIRST, fixed_len=L)
            outs = dict(flags=torch.empty(n, dtype=torch.int32, device="cuda"),
                        data=torch.empty(n, dtype=torch.int32, device="cuda"))

            def gpu_device():
                with torch.cuda.stream(stream):
                    mi.rx_offload(sub, out=outs, stream=stream)
                    pin_fl[:n].copy_(outs["flags"], non_blocking=True)
                    pin_cd[:n].copy_(outs["data"], non_blocking=True)
                stream.synchronize()

            def cpu_ref():
                ref.ipv4_verify_batch(host, n, stride=STRIDE, first_off=FIRST, fixed_flen=L)

            res = dict(burst=n, datagram_len=L, slot_stride=STRIDE, unit="us per burst (median)",
                       iters=a.iters, busy_wait=True)
            res["gpu_zero_copy"] = med_us(gpu_zc, a.iters)
            want_fl = fl[:n].copy()
            assert np.all(want_fl == 0xF00), want_fl[:4]  # IP_CHECKED|IP_VALID|DATA_VALID|PSEUDO_HDR
            res["gpu_staged"] = med_us(gpu_staged, a.iters)
            assert np.array_equal(fl[:n], want_fl)
            res["gpu_device_resident"] = med_us(gpu_device, a.iters)
            assert np.array_equal(pin_fl[:n].numpy().astype(np.uint32), want_fl)
            res["cpu_reference_1thread"] = med_us(cpu_ref, max(20, a.iters // 4))
            res["cpu_kind"] = ref.kind
            for k in ("gpu_zero_copy", "gpu_staged", "gpu_device_resident", "cpu_reference_1thread"):
                res[k + "_mpps"] = round(n / res[k], 3)
            print(json.dumps(res), flush=True)
    finally:
        mi.host_unregister(host)


if __name__ == "__main__":
    main()
