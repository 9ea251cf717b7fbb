#!/usr/bin/env python3
"""The per-wave streaming verify (MI_CKSUM_STREAM=1) on one stream: GPU time
per batch for single launches and multi-batch launches at several grid caps,
against the lane-group kernel (k_ipv4_verify<16,6>) on the same batches.

    python tools/stream_probe.py [--config 1500] [--caps 0,512,1024,1792,2048,4096]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import libunsod_amd as mi  # noqa: E402

CFG = {"1500": (65536, 1500, 2176, 142), "9000": (65536, 9000, 9216, 142)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="1500")
    ap.add_argument("--caps", default="0,512,1024,2048,4096")
    ap.add_argument("--ms", default="1,16")
    ap.add_argument("--batches", type=int, default=320)
    ap.add_argument("--kernels", default="stream,lanegroup")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    lib = mi.load()
    lib.mi__stream_blocks_per_cu.restype = C.c_int
    print(json.dumps(dict(stream_blocks_per_cu=lib.mi__stream_blocks_per_cu(),
                          cus=torch.cuda.get_device_properties(0).multi_processor_count)), flush=True)
    n, L, stride, first = CFG[a.config]
    size = (first + (n - 1) * stride + L + 64 + 255) & ~255
    R = max(16, 1 + -(-(2 << 30) // (n * L)))
    bs, outs = [], []
    for r in range(R):
        b = mi.PktBatch(torch.empty(size, dtype=torch.uint8, device="cuda"), n, stride=stride, first_off=first,
                        fixed_len=L)
        mi.synth_ipv4(b, seed=r + 9)
        mi.ipv4_finalize(b)
        bs.append(b)
        outs.append(dict(ip=torch.empty(n, dtype=torch.uint16, device="cuda"),
                         l4=torch.empty(n, dtype=torch.uint16, device="cuda"),
                         status=torch.empty(n, dtype=torch.uint8, device="cuda")))
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    alg = n * L + 5 * n
    for kernel in a.kernels.split(","):
        os.environ["MI_CKSUM_STREAM"] = "1" if kernel == "stream" else "0"
        for cap in [int(x) for x in a.caps.split(",")]:
            for m in [int(x) for x in a.ms.split(",")]:
                mi.set_shape(0, 0, cap)
                launches = a.batches // m

                def go(k):
                    for q in range(k):
                        idx = [((q * m) + t) % R for t in range(m)]
                        if m == 1:
                            mi.ipv4_verify(bs[idx[0]], out=outs[idx[0]], stream=s)
                        else:
                            mi.ipv4_verify_multi([bs[j] for j in idx], [outs[j] for j in idx], stream=s)

                with torch.cuda.stream(s):
                    go(max(4, launches // 4))
                s.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                with torch.cuda.stream(s):
                    e0.record(s)
                    go(launches)
                    e1.record(s)
                s.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / (launches * m)
                ok = int(outs[0]["status"].sum().item()) == 0
                print(json.dumps(dict(config=a.config, kernel=mi.verify_plan(bs[0]), cap=cap or "default",
                                      batches_per_launch=m, us_per_batch=round(us, 3),
                                      frac=round(alg / us / 8e6, 4), all_valid=ok)), flush=True)
    mi.set_shape(0, 0, 0)


if __name__ == "__main__":
    main()
