#!/usr/bin/env python3
"""Single-queue submission: m batches per launch (mi_cksum_ipv4_verify_multi)
against one launch per batch, all on ONE stream (a lone RX queue), R rotating
batches (>= 2 GiB read between reuses).  GPU time per batch from events around
many back-to-back launches.

    python tools/bench_multi.py [--config 1500] [--ms 1,2,4,8,16]
"""
from __future__ import annotations

import argparse
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
    ap.add_argument("--ms", default="1,2,4,8,16")
    ap.add_argument("--batches", type=int, default=320, help="batches verified per measurement")
    ap.add_argument("--shapes", default="auto", help="lane-group shapes GxU to sweep (auto: the library's choice)")
    ap.add_argument("--caps", default="0", help="workgroup caps to sweep (0: the library default -- a resident-sized grid for "
                                                "the multi-batch launch, 2048 for single launches)")
    ap.add_argument("--offs", action="store_true", help="describe the slots by an int64 offset array (descriptor loads)")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    n, L, stride, first = CFG[a.config]
    size = (first + (n - 1) * stride + L + 64 + 255) & ~255
    R = max(16, 1 + -(-(2 << 30) // (n * L)))
    bs, outs = [], []
    for r in range(R):
        b = mi.PktBatch(torch.empty(size, dtype=torch.uint8, device="cuda"), n, stride=stride, first_off=first,
                        fixed_len=L)
        mi.synth_ipv4(b, seed=r + 9)
        mi.ipv4_finalize(b)
        if a.offs:
            b = mi.PktBatch(b.buf, n, offs=first + torch.arange(n, dtype=torch.int64, device="cuda") * stride,
                            fixed_len=L)
        bs.append(b)
        outs.append(dict(ip=torch.empty(n, dtype=torch.uint16, device="cuda"),
                         l4=torch.empty(n, dtype=torch.uint16, device="cuda"),
                         status=torch.empty(n, dtype=torch.uint8, device="cuda")))
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    alg = n * L + 5 * n
    shapes = [(0, 0) if x == "auto" else tuple(int(v) for v in x.split("x")) for x in a.shapes.split(",")]
    for (g, u), cap, m in [(sh, c, m) for sh in shapes for c in [int(x) for x in a.caps.split(",")]
                           for m in [int(x) for x in a.ms.split(",")]]:
        mi.set_shape(g, u, cap)
        launches = a.batches // m

        def go(k):
            for q in range(k):
                j0 = (q * m) % R
                idx = [(j0 + t) % R for t in range(m)]
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
        print(json.dumps(dict(config=a.config, layout="offs" if a.offs else "stride", shape=f"{g}x{u}" if g else "auto", batches_per_launch=m, launches=launches, streams=1, cap=cap or "default",
                              us_per_batch=round(us, 3), frac=round(alg / us / 8e6, 4),
                              GiBps=round(n * L / (us * 1e-6) / 2**30, 1))), flush=True)


    mi.set_shape(0, 0, 0)


if __name__ == "__main__":
    main()
