#!/usr/bin/env python3
"""Grid cap of the lane-group verify kernel vs the single-queue (1-stream)
and overlapped (2-stream) cost per launch -- a single RX queue submitting one
batch at a time pays the isolated figure (VERDICT r1 weak point 4).

    python tools/grid_iso.py [--config 1500] [--caps 512,1024,1280,2048,4096,8192]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import libunsod_amd as mi  # noqa: E402

CFG = {"1500": (65536, 1500, 2176, 142), "9000": (65536, 9000, 9216, 142)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="1500")
    ap.add_argument("--caps", default="512,1024,1280,1536,2048,4096,8192")
    ap.add_argument("--shape", default="")
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    n, L, stride, first = CFG[a.config]
    size = (first + (n - 1) * stride + L + 64 + 255) & ~255
    R = 1 + -(-(2 << 30) // (n * L))
    bs, outs = [], []
    for r in range(R):
        b = mi.PktBatch(torch.empty(size, dtype=torch.uint8, device="cuda"), n, stride=stride, first_off=first,
                        fixed_len=L)
        mi.synth_ipv4(b, seed=r + 1)
        mi.ipv4_finalize(b)
        bs.append(b)
        outs.append(dict(ip=torch.empty(n, dtype=torch.uint16, device="cuda"),
                         l4=torch.empty(n, dtype=torch.uint16, device="cuda"),
                         status=torch.empty(n, dtype=torch.uint8, device="cuda")))
    torch.cuda.synchronize()
    g, u = (int(x) for x in a.shape.split("x")) if a.shape else (0, 0)
    alg = n * L + 5 * n
    for cap in [int(x) for x in a.caps.split(",")]:
        mi.set_shape(g, u, cap)
        row = dict(config=a.config, cap=cap, shape=a.shape or "auto", kernel=mi.verify_plan(bs[0]))
        for ns in (1, 2):
            rep = mi.VerifyRepeat(bs, outs, nstreams=ns)
            rep.run(400)
            rep.run(a.steps, timed=True)
            us = rep.span() / a.steps
            rep.close()
            row[f"us_{ns}stream"] = round(us, 3)
            row[f"frac_{ns}stream"] = round(alg / us / 8e6, 4)
        iso, _ = mi.ipv4_verify_repeat(bs[:16], outs[:16], 100, nstreams=1, timing="pass")
        row["isolated_us"] = round(float(np.median(iso)), 3)
        print(json.dumps(row), flush=True)
    mi.set_shape(0, 0, 0)


if __name__ == "__main__":
    main()
