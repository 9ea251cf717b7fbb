#!/usr/bin/env python3
"""Shape / grid sweep of the RX-verify kernel on one GPU (tuning aid).

For each config, every compiled lane-group shape (G lanes x U loads) that the
packet length can use, and a few grid caps, time `steps` back-to-back launches
over rotating batches (>= 1 GiB footprint) and print one JSON line per point:
median kernel us (hipEvents), achieved GB/s (sum L + 5 B/pkt), step us.
Results never change with the shape -- tests/test_gpu_parity.py checks that.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import libunsod_amd as mi  # noqa: E402
from libunsod_amd import synth  # noqa: E402

SHAPES = [(1, 4), (1, 8), (4, 1), (4, 2), (4, 4), (8, 2), (8, 4), (8, 8), (8, 12), (16, 2), (16, 4), (16, 6), (16, 8), (32, 2),
          (32, 3), (32, 4), (32, 6), (64, 2), (64, 3), (64, 4), (64, 6), (64, 9)]
CONFIGS = {"1500": (65536, 1500, 2176, 142), "9000": (65536, 9000, 9216, 142), "64": (1 << 20, 46, 64, 14)}


def make_batches(cfg, dev):
    if cfg == "pareto":
        n = 1 << 19
        lens = synth.pareto_lengths(n)
        offs = synth.packed_offsets(lens, first_off=2)
        size = int(offs[-1] + lens[-1]) + 256
        R = max(1, -(-(1 << 30) // size))
        bs = []
        for r in range(R):
            buf = torch.empty(size, dtype=torch.uint8, device=dev)
            b = mi.PktBatch(buf, n, offs=torch.from_numpy(offs.astype(np.int64)).to(dev),
                            lens=torch.from_numpy(lens.astype(np.int32)).to(dev), max_len=int(lens.max()))
            bs.append(b)
        return bs, n, int(lens.sum()), int(lens.max())
    n, L, stride, first = CONFIGS[cfg]
    size = (first + (n - 1) * stride + L + 64 + 255) & ~255
    R = max(1, -(-(1 << 30) // size))
    bs = []
    for r in range(R):
        buf = torch.empty(size, dtype=torch.uint8, device=dev)
        bs.append(mi.PktBatch(buf, n, stride=stride, first_off=first, fixed_len=L))
    return bs, n, n * L, L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="1500,9000,64,pareto")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--grids", default="0,1024,2048,8192,16384")
    ap.add_argument("--streams", default="1,2,3,4")
    ap.add_argument("--shapes", default="", help="e.g. 8x2,16x6 (default: all that fit)")
    ap.add_argument("--rounds", type=int, default=1, help="interleaved repetitions of the whole grid")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for cfg in a.configs.split(","):
        bs, n, lsum, maxlen = make_batches(cfg, dev)
        for b in bs:
            mi.synth_ipv4(b, seed=1234)
            mi.ipv4_finalize(b)
        outs = [dict(ip=torch.empty(n, dtype=torch.uint16, device=dev),
                     l4=torch.empty(n, dtype=torch.uint16, device=dev),
                     status=torch.empty(n, dtype=torch.uint8, device=dev)) for _ in bs]
        torch.cuda.synchronize()
        ch = (maxlen + 30) // 16
        shapes = [tuple(int(x) for x in t.split("x")) for t in a.shapes.split(",")] if a.shapes else SHAPES
        for rnd, (g, u) in [(r, sh) for r in range(a.rounds) for sh in shapes]:
            if not a.shapes and (g * u > 4 * max(ch, 4) or g * u * 9 < ch):  # skip hopeless shapes
                continue
            for grid in [int(x) for x in a.grids.split(",")]:
                mi.set_shape(g, u, grid)
                iso, _ = mi.ipv4_verify_repeat(bs, outs, 60, nstreams=1, timing="pass")
                for ns in [int(x) for x in a.streams.split(",")]:
                    mi.ipv4_verify_repeat(bs, outs, 20, nstreams=ns, timing="none")
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    span = mi.ipv4_verify_repeat(bs, outs, a.steps, nstreams=ns, timing="region")
                    dt = time.perf_counter() - t0
                    chk = mi.ipv4_verify(bs[0], bad_count=True)
                    torch.cuda.synchronize()
                    ok = int(chk["bad"].item()) == 0
                    med = float(np.median(iso))
                    print(json.dumps(dict(config=cfg, round=rnd, g=g, u=u, grid=grid, streams=ns, iso_kern_us=round(med, 2),
                                          iso_GBps=round((lsum + 5 * n) / med / 1e3, 1),
                                          gpu_us_per_launch=round(span / a.steps, 2),
                                          step_us=round(dt / a.steps * 1e6, 2),
                                          job_GiBps=round(lsum * a.steps / dt / 2**30, 1), ok=ok)), flush=True)
        mi.set_shape(0, 0, 0)
        del bs, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
