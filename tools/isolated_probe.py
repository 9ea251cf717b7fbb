#!/usr/bin/env python3
"""One verify launch in flight -- the RX hook's real shape (one kthread, one
queue, one burst at a time; uinet_if_dpdk.c:900-937) -- measured three ways
on the bench's batches (VERDICT r5 "what's weak" 4):

  kernel_us   a single AQL packet on one queue, submitted alone and waited
              for: its dispatch timestamps (start -> end of the kernel itself)
  serial_us   K packets on ONE queue with the barrier bit: back to back, no
              overlap between launches (span / K)
  wall_us     host wall clock of one synchronous submission (submit, spin on
              the completion signal): what a caller waiting for its burst sees
  overlap_us  the bench's two-queue region (span / K), for reference

    python tools/isolated_probe.py [--configs 1500,9000,64,pareto] [--reps 200]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="1500,9000,64,pareto")
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--k", type=int, default=200)
    ap.add_argument("--caps", default="0", help="grid caps to try (mi_cksum_set_shape(0, 0, cap); 0 = the plan's)")
    args = ap.parse_args()
    import bench
    import libunsod_amd as mi
    from libunsod_amd import shard, synth
    mi.set_busy_wait(True)
    dev = torch.device("cuda", 0)
    for cfg in args.configs.split(","):
        wl = bench.build_workload(mi, synth, shard, cfg, 0, False, dev, 0, 1)
        n, L_sum = wl["n"], wl["L_sum"]
        alg = L_sum + float(wl.get("out_bytes", 5)) * n
        torch.cuda.synchronize()
        for cap in [int(c) for c in args.caps.split(",")]:
            mi.set_shape(0, 0, cap)
            measure(mi, bench, wl, cfg, cap, alg, args)
        mi.set_shape(0, 0, 0)
        del wl
        torch.cuda.empty_cache()


def measure(mi, bench, wl, cfg, cap, alg, args):
    one = mi.VerifyRepeat(wl["batches"], wl["outs"], nstreams=1, engine="aql")
    two = mi.VerifyRepeat(wl["batches"], wl["outs"], nstreams=2, engine="aql")
    one.run(args.k, timed=True)  # warm
    two.run(args.k, timed=True)
    kern, wall = [], []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        one.run(1, timed=True)
        wall.append((time.perf_counter() - t0) * 1e6)
        kern.append(one.span())
    one.run(args.k, timed=True)
    serial = one.span() / args.k
    two.run(args.k, timed=True)
    overlap = two.span() / args.k
    one.close()
    two.close()
    km, wm = float(np.median(kern)), float(np.median(wall))
    print(json.dumps(dict(config=cfg, grid_cap=cap or "plan", plan=bench.repeat_plan(wl["batches"][0]), alg_bytes=int(alg),
                          kernel_us=round(km, 2), kernel_frac=round(alg / km / 1e3 / bench.HBM_PEAK_GBS, 4),
                          kernel_us_p10_p90=[round(float(np.percentile(kern, q)), 2) for q in (10, 90)],
                          wall_us=round(wm, 2), wall_frac=round(alg / wm / 1e3 / bench.HBM_PEAK_GBS, 4),
                          serial_us=round(serial, 2), serial_frac=round(alg / serial / 1e3 / bench.HBM_PEAK_GBS, 4),
                          overlap_us=round(overlap, 2),
                          overlap_frac=round(alg / overlap / 1e3 / bench.HBM_PEAK_GBS, 4))), flush=True)


if __name__ == "__main__":
    main()
