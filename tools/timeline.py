#!/usr/bin/env python3
"""Per-wave timelines of the 1500 B RX verify (VERDICT r3 "do this" 2).

tools/libtimeline.so (tools/timeline.hip) runs the product's verify bodies with
three s_memrealtime stamps per wave (start, first datagram folded, end) and
the wave's XCC id.  For each submission shape this prints, per launch:

  span      first wave start -> last wave end (us)
  ramp      start -> the first time the number of running waves reaches 90 %
            of its peak
  tail      the last time running waves are >= 90 % of the peak -> end
  disp      first -> last wave start (how long the dispatcher takes to start
            every wave of the grid)
  first_us  median wave start -> its first datagram folded (first loads' latency)
  bw_*      a bytes-vs-time curve (each wave's datagram bytes spread evenly over
            its life): TB/s in the steady part and over the whole span
  per-XCD   first start, last start, last end relative to the launch start

and one summary line per shape (medians over launches).  Read shares, not the
absolute run time (the stamps cost a little).

    python tools/timeline.py [--launches 24] > timeline.jsonl
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import libunsod_amd as mi  # noqa: E402
from libunsod_amd._lib import PktBatchC  # noqa: E402

TICK_US = 0.01  # s_memrealtime: 100 MHz
N, L, STRIDE, FIRST = 65536, 1500, 2176, 142


def analyse(rec: np.ndarray, bytes_per_pkt: int) -> dict:
    t0 = rec[:, 0].astype(np.int64)
    t1 = rec[:, 1].astype(np.int64)
    t2 = rec[:, 2].astype(np.int64)
    xcc = (rec[:, 3] & 0xF).astype(np.int64)
    pk = (rec[:, 3] >> 8).astype(np.int64)
    live = t2 > 0
    t0, t1, t2, xcc, pk = t0[live], t1[live], t2[live], xcc[live], pk[live]
    base = int(t0.min())
    t0, t1, t2 = t0 - base, t1 - base, t2 - base
    end = int(t2.max())
    # running waves and bytes per tick
    run = np.zeros(end + 2, np.int64)
    np.add.at(run, t0, 1)
    np.add.at(run, t2, -1)
    run = np.cumsum(run)[:end + 1]
    peak = int(run.max())
    hi = np.nonzero(run >= 0.9 * peak)[0]
    ramp, tail = int(hi[0]), end - int(hi[-1])
    rate = np.zeros(end + 2, np.float64)
    life = np.maximum(t2 - t0, 1)
    per_tick = pk * bytes_per_pkt / life
    np.add.at(rate, t0, per_tick)
    np.add.at(rate, t2, -per_tick)
    rate = np.cumsum(rate)[:end + 1]  # bytes per tick
    tb = lambda b, ticks: b / (ticks * TICK_US) / 1e6 if ticks > 0 else 0.0  # noqa: E731
    steady = rate[int(hi[0]):int(hi[-1]) + 1]
    per_xcd = {}
    for x in np.unique(xcc):
        m = xcc == x
        per_xcd[int(x)] = [round(int(t0[m].min()) * TICK_US, 2), round(int(t0[m].max()) * TICK_US, 2),
                           round(int(t2[m].max()) * TICK_US, 2), int(m.sum())]
    return dict(span=round(end * TICK_US, 2), ramp=round(ramp * TICK_US, 2), tail=round(tail * TICK_US, 2),
                disp=round(int(t0.max()) * TICK_US, 2), waves=int(live.sum()), peak_running=peak,
                first_us=round(float(np.median(t1 - t0)) * TICK_US, 2),
                life_us=round(float(np.median(t2 - t0)) * TICK_US, 2),
                bw_steady_TBps=round(float(steady.mean()) / TICK_US / 1e6, 3) if steady.size else 0.0,
                bw_span_TBps=round(tb(float((pk * bytes_per_pkt).sum()), end), 3),
                bw_ramp_TBps=round(float(rate[:max(ramp, 1)].mean()) / TICK_US / 1e6, 3),
                bw_tail_TBps=round(float(rate[end - tail:].mean()) / TICK_US / 1e6, 3) if tail > 0 else 0.0,
                per_xcd=per_xcd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=24)
    ap.add_argument("--rotate", type=int, default=24)
    ap.add_argument("--only", default="", help="comma-separated name prefixes of the shapes to run")
    a = ap.parse_args()
    lib = C.CDLL(os.path.join(ROOT, "tools", "libtimeline.so"))
    lib.tl_run.restype = C.c_float
    lib.tl_run.argtypes = [C.c_int, C.POINTER(PktBatchC), C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                           C.POINTER(C.c_void_p), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                           C.c_uint32]
    lib.tl_occupancy.restype = C.c_int
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    size = (FIRST + (N - 1) * STRIDE + L + 64 + 255) & ~255
    R = a.rotate
    bs, outs = [], []
    for r in range(R):
        buf = torch.empty(size, dtype=torch.uint8, device=dev)
        b = mi.PktBatch(buf, N, stride=STRIDE, first_off=FIRST, fixed_len=L)
        mi.synth_ipv4(b, seed=0x5EED5EED + 7919 * r)
        mi.ipv4_finalize(b)
        bs.append(b)
        outs.append(dict(ip=torch.empty(N, dtype=torch.uint16, device=dev),
                         l4=torch.empty(N, dtype=torch.uint16, device=dev),
                         status=torch.empty(N, dtype=torch.uint8, device=dev)))
    torch.cuda.synchronize()
    arr = (PktBatchC * R)(*[b.c for b in bs])
    VP = C.c_void_p * R
    ips, l4s, sts = (VP(*[o[k].data_ptr() for o in outs]) for k in ("ip", "l4", "status"))
    occ = {m: lib.tl_occupancy(m) for m in (0, 1, 2)}
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    print(json.dumps(dict(occupancy_blocks_per_cu=occ, cus=cus)), flush=True)
    K = a.launches
    shapes = [
        ("single_16x6_1stream", 0, 1, 1, 2048),
        ("single_16x6_2streams", 0, 1, 2, 2048),
        ("single_16x6_isolated", 0, 1, 1, 2048),     # one launch, synchronize, next
        ("multi_8x2_x16_1stream", 1, 16, 1, occ[1] * cus),
        ("multi_8x2_x4_1stream", 1, 4, 1, occ[1] * cus),
        # round 5: dealt units (verify_dyn_body), one resident generation
        ("dealt_16x6_1stream", 2, 1, 1, occ[2] * cus),
        ("dealt_16x6_2streams", 2, 1, 2, occ[2] * cus),
        ("dealt_16x6_isolated", 2, 1, 1, occ[2] * cus),
    ]
    if a.only:
        shapes = [s for s in shapes if any(s[0].startswith(p) for p in a.only.split(","))]
    for name, mode, per, nst, grid in shapes:
        waves = grid * 4
        tl = torch.zeros(K * waves * 8, dtype=torch.int32, device=dev)
        # warm up
        if lib.tl_run(mode, arr, R, ips, l4s, sts, per, 8, nst, grid, 16, 6, tl.data_ptr(), tl.numel() * 4) < 0:
            raise SystemExit(f"{name}: tl_run failed")
        tl.zero_()
        if name.endswith("isolated"):
            span = 0.0
            for k in range(K):
                sub = tl[k * waves * 8:(k + 1) * waves * 8]
                j = k % R
                one = (PktBatchC * 1)(bs[j].c)
                V1 = C.c_void_p * 1
                s = lib.tl_run(mode, one, 1, V1(ips[j]), V1(l4s[j]), V1(sts[j]), 1, 1, 1, grid, 16, 6,
                               sub.data_ptr(), sub.numel() * 4)
                torch.cuda.synchronize()
                span += s
        else:
            span = lib.tl_run(mode, arr, R, ips, l4s, sts, per, K, nst, grid, 16, 6, tl.data_ptr(), tl.numel() * 4)
        torch.cuda.synchronize()
        if span < 0:
            raise SystemExit(f"{name}: tl_run failed ({span})")
        recs = tl.cpu().numpy().view(np.uint32).reshape(K, waves, 8)
        rows = []
        for k in range(K):
            r = recs[k]
            t = np.stack([r[:, 0].astype(np.uint64) | (r[:, 1].astype(np.uint64) << 32),
                          r[:, 2].astype(np.uint64) | (r[:, 3].astype(np.uint64) << 32),
                          r[:, 4].astype(np.uint64) | (r[:, 5].astype(np.uint64) << 32),
                          r[:, 6].astype(np.uint64)], axis=1)
            an = analyse(t, L)
            an.update(name=name, launch=k, batches=per)
            rows.append(an)
            print(json.dumps(an), flush=True)
        # launch-to-launch gaps (wall of the GPU timeline)
        starts = []
        for k in range(K):
            r = recs[k]
            t0 = r[:, 0].astype(np.int64) | (r[:, 1].astype(np.int64) << 32)
            t2 = r[:, 4].astype(np.int64) | (r[:, 5].astype(np.int64) << 32)
            live = t2 > 0
            starts.append((int(t0[live].min()), int(t2[live].max())))
        gaps = [round((starts[k + 1][0] - starts[k][1]) * TICK_US, 2) for k in range(K - 1)]
        med = lambda key: round(float(np.median([x[key] for x in rows])), 3)  # noqa: E731
        print(json.dumps(dict(summary=name, batches_per_launch=per, streams=nst, grid=grid, events_span_us=round(span, 2),
                              us_per_batch_events=round(span / K / per, 2),
                              **{k: med(k) for k in ("span", "ramp", "tail", "disp", "first_us", "life_us",
                                                     "bw_steady_TBps", "bw_span_TBps", "bw_ramp_TBps",
                                                     "bw_tail_TBps", "peak_running")},
                              gap_median_us=float(np.median(gaps)) if gaps else None)), flush=True)
        del tl


if __name__ == "__main__":
    main()
