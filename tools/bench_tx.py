#!/usr/bin/env python3
"""TX checksum offload fused with the driver's copy (mi_cksum_tx_copy,
SURVEY.md 8(f) rank 2): device-resident throughput on one GPU.

A step = one launch over a batch of n frames: every frame's mbuf chain
(socket layout: a 54 B header mbuf + payload pieces in 2 KiB socket-buffer
clusters, synth.build_tx_chains) gathered into its rte_mbuf slot (stride
2176, data at +128) with ip_sum and th_sum computed on the way.  Algorithmic
bytes per frame = len read + len written + 1 B status.  Batches rotate so the
footprint exceeds the 256 MiB Infinity Cache.  The reference's software path
(in_delayed_cksum + in_cksum + m_copydata per frame, oracle/_ref) is timed on
a bounded sample of the same frames.

    python tools/bench_tx.py [--ip-len 1500] [--n 65536] [--steps 200] [--layout socket]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ip-len", type=int, default=1500)
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--layout", default="socket")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--cpu-seconds", type=float, default=5.0)
    ap.add_argument("--check", action="store_true", help="compare one batch with the oracle")
    ap.add_argument("--shape", default="", help="GxU (mi_cksum_set_shape); default automatic")
    args = ap.parse_args()

    import libunsod_amd as mi
    from libunsod_amd import synth
    from tx_cases import make_case, run_oracle

    if args.shape:
        mi.set_shape(*[int(x) for x in args.shape.split("x")])
    n, L = args.n, args.ip_len
    stride = 2176 if L <= 2048 - 14 else ((L + 14 + 128 + 255) // 256) * 256
    c = make_case(n, L, layout=args.layout, seed=41, stride=stride)
    frame = L + 14
    dev = torch.device("cuda", 0)
    per = c["src"].nbytes + c["dst"].nbytes
    R = max(2, -(-(1 << 30) // per))
    batches = []
    for r in range(R):
        src = torch.from_numpy(c["src"]).to(dev)
        dst = torch.from_numpy(c["dst"]).to(dev)
        tb = mi.TxBatch(src, c["seg_off"], c["seg_len"], c["pkt_seg"], c["pkt_len"], dst, dst_stride=stride,
                        dst_first=c["dst_first"], room=c["room"], l3_off=14, max_len=frame)
        st = torch.empty(n, dtype=torch.uint8, device=dev)
        batches.append((tb, st))
    torch.cuda.synchronize()
    res = {}
    if args.check:
        want_dst, want_st = run_oracle(__import__("oracle.pyoracle", fromlist=["Oracle"]).Oracle("port"), c)
        mi.tx_copy(batches[0][0], status=batches[0][1])
        torch.cuda.synchronize()
        got = batches[0][0].dst.cpu().numpy()
        res["check"] = bool(np.array_equal(got, want_dst) and
                            np.array_equal(batches[0][1].cpu().numpy(), want_st))
    streams = [torch.cuda.Stream(dev) for _ in range(args.streams)]

    def run(k):
        for j in range(k):
            tb, st = batches[j % R]
            mi.tx_copy(tb, status=st, stream=streams[j % len(streams)])

    run(args.warmup)
    torch.cuda.synchronize()
    t_end = time.perf_counter() + 0.3
    while time.perf_counter() < t_end:
        run(50)
        torch.cuda.synchronize()
    ev0 = [torch.cuda.Event(enable_timing=True) for _ in streams]
    ev1 = [torch.cuda.Event(enable_timing=True) for _ in streams]
    gate = torch.cuda.Event()
    gate.record(streams[0])
    for s in streams[1:]:
        s.wait_event(gate)
    for e, s in zip(ev0, streams):
        e.record(s)
    t0 = time.perf_counter()
    run(args.steps)
    for e, s in zip(ev1, streams):
        e.record(s)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    span_ms = max(ev0[0].elapsed_time(e) for e in ev1)
    us = span_ms * 1e3 / args.steps
    alg = n * (2.0 * frame + 1)
    iso = []
    for j in range(20):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        mi.tx_copy(batches[j % R][0], status=batches[j % R][1])
        b.record()
        torch.cuda.synchronize()
        iso.append(a.elapsed_time(b) * 1e3)
    res.update(shape=args.shape or os.environ.get("MI_CKSUM_TX_SHAPE", "auto"), op="tx_copy (fused m_copydata + in_delayed_cksum + ip_sum)", layout=args.layout, frames=n,
               frame_len=frame, segments_per_frame=round((len(c["seg_len"])) / n, 2), rotating=R,
               us_per_launch=round(us, 2), isolated_us=round(float(np.median(iso)), 2),
               frames_GiBps=round(n * frame / (us / 1e6) / 2**30, 1),
               roofline=dict(bound="hbm", achieved=round(alg / (us / 1e6) / 1e9, 1), peak=HBM_PEAK_GBS,
                             unit="GB/s", frac=round(alg / (us / 1e6) / 1e9 / HBM_PEAK_GBS, 4),
                             alg_bytes_per_launch=int(alg)),
               wall_GiBps=round(n * frame * args.steps / wall / 2**30, 1))
    if args.cpu_seconds > 0:
        from oracle.pyoracle import Oracle, available
        kind = "reference" if available("reference") else "port"
        o = Oracle(kind)
        m = min(n, 8192)
        sub = make_case(m, L, layout=args.layout, seed=41, stride=stride)
        passes, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < args.cpu_seconds:
            run_oracle(o, sub)
            passes += 1
        dt = time.perf_counter() - t0
        res["cpu_baseline"] = dict(value=round(passes * m * frame / dt / 2**30, 3), unit="GiB/s of frames",
                                   cores=1, kind=kind,
                                   sample=f"{passes} passes x {m} frames ({dt:.1f} s, 1 thread): m_copydata + "
                                          "in_delayed_cksum + in_cksum per frame")
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
