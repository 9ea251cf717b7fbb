#!/usr/bin/env python3
"""Device-resident throughput of the batch operations besides the headline RX
verify, on the 1500 B slot batch and the 2^22 Pareto packed batch: TX finalize
in place, RX offload flags, RX verify with the per-protocol rules
(MI_BATCH_DEMUX), and a plain in_cksum_skip span fold.  One JSON line per
(layout, op): GPU span per launch over K launches on 2 streams, batches rotated
past the 256 MiB Infinity Cache, algorithmic bytes = datagram bytes read +
the op's output bytes written (finalize: + 4 B stored per datagram).

    python tools/bench_ops.py [--steps 200]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import libunsod_amd as mi  # noqa: E402
from libunsod_amd import synth  # noqa: E402

PEAK = 8000.0


def layouts(dev):
    n, L, stride, first = 65536, 1500, 2176, 142
    size = (first + (n - 1) * stride + L + 64 + 255) & ~255
    yield "1500", n, n * L, size, lambda buf, demux=False: mi.PktBatch(
        buf, n, stride=stride, first_off=first, fixed_len=L, demux=demux)
    n = 1 << 22
    lens = synth.pareto_lengths(n)
    offs = synth.packed_offsets(lens, first_off=2)
    size = (int(offs[-1] + lens[-1]) + 64 + 255) & ~255
    d_offs = torch.from_numpy(offs.astype(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.astype(np.int32)).to(dev)
    yield "pareto", n, int(lens.sum()), size, lambda buf, demux=False: mi.PktBatch(
        buf, n, offs=d_offs, lens=d_lens, max_len=int(lens.max()), packed=True, demux=demux)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--only-chain", action="store_true", help="just the scatter-gather chain op")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    for name, n, lsum, size, make in ([] if args.only_chain else layouts(dev)):
        R = max(2, -(-(1 << 30) // size))
        bufs = [torch.empty(size, dtype=torch.uint8, device=dev) for _ in range(R)]
        for b in bufs:
            pb = make(b)
            mi.synth_ipv4(pb, seed=17)
            mi.ipv4_finalize(pb)
        torch.cuda.synchronize()
        outs = [dict(ip=torch.empty(n, dtype=torch.uint16, device=dev), l4=torch.empty(n, dtype=torch.uint16, device=dev),
                     status=torch.empty(n, dtype=torch.uint8, device=dev),
                     flags=torch.empty(n, dtype=torch.int32, device=dev), data=torch.empty(n, dtype=torch.int32, device=dev),
                     span=torch.empty(n, dtype=torch.uint16, device=dev)) for _ in range(R)]
        plain = [make(b) for b in bufs]
        demux = [make(b, demux=True) for b in bufs]
        ops = {
            "ipv4_finalize (TX, in place)": (lambda j, s: mi.ipv4_finalize(plain[j], stream=s), 4),
            "rx_offload (csum_flags + csum_data)": (lambda j, s: mi.rx_offload(plain[j], out=outs[j], stream=s), 8),
            "ipv4_verify MI_BATCH_DEMUX": (lambda j, s: mi.ipv4_verify(demux[j], out=outs[j], stream=s), 5),
            "span_batch (in_cksum_skip)": (lambda j, s: mi.span_batch(plain[j], out=outs[j]["span"], stream=s), 2),
        }
        for op, (fn, wbytes) in ops.items():
            for k in range(20):
                fn(k % R, streams[k % 2])
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = [torch.cuda.Event(enable_timing=True) for _ in streams]
            e0.record(streams[0])
            streams[1].wait_event(e0)
            for k in range(args.steps):
                fn(k % R, streams[k % 2])
            for e, s in zip(e1, streams):
                e.record(s)
            torch.cuda.synchronize()
            us = max(e0.elapsed_time(e) for e in e1) * 1e3 / args.steps
            alg = lsum + wbytes * n
            print(json.dumps(dict(layout=name, op=op, datagrams=n, us_per_launch=round(us, 2),
                                  GiBps=round(lsum / (us / 1e6) / 2**30, 1),
                                  roofline=dict(bound="hbm", achieved=round(alg / (us / 1e6) / 1e9, 1), peak=PEAK,
                                                unit="GB/s", frac=round(alg / (us / 1e6) / 1e9 / PEAK, 4),
                                                alg_bytes_per_launch=int(alg)))), flush=True)
        del bufs, outs, plain, demux
        torch.cuda.empty_cache()
    # scatter-gather: in_cksum_skip over TX socket-buffer chains (a 54 B header
    # mbuf + 1-2 cluster pieces per 1514 B frame), the L4 part (skip 14 + 20)
    n = 65536
    c = synth.build_tx_chains(n, 1500, layout="socket", seed=3)
    R = max(2, -(-(1 << 30) // c["src"].nbytes))
    cbs = []
    for r in range(R):
        cb = mi.ChainBatch.__new__(mi.ChainBatch)
        cb.n, cb.max_seg = n, int(c["seg_len"].max())
        cb.buf = torch.from_numpy(c["src"]).to(dev)
        cb.seg_off = torch.from_numpy(c["seg_off"].astype(np.int64)).to(dev)
        cb.seg_len = torch.from_numpy(c["seg_len"].astype(np.int32)).to(dev)
        cb.pkt_seg = torch.from_numpy(c["pkt_seg"].astype(np.int32)).to(dev)
        cbs.append(cb)
    length = torch.from_numpy(c["pkt_len"].astype(np.int32)).to(dev)
    skip = torch.full((n,), 34, dtype=torch.int32, device=dev)
    outc = torch.empty(n, dtype=torch.uint16, device=dev)
    fn = lambda j, s: mi.chain_batch(cbs[j], length, skip, out=outc, stream=s)  # noqa: E731
    for k in range(20):
        fn(k % R, streams[k % 2])
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = [torch.cuda.Event(enable_timing=True) for _ in streams]
    e0.record(streams[0])
    streams[1].wait_event(e0)
    t_host = time.perf_counter()
    for k in range(args.steps):
        fn(k % R, streams[k % 2])
    for e, s in zip(e1, streams):
        e.record(s)
    t_host = time.perf_counter() - t_host
    torch.cuda.synchronize()
    us = max(e0.elapsed_time(e) for e in e1) * 1e3 / args.steps
    lsum = int(c["pkt_len"].sum()) - 34 * n
    alg = lsum + 2 * n
    print(json.dumps(dict(layout="socket chains 1514 B", op="chain_batch (in_cksum_skip over mbuf chains)",
                          datagrams=n, segments_per_chain=round(len(c["seg_len"]) / n, 2), us_per_launch=round(us, 2),
                          host_us_per_call=round(t_host * 1e6 / args.steps, 2), shape=os.environ.get("MI_CKSUM_SHAPE", "auto"),
                          GiBps=round(lsum / (us / 1e6) / 2**30, 1),
                          roofline=dict(bound="hbm", achieved=round(alg / (us / 1e6) / 1e9, 1), peak=PEAK, unit="GB/s",
                                        frac=round(alg / (us / 1e6) / 1e9 / PEAK, 4), alg_bytes_per_launch=int(alg)))),
          flush=True)


if __name__ == "__main__":
    main()
