#!/usr/bin/env python3
"""Lane-group shape x grid cap sweep of the fused TX copy (mi_cksum_tx_copy).

The copy-ceiling probe (tools/ceiling_copy.py) is fastest with every lane
issuing its loads once and leaving (grid 16384, 2 chunks per lane: 0.67 of
8 TB/s on the slot geometry, against 0.56-0.62 at grid 2048-8192).  The TX
kernel's default (8x2, cap 2048) walks each frame in six serialized 256-byte
passes per lane group instead.  Here every compiled TX shape (G lanes per
frame x U chunks per lane per pass) runs at several grid caps over the same
rotating batches (two streams, back-to-back launches, as tools/bench_tx.py);
every point's frames and status bytes are compared with the default's.  One
JSON line per point.

    python tools/tx_sweep.py [--layout socket] [--shapes 8x2,16x6,32x4,64x2] [--caps 2048,8192,16384]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layout", default="socket")
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--ip-len", type=int, default=1500)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--shapes", default="8x2,16x2,16x6,32x4,64x2")
    ap.add_argument("--caps", default="2048,8192,16384")
    a = ap.parse_args()

    import libunsod_amd as mi
    from tx_cases import make_case

    n, L = a.n, a.ip_len
    stride = 2176
    c = make_case(n, L, layout=a.layout, seed=41, stride=stride)
    frame = L + 14
    dev = torch.device("cuda", 0)
    per = c["src"].nbytes + c["dst"].nbytes
    R = max(2, -(-(1 << 30) // per))
    batches = []
    for _ in range(R):
        src = torch.from_numpy(c["src"]).to(dev)
        dst = torch.from_numpy(c["dst"]).to(dev)
        tb = mi.TxBatch(src, c["seg_off"], c["seg_len"], c["pkt_seg"], c["pkt_len"], dst, dst_stride=stride,
                        dst_first=c["dst_first"], room=c["room"], l3_off=14, max_len=frame)
        batches.append((tb, torch.empty(n, dtype=torch.uint8, device=dev)))
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    alg = n * (2.0 * frame + 1)

    def run(k):
        for j in range(k):
            tb, st = batches[j % R]
            mi.tx_copy(tb, status=st, stream=streams[j % 2])

    def timed(k):
        ev0 = [torch.cuda.Event(enable_timing=True) for _ in streams]
        ev1 = [torch.cuda.Event(enable_timing=True) for _ in streams]
        gate = torch.cuda.Event()
        gate.record(streams[0])
        for s in streams[1:]:
            s.wait_event(gate)
        for e, s in zip(ev0, streams):
            e.record(s)
        run(k)
        for e, s in zip(ev1, streams):
            e.record(s)
        torch.cuda.synchronize()
        return max(ev0[0].elapsed_time(e) for e in ev1) * 1e3 / k

    def isolated():
        iso = []
        for j in range(20):
            x, y = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            x.record()
            mi.tx_copy(batches[j % R][0], status=batches[j % R][1])
            y.record()
            torch.cuda.synchronize()
            iso.append(x.elapsed_time(y) * 1e3)
        return sorted(iso)[len(iso) // 2]

    ref = None
    for shape in a.shapes.split(","):
        os.environ["MI_CKSUM_TX_SHAPE"] = shape
        for cap in [int(x) for x in a.caps.split(",")]:
            mi.set_shape(0, 0, cap)
            tb, st = batches[0]
            tb.dst.fill_(0xA5)
            st.fill_(0xA5)
            mi.tx_copy(tb, status=st)
            torch.cuda.synchronize()
            got = (tb.dst.clone(), st.clone())
            if ref is None:
                ref = got
            same = torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])
            run(20)
            torch.cuda.synchronize()
            us = min(timed(a.steps), timed(a.steps))
            print(json.dumps(dict(layout=a.layout, shape=shape, grid_cap=cap, same_as_first=same,
                                  us_per_launch=round(us, 2), isolated_us=round(isolated(), 2),
                                  frac=round(alg / (us * 1e-6) / 8e12, 4))), flush=True)
            if not same:
                raise SystemExit("outputs differ")
    mi.set_shape(0, 0, 0)


if __name__ == "__main__":
    main()
