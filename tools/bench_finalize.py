#!/usr/bin/env python3
"""TX finalize in place (in_delayed_cksum ip_output.c:958-983 + ip_sum
:667-672) beside RX verify on the same batches, submitted like bench.py (a
prepared handle, K back-to-back passes alternating over 2 streams, R rotating
batches with >= 2 GiB read between two uses of one).  One JSON line per
(config, op): GPU span per pass, algorithmic bytes = datagram bytes read + the
op's bytes written (finalize: 4 B, verify: 5 B per datagram), fraction of the
8 TB/s spec peak.  MI_CKSUM_TX_BLOCKS=0 selects the byte-store finalize (A/B).

    python tools/bench_finalize.py [--configs 1500,9000,pareto,64] [--steps 400]
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
from libunsod_amd import synth  # noqa: E402

CFG = {"1500": (65536, 1500, 2176, 142), "9000": (65536, 9000, 9216, 142), "64": (1 << 20, 46, 64, 14)}


def make_batches(cfg, dev):
    if cfg == "pareto":
        n = 1 << 22
        lens = synth.pareto_lengths(n)
        offs = synth.packed_offsets(lens, first_off=2)
        size = (int(offs[-1] + lens[-1]) + 64 + 255) & ~255
        d_offs = torch.from_numpy(offs.astype(np.int64)).to(dev)
        d_lens = torch.from_numpy(lens.astype(np.int32)).to(dev)
        lsum = int(lens.sum())
        mk = lambda buf: mi.PktBatch(buf, n, offs=d_offs, lens=d_lens, max_len=int(lens.max()),  # noqa: E731
                                     packed=True, offs32=True)
    else:
        n, L, stride, first = CFG[cfg]
        size = (first + (n - 1) * stride + L + 64 + 255) & ~255
        lsum = n * L
        mk = lambda buf: mi.PktBatch(buf, n, stride=stride, first_off=first, fixed_len=L)  # noqa: E731
    read = min(size, lsum + 16 * n)
    R = 1 + -(-(2 << 30) // read)
    bs = []
    for r in range(R):
        b = mk(torch.empty(size, dtype=torch.uint8, device=dev))
        mi.synth_ipv4(b, seed=0x5EED + r)
        mi.ipv4_finalize(b)
        bs.append(b)
    torch.cuda.synchronize()
    return bs, n, lsum


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="1500,9000,pareto,64")
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--ops", default="finalize,verify", help="order of the measured ops (A/A: verify,verify)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    blocks = os.environ.get("MI_CKSUM_TX_BLOCKS", "1") != "0"
    for cfg in a.configs.split(","):
        bs, n, lsum = make_batches(cfg, dev)
        outs = [dict(ip=torch.empty(n, dtype=torch.uint16, device=dev),
                     l4=torch.empty(n, dtype=torch.uint16, device=dev),
                     status=torch.empty(n, dtype=torch.uint8, device=dev)) for _ in bs]
        wbytes = {"finalize": 4, "verify": 5}
        # one handle at a time: two live handles' streams can share a hardware
        # queue (GPU_MAX_HW_QUEUES = 4) and serialise the 2-stream overlap
        for rnd in range(a.rounds):
            for op in a.ops.split(","):
                rep = mi.VerifyRepeat(bs, outs if op == "verify" else None, nstreams=2, op=op)
                rep.run(1000)
                rep.run(a.steps, timed=True)
                us = rep.span() / a.steps
                rep.close()
                alg = lsum + wbytes[op] * n
                print(json.dumps(dict(config=cfg, op=op, tx_blocks=blocks, lib=os.path.basename(mi.LIB_PATH),
                                      round=rnd, R=len(bs), datagrams=n,
                                      us_per_launch=round(us, 3), GiBps=round(lsum / (us * 1e-6) / 2**30, 1),
                                      alg_TBps=round(alg / us / 1e6, 3), frac=round(alg / us / 8e6, 4))),
                      flush=True)
        del bs, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
