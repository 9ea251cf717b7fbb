#!/usr/bin/env python3
"""Do two lock-stepped queues lose a ramp/drain bubble at every pass pair?

The bench's two queues start their first passes together and, passes being
equal, stay in step: every pair of passes drains and ramps together.  Here the
same kernels run on two HIP streams over the same rotating 1500 B batches,
(a) in step (both streams start with a whole batch) and (b) staggered by half a
pass (stream 1 starts with half a batch -- the half-batch views cover the same
bytes -- so its passes start mid-way through stream 0's).  GPU span per whole
batch from events, interleaved rounds.

    python tools/stagger_probe.py [--steps 400] [--rounds 3]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import libunsod_amd as mi  # noqa: E402
from libunsod_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    n, L, stride, first = 65536, 1500, synth.STRIDE_1500, synth.IP_OFF
    size = (first + (n - 1) * stride + L + 64 + 255) & ~255
    R = 2 * (1 + -(-(2 << 30) // (n * L)) // 2)
    bs, outs = [], []
    for r in range(R):
        buf = torch.empty(size, dtype=torch.uint8, device="cuda")
        b = mi.PktBatch(buf, n, stride=stride, first_off=first, fixed_len=L)
        mi.synth_ipv4(b, seed=0x5EED5EED + 7919 * r)
        mi.ipv4_finalize(b)
        bs.append(b)
        outs.append(dict(ip=torch.empty(n, dtype=torch.uint16, device="cuda"),
                         l4=torch.empty(n, dtype=torch.uint16, device="cuda"),
                         status=torch.empty(n, dtype=torch.uint8, device="cuda")))
    h = n // 2
    half = mi.PktBatch(bs[1].buf, h, stride=stride, first_off=first, fixed_len=L)
    half_out = {k: t[:h] for k, t in outs[1].items()}
    torch.cuda.synchronize()
    mi.set_busy_wait(True)
    s = [torch.cuda.Stream(), torch.cuda.Stream()]
    alg = n * L + 5 * n
    K = a.steps

    def go(stagger):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = [torch.cuda.Event(enable_timing=True) for _ in s]
        e0.record(s[0])
        s[1].wait_event(e0)
        work = 0.0
        if stagger:  # stream 1 opens with half a batch
            mi.ipv4_verify(half, out=half_out, stream=s[1])
            work += 0.5
        for k in range(K):
            q = k % 2
            mi.ipv4_verify(bs[k % R], out=outs[k % R], stream=s[q])
            work += 1
        for e, st in zip(e1, s):
            e.record(st)
        torch.cuda.synchronize()
        return max(e0.elapsed_time(e) for e in e1) * 1e3 / work

    go(False)
    go(True)
    for rnd in range(a.rounds):
        for stagger in (False, True):
            us = go(stagger)
            print(json.dumps(dict(round=rnd, streams=2, stagger=stagger, steps=K, us_per_batch=round(us, 3),
                                  frac=round(alg / us / 8e6, 4))), flush=True)


if __name__ == "__main__":
    main()
