#!/usr/bin/env python3
"""Does reading ONE batch with both queues beat reading two batches at once?
The bench's AQL engine gives pass k (a whole batch) to queue k % 2, so the two
queues read two different batches at any moment.  Here the same batches are
also submitted as half-batch dispatches (first half -> queue 0, second half ->
queue 1), so both queues read adjacent halves of one batch.  Same bytes, same
kernels; GPU span per whole batch, interleaved rounds.

    python tools/split_probe.py [--steps 400] [--rounds 3]
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
    R = 1 + -(-(2 << 30) // (n * L))
    whole, halves, ow, oh = [], [], [], []
    for r in range(R):
        buf = torch.empty(size, dtype=torch.uint8, device="cuda")
        b = mi.PktBatch(buf, n, stride=stride, first_off=first, fixed_len=L)
        mi.synth_ipv4(b, seed=0x5EED5EED + 7919 * r)
        mi.ipv4_finalize(b)
        o = dict(ip=torch.empty(n, dtype=torch.uint16, device="cuda"), l4=torch.empty(n, dtype=torch.uint16, device="cuda"),
                 status=torch.empty(n, dtype=torch.uint8, device="cuda"))
        whole.append(b)
        ow.append(o)
        h = n // 2
        for k in range(2):
            halves.append(mi.PktBatch(buf, h, stride=stride, first_off=first + k * h * stride, fixed_len=L))
            oh.append({key: t[k * h:(k + 1) * h] for key, t in o.items()})
    torch.cuda.synchronize()
    rw = mi.VerifyRepeat(whole, ow, nstreams=2, engine="aql")
    rh = mi.VerifyRepeat(halves, oh, nstreams=2, engine="aql")
    K = a.steps
    rw.run(2000)
    rh.run(4000)
    alg = n * L + 5 * n
    for rnd in range(a.rounds):
        for name, rep, k in (("whole batches, queue k%2", rw, K), ("half batches, both queues on one batch", rh, 2 * K)):
            rep.run(k, timed=True)
            us = rep.span() / K
            print(json.dumps(dict(round=rnd, submission=name, steps=K, us_per_batch=round(us, 3),
                                  frac=round(alg / us / 8e6, 4))), flush=True)
    chk = mi.ipv4_verify(whole[0], bad_count=True)
    torch.cuda.synchronize()
    assert int(chk["bad"].item()) == 0
    rw.close()
    rh.close()


if __name__ == "__main__":
    main()
