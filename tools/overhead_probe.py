#!/usr/bin/env python3
"""Where the wall clock of a short timed region goes.

The driver runs ``bench.py --steps 20 --warmup 5``: 20 verify launches of
~14 us each, so a fixed per-region cost of tens of us is a visible share of
``value``.  This probe times, on the bench's own 1500 B workload:

  * an idle ``torch.cuda.synchronize()``;
  * the round-1 path (``ipv4_verify_repeat``: ctypes marshalling of 8 batch
    structs, legacy-stream gate, hipStreamSynchronize per stream);
  * the prepared handle (``VerifyRepeat``) with and without region timing;
  * K = 1 and K = 20 regions, sync -> t0 -> run -> sync -> t1 (the bench's
    bracket), median over many trials, beside the GPU span of the same run;
  * the same with R rotating batches (the MALL question: R = 8 reads 789 MB
    between two reads of one batch, R = 24 reads 2.3 GB).

One JSON line per measurement on stdout.  MI_CKSUM_REPEAT_WAIT selects how
a synchronous run waits (spin / event / stream).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import libunsod_amd as mi  # noqa: E402

CFG = {"1500": (65536, 1500, 2176, 142), "9000": (65536, 9000, 9216, 142), "64": (1 << 20, 46, 64, 14)}


def batches_for(cfg: str, R: int, dev):
    n, L, stride, first = CFG[cfg]
    size = (first + (n - 1) * stride + L + 64 + 255) & ~255
    bs, outs = [], []
    for r in range(R):
        buf = torch.empty(size, dtype=torch.uint8, device=dev)
        b = mi.PktBatch(buf, n, stride=stride, first_off=first, fixed_len=L)
        mi.synth_ipv4(b, seed=0x5EED5EED + 7919 * r)
        mi.ipv4_finalize(b)
        bs.append(b)
        outs.append(dict(ip=torch.empty(n, dtype=torch.uint16, device=dev),
                         l4=torch.empty(n, dtype=torch.uint16, device=dev),
                         status=torch.empty(n, dtype=torch.uint8, device=dev)))
    torch.cuda.synchronize()
    return bs, outs, n * L + 5 * n, n * L


def bracket(fn, trials: int):
    walls, spans = [], []
    for _ in range(trials):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s = fn()
        torch.cuda.synchronize()
        walls.append((time.perf_counter() - t0) * 1e6)
        if s is not None:
            spans.append(s)
    return walls, spans


def summ(x):
    if not x:
        return None
    return dict(median=round(statistics.median(x), 2), min=round(min(x), 2),
                p90=round(sorted(x)[int(0.9 * (len(x) - 1))], 2))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="1500", choices=list(CFG))
    ap.add_argument("--rotations", default="8,24")
    ap.add_argument("--trials", type=int, default=60)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    wait = os.environ.get("MI_CKSUM_REPEAT_WAIT", "spin")

    def emit(**kw):
        kw.update(config=a.config, wait=wait, tag=a.tag)
        print(json.dumps(kw), flush=True)

    # idle device sync
    torch.cuda.synchronize()
    t = []
    for _ in range(200):
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        t.append((time.perf_counter() - t0) * 1e6)
    emit(what="idle_torch_sync_us", **summ(t))

    for R in [int(x) for x in a.rotations.split(",")]:
        bs, outs, alg, payload = batches_for(a.config, R, dev)
        rep = mi.VerifyRepeat(bs, outs, nstreams=2)
        # settle (clocks): 0.3 s of back-to-back launches
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.3:
            rep.run(500)
        # marshalling cost of the round-1 call alone (no GPU work)
        import ctypes as C
        from libunsod_amd._lib import PktBatchC
        tm = []
        for _ in range(200):
            t0 = time.perf_counter()
            arr = (PktBatchC * R)(*[b.c for b in bs])
            VP = C.c_void_p * R
            _ = {k: VP(*[o[k].data_ptr() for o in outs]) for k in ("ip", "l4", "status")}
            tm.append((time.perf_counter() - t0) * 1e6)
        emit(what="r1_marshal_us", R=R, **summ(tm))
        for K in (1, 20, 400):
            trials = a.trials if K < 400 else 10
            if R > 16:  # the round-1 call takes at most 16 batches
                w = None
            else:
                w, s = bracket(lambda: mi.ipv4_verify_repeat(bs, outs, K, nstreams=2, timing="region"), trials)
            w and emit(what="r1_repeat", R=R, K=K, wall_us=summ(w), span_us=summ(s),
                 wall_gibs=round(payload * K / (statistics.median(w) * 1e-6) / 2**30, 1),
                 span_frac=round(alg * K / (statistics.median(s) * 1e-6) / 8e12, 4))
            for timed in (False, True):
                w, s = bracket(lambda: rep.run(K, timed=timed), trials)
                emit(what="handle", timed=timed, R=R, K=K, wall_us=summ(w), span_us=summ(s),
                     wall_gibs=round(payload * K / (statistics.median(w) * 1e-6) / 2**30, 1),
                     span_frac=round(alg * K / (statistics.median(s) * 1e-6) / 8e12, 4) if s else None)
            # asynchronous run: torch.cuda.synchronize() is the only wait
            w, _ = bracket(lambda: rep.run(K, timed=True, wait=False), trials)
            emit(what="handle_async", R=R, K=K, wall_us=summ(w),
                 wall_gibs=round(payload * K / (statistics.median(w) * 1e-6) / 2**30, 1))
        rep.close()
        del bs, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
