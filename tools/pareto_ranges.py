#!/usr/bin/env python3
"""Byte-balanced ranges for the Pareto batch (VERDICT r4 "do this" 3): how
much does balancing buy, before paying for the pass that computes them?

The bench's 2^22-datagram Pareto batch (64-9000 B, packed, u32 offsets), 3
rotating batches, two HIP streams, back-to-back launches.  The flat-run
kernel gives each wave 64 consecutive datagrams; the byte counts of those
ranges vary by an order of magnitude.  mi__verify_ranges gives wave w the
datagrams [starts[w], starts[w+1]) instead, at most 64, from a table built
here on the host (untimed -- this bounds the gain; a product version would
build it on the GPU inside the timed region):

  greedy  close a range when it holds >= T bytes or 64 datagrams;
  bucket  cut at every multiple of T of the running byte count and every
          64th datagram after such a cut (a rule a GPU pass can apply per
          datagram with no scan);
  lpt     the same ranges dispatched heaviest first (list scheduling's
          longest-processing-time order).

T runs over multiples of the mean 64-datagram range.  Each case's outputs
are checked equal to the default kernel's.  One JSON line per case.

    python tools/pareto_ranges.py [--steps 200]
"""
from __future__ import annotations

import argparse
import ctypes as C
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
from libunsod_amd._lib import check  # noqa: E402


def greedy(lens: np.ndarray, T: float) -> np.ndarray:
    starts = [0]
    acc, cnt = 0, 0
    ll = lens.tolist()
    for i, L in enumerate(ll):
        if cnt == 64 or (cnt and acc >= T):
            starts.append(i)
            acc, cnt = 0, 0
        acc += L
        cnt += 1
    starts.append(len(ll))
    return np.array(starts, np.uint32)


def bucket(lens: np.ndarray, T: float) -> np.ndarray:
    n = len(lens)
    pre = np.concatenate([[0], np.cumsum(lens, dtype=np.int64)[:-1]])
    b = (pre // int(T)).astype(np.int64)
    first = np.concatenate([[0], np.nonzero(np.diff(b))[0] + 1])
    idx = np.arange(n)
    bf = first[np.searchsorted(first, idx, side="right") - 1]
    cut = ((idx - bf) % 64) == 0
    return np.concatenate([np.nonzero(cut)[0], [n]]).astype(np.uint32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rotate", type=int, default=3)
    a = ap.parse_args()
    lib = mi.load()
    lib.mi__verify_ranges.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_void_p, C.c_void_p, C.c_void_p]
    dev = torch.device("cuda", 0)
    n = 1 << 22
    lens = synth.pareto_lengths(n)
    offs = synth.packed_offsets(lens, first_off=2)
    size = (int(offs[-1] + lens[-1]) + 64 + 255) & ~255
    bs, outs = [], []
    for r in range(a.rotate):
        buf = torch.empty(size, dtype=torch.uint8, device=dev)
        b = mi.PktBatch(buf, n, offs=torch.from_numpy(offs.astype(np.int64)).to(dev),
                        lens=torch.from_numpy(lens.astype(np.int32)).to(dev), max_len=int(lens.max()),
                        packed=True, offs32=True)
        mi.synth_ipv4(b, seed=0x5EED5EED + 7919 * r)
        mi.ipv4_finalize(b)
        bs.append(b)
        outs.append({k: torch.empty(n, dtype=dt, device=dev)
                     for k, dt in (("ip", torch.uint16), ("l4", torch.uint16), ("status", torch.uint8))})
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    alg = float(lens.sum()) + 5.0 * n
    mean64 = float(lens.sum()) / (n / 64)

    def run(launch, steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            launch(k % a.rotate, streams[k % 2])
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e6

    def base(j, s):
        o = outs[j]
        check("verify", lib.mi_cksum_ipv4_verify(C.byref(bs[j].c), o["ip"].data_ptr(), o["l4"].data_ptr(),
                                                 o["status"].data_ptr(), None, C.c_void_p(s.cuda_stream)))

    run(base, 20)
    ref = [{k: v.clone() for k, v in o.items()} for o in outs]
    t_base = [round(run(base, a.steps), 2) for _ in range(2)]
    print(json.dumps(dict(case="default 64-datagram ranges", waves=n // 64, us_per_launch=t_base,
                          frac=round(alg / (min(t_base) * 1e-6) / 8e12, 4))), flush=True)
    byts = np.add.reduceat(lens.astype(np.int64), np.arange(0, n, 64))
    print(json.dumps(dict(case="range bytes, default", mean=round(float(byts.mean())), std=round(float(byts.std())),
                          max=int(byts.max()))), flush=True)
    # longest first: the default 64-datagram ranges (and greedy 1.25x ones),
    # dispatched heaviest first -- list scheduling's LPT order (ranges in any
    # order through an explicit end per range)
    for kind, st in (("lpt, 64-datagram ranges", np.arange(0, n + 1, 64, dtype=np.int64)),
                     ("lpt, greedy 1.25x", greedy(lens, mean64 * 1.25).astype(np.int64))):
        rb = np.add.reduceat(lens.astype(np.int64), st[:-1])
        order = np.argsort(-rb, kind="stable")
        s0 = torch.from_numpy(st[:-1][order].astype(np.int32)).to(dev)
        e0 = torch.from_numpy(st[1:][order].astype(np.int32)).to(dev)
        nr = len(order)

        def lpt(j, s, s0=s0, e0=e0, nr=nr):
            o = outs[j]
            check("ranges", lib.mi__verify_ranges(C.byref(bs[j].c), s0.data_ptr(), nr, o["ip"].data_ptr(),
                                                  o["l4"].data_ptr(), o["status"].data_ptr(), None,
                                                  C.c_void_p(s.cuda_stream), e0.data_ptr()))

        for o in outs:
            for v in o.values():
                v.fill_(0xA5)
        run(lpt, a.rotate)
        same = all(torch.equal(outs[j][k], ref[j][k]) for j in range(a.rotate) for k in ref[j])
        t = [round(run(lpt, a.steps), 2) for _ in range(2)]
        print(json.dumps(dict(case=kind, waves=nr, outputs_equal=same, us_per_launch=t,
                              frac=round(alg / (min(t) * 1e-6) / 8e12, 4), vs_default=round(min(t_base) / min(t), 3))),
              flush=True)
        if not same:
            raise SystemExit("outputs differ")
    for kind, fn in (("greedy", greedy), ("bucket", bucket)):
        for f in (0.75, 1.0, 1.25, 1.5):
            T = mean64 * f
            st = fn(lens, T)
            nr = len(st) - 1
            assert st[0] == 0 and st[-1] == n and np.all(np.diff(st.astype(np.int64)) >= 1) and \
                np.all(np.diff(st.astype(np.int64)) <= 64)
            rb = np.add.reduceat(lens.astype(np.int64), st[:-1].astype(np.int64))
            sdev = torch.from_numpy(st.astype(np.int32)).to(dev)

            def ranged(j, s, sdev=sdev, nr=nr):
                o = outs[j]
                check("ranges", lib.mi__verify_ranges(C.byref(bs[j].c), sdev.data_ptr(), nr, o["ip"].data_ptr(),
                                                      o["l4"].data_ptr(), o["status"].data_ptr(), None,
                                                      C.c_void_p(s.cuda_stream), None))

            for o in outs:
                for v in o.values():
                    v.fill_(0xA5)
            run(ranged, a.rotate)
            same = all(torch.equal(outs[j][k], ref[j][k]) for j in range(a.rotate) for k in ref[j])
            t = [round(run(ranged, a.steps), 2) for _ in range(2)]
            print(json.dumps(dict(case=kind, T_over_mean=f, waves=nr, range_bytes_mean=round(float(rb.mean())),
                                  range_bytes_std=round(float(rb.std())), range_bytes_max=int(rb.max()),
                                  outputs_equal=same, us_per_launch=t,
                                  frac=round(alg / (min(t) * 1e-6) / 8e12, 4),
                                  vs_default=round(min(t_base) / min(t), 3))), flush=True)
            if not same:
                raise SystemExit("outputs differ")


if __name__ == "__main__":
    main()
