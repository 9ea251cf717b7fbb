#!/usr/bin/env python3
"""Read ceiling of the bench's pattern, beside the verify kernel.

For each config and rotation depth R: the verify kernel (bench submission:
K back-to-back launches alternating over 2 streams, R rotating batches) and
tools/libceiling.so's read-only kernels over the SAME batches with the same
submission -- slot envelopes (the verify kernel's bytes, no arithmetic) and
one flat run of the same byte count.  R small lets the 256 MiB Infinity Cache
keep part of a batch between two reads of it; R large (>= 2 GiB read between
reuses) does not, so the pair of R values shows whether MALL hits contribute.

    python tools/ceiling.py [--configs 1500,9000] [--steps 400] > out.jsonl
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import libunsod_amd as mi  # noqa: E402

CFG = {"1500": (65536, 1500, 2176, 142), "9000": (65536, 9000, 9216, 142)}
ROT = {"1500": (8, 24), "9000": (2, 8), "pareto": (3,)}


def pareto(a, lib, dev, K):
    """The Pareto batch (2^22 packed datagrams, u32 offsets, 3 rotating
    batches as the bench): the flat-run verify kernel against a read-only flat
    sweep of each batch's whole packed byte region, same submission."""
    import numpy as np
    from libunsod_amd import synth
    n = 1 << 22
    lens = synth.pareto_lengths(n)
    offs = synth.packed_offsets(lens, first_off=2)
    size = (int(offs[-1] + lens[-1]) + 256 + 255) & ~255
    alg = int(lens.sum()) + 5 * n
    bs, outs = [], []
    for r in range(ROT["pareto"][0]):
        buf = torch.empty(size, dtype=torch.uint8, device=dev)
        b = mi.PktBatch(buf, n, offs=torch.from_numpy(offs.astype(np.int64)).to(dev),
                        lens=torch.from_numpy(lens.astype(np.int32)).to(dev), max_len=int(lens.max()), packed=True,
                        offs32=True)
        mi.synth_ipv4(b, seed=0x9A7E70 + r)
        mi.ipv4_finalize(b)
        bs.append(b)
        outs.append(dict(ip=torch.empty(n, dtype=torch.uint16, device=dev),
                         l4=torch.empty(n, dtype=torch.uint16, device=dev),
                         status=torch.empty(n, dtype=torch.uint8, device=dev)))
    torch.cuda.synchronize()
    rep = mi.VerifyRepeat(bs, outs, nstreams=2)
    rep.run(100)
    bases = (C.c_void_p * len(bs))(*[b.buf.data_ptr() for b in bs])
    flat = size & ~15
    for rnd in range(a.rounds):
        rep.run(K, timed=True)
        span = rep.span()
        us = span / K
        print(json.dumps(dict(config="pareto", round=rnd, kernel=mi.verify_plan(bs[0]), us_per_launch=round(us, 3),
                              alg_TBps=round(alg / us / 1e6, 3), frac_8TBps=round(alg / us / 8e6, 4))), flush=True)
        for unroll in (4, 8, 16):
            for grid in (2048, 8192, 32768):
                sp = lib.ceil_run(bases, len(bs), size, 1, 0, 0, flat // 16, 1, unroll, grid, K, 2)
                if sp <= 0:
                    raise SystemExit(f"ceil_run failed: {sp}")
                u = sp / K
                print(json.dumps(dict(config="pareto", round=rnd, kernel="probe_flat", unroll=unroll, grid=grid,
                                      us_per_launch=round(u, 3), read_TBps=round(flat / u / 1e6, 3),
                                      alg_TBps_at_probe=round(alg / u / 1e6, 3))), flush=True)
    rep.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="1500,9000")
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--streams", type=int, default=2,
                    help="1 = every launch serialized after the previous one on one stream (the\n"
                         "single-submission case, VERDICT r2 item 4): the probe then shows what ANY\n"
                         "read kernel of these bytes pays per serialized launch")
    ap.add_argument("--grids", default="2048,4096,8192")
    ap.add_argument("--modes", default="0,1", help="ceil_run modes (tools/ceiling_probe.hip); 4 = the\n"
                    "envelope read plus 4 B per slot into a dense side array, i.e. verify's writes")
    ap.add_argument("--outputs", choices=("all", "status"), default="all")
    a = ap.parse_args()
    lib = C.CDLL(os.path.join(ROOT, "tools", "libceiling.so"))
    lib.ceil_run.restype = C.c_float
    lib.ceil_run.argtypes = [C.POINTER(C.c_void_p), C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                             C.c_uint32, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    K = a.steps
    for cfg in a.configs.split(","):
        if cfg == "pareto":
            pareto(a, lib, dev, K)
            continue
        n, L, stride, first = CFG[cfg]
        size = (first + (n - 1) * stride + L + 64 + 255) & ~255
        env_off = first & ~15
        nch = (first + L + 15) // 16 - env_off // 16
        alg = n * L + 5 * n           # verify's algorithmic bytes per launch
        env_bytes = n * nch * 16      # what the probe reads per launch
        for R in ROT[cfg]:
            bs, outs = [], []
            for r in range(R):
                buf = torch.empty(size, dtype=torch.uint8, device=dev)
                b = mi.PktBatch(buf, n, stride=stride, first_off=first, fixed_len=L)
                mi.synth_ipv4(b, seed=0x5EED5EED + 7919 * r)
                mi.ipv4_finalize(b)
                bs.append(b)
                o = dict(status=torch.empty(n, dtype=torch.uint8, device=dev))
                if a.outputs == "all":
                    o.update(ip=torch.empty(n, dtype=torch.uint16, device=dev),
                             l4=torch.empty(n, dtype=torch.uint16, device=dev))
                outs.append(o)
            torch.cuda.synchronize()
            rep = mi.VerifyRepeat(bs, outs, nstreams=a.streams)
            rep.run(2000)  # settle
            bases = (C.c_void_p * R)(*[b.buf.data_ptr() for b in bs])
            between = (R - 1) * env_bytes
            for rnd in range(a.rounds):
                rep.run(K, timed=True)
                span = rep.span()
                us = span / K
                print(json.dumps(dict(config=cfg, R=R, streams=a.streams, read_between_reuse_MB=round(between / 1e6), round=rnd,
                                      kernel=mi.verify_plan(bs[0]), outputs=a.outputs, us_per_launch=round(us, 3),
                                      alg_TBps=round(alg / us / 1e6, 3), frac_8TBps=round(alg / us / 8e6, 4),
                                      env_TBps=round(env_bytes / us / 1e6, 3))), flush=True)
                for mode in [int(m) for m in a.modes.split(",")]:
                    for unroll in (4, 8, 16):
                        for grid in [int(g) for g in a.grids.split(",")]:
                            sp = lib.ceil_run(bases, R, size, n, stride, env_off, nch, mode, unroll, grid, K,
                                              a.streams)
                            if sp <= 0:
                                raise SystemExit(f"ceil_run failed: {sp}")
                            u = sp / K
                            print(json.dumps(dict(config=cfg, R=R, streams=a.streams, round=rnd,
                                                  kernel={0: "probe_env", 1: "probe_flat", 4: "probe_env_w4dense"}.get(mode, f"mode{mode}"),
                                                  unroll=unroll, grid=grid, us_per_launch=round(u, 3),
                                                  read_TBps=round(env_bytes / u / 1e6, 3))), flush=True)
            rep.close()
            del bs, outs, rep
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
