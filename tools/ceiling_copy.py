#!/usr/bin/env python3
"""Copy ceiling for the fused TX copy: what does a kernel
that only MOVES the bytes mi_cksum_tx_copy moves get -- frames read from a
source blob and written into rte_mbuf slots (stride 2176, data at +128), no
gather arithmetic, no sums -- submitted the way tools/bench_tx.py submits
(back-to-back launches over rotating batches, 2 streams)?  One JSON line per
(source misalignment, unroll); the fused kernel's number on the same geometry
is tools/bench_tx.py's.

    hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/ceiling_probe.hip -o tools/libceiling.so
    python tools/ceiling_copy.py
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--frame", type=int, default=1514)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--grid", default="8192")
    ap.add_argument("--unroll", default="4", help="comma list of 2, 4, 8")
    ap.add_argument("--saux", default="0,1,2,3", help="comma list of store policies")
    ap.add_argument("--geom", default="slots,dense")
    ap.add_argument("--soff", default="0,6")
    ap.add_argument("--torch-copy", dest="torch_copy", default="torch", help="'torch': also time torch copy_; '' skips")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    lib = C.CDLL(os.path.join(ROOT, "tools", "libceiling.so"))
    lib.ceil_copy.restype = C.c_float
    lib.ceil_copy.argtypes = [C.c_void_p, C.c_void_p, C.c_int] + [C.c_uint32] * 8 + [C.c_int] * 5
    n, fr = a.n, a.frame
    nch = (fr + 15) // 16
    sstride, dstride, doff = 1600, 2176, 128  # source: frames ~1.6 KB apart in the socket blob
    sbytes = (n * sstride + 4096 + 255) & ~255
    dbytes = (doff + n * dstride + 255) & ~255
    per = sbytes + dbytes
    R = max(2, -(-(1 << 30) // per))
    srcs = [torch.randint(0, 255, (sbytes,), dtype=torch.uint8, device="cuda") for _ in range(R)]
    dsts = [torch.empty(dbytes, dtype=torch.uint8, device="cuda") for _ in range(R)]
    sp = (C.c_void_p * R)(*[t.data_ptr() for t in srcs])
    dp = (C.c_void_p * R)(*[t.data_ptr() for t in dsts])
    alg = n * (2 * fr + 1)
    geoms = {"slots": (sstride, dstride, doff), "dense": (nch * 16, nch * 16, 0)}
    ints = lambda x: [int(v) for v in x.split(",")]  # noqa: E731
    for geom in a.geom.split(","):
        ss, ds_, do = geoms[geom]
        for soff in ints(a.soff):
            for saux in ints(a.saux):
                for unroll in ints(a.unroll):
                    for grid in [int(g) for g in a.grid.split(",")]:
                        args = (sp, dp, R, sbytes, dbytes, n, ss, soff, ds_, do, nch, unroll, grid)
                        lib.ceil_copy(*args, 100, 2, saux)
                        us = lib.ceil_copy(*args, a.steps, 2, saux) / a.steps
                        print(json.dumps(dict(probe="copy ceiling", geometry=geom, frames=n, frame_len=fr,
                                              src_misalign=soff, store_aux=saux, unroll=unroll, grid=grid, R=R,
                                              us_per_launch=round(us, 3), frac_of_8TBps=round(alg / us / 8e6, 4))),
                              flush=True)

    if "torch" in a.torch_copy:
        # the runtime's own device-to-device copy of the same byte count
        # (n frames back to back, no slots): torch copy_ over rotating buffers
        # alternating over two streams, span from events on those streams
        nb = n * fr
        tsrc = [t[:nb] for t in srcs]
        tdst = [t[:nb] for t in dsts]
        streams = [torch.cuda.Stream() for _ in range(2)]

        def run(k):
            for j in range(k):
                with torch.cuda.stream(streams[j % 2]):
                    tdst[j % R].copy_(tsrc[j % R])
        run(100)
        torch.cuda.synchronize()
        e0 = [torch.cuda.Event(enable_timing=True) for _ in streams]
        e1 = [torch.cuda.Event(enable_timing=True) for _ in streams]
        g = torch.cuda.Event()
        g.record(streams[0])
        streams[1].wait_event(g)
        for e, s_ in zip(e0, streams):
            e.record(s_)
        run(a.steps)
        for e, s_ in zip(e1, streams):
            e.record(s_)
        torch.cuda.synchronize()
        us = max(e0[0].elapsed_time(e) for e in e1) * 1e3 / a.steps
        print(json.dumps(dict(probe="torch copy_ (dense D2D)", bytes=nb, R=R, us_per_launch=round(us, 3),
                              frac_of_8TBps=round(n * (2 * fr + 1) / us / 8e6, 4))), flush=True)


if __name__ == "__main__":
    main()
