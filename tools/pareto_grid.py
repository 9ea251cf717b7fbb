#!/usr/bin/env python3
"""Grid-cap sweep of the packed (mixed-length) verify kernel on one GPU."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import libunsod_amd as mi
from libunsod_amd import synth

dev = torch.device("cuda", 0)
n = int(os.environ.get("N", 1 << 19))
lens = synth.pareto_lengths(n)
offs = synth.packed_offsets(lens, first_off=2)
size = (int(offs[-1] + lens[-1]) + 256 + 255) & ~255
R = max(1, -(-(1 << 30) // size))
bs = []
for r in range(R):
    buf = torch.empty(size, dtype=torch.uint8, device=dev)
    b = mi.PktBatch(buf, n, offs=torch.from_numpy(offs.astype(np.int64)).to(dev),
                    lens=torch.from_numpy(lens.astype(np.int32)).to(dev), max_len=int(lens.max()), packed=True)
    mi.synth_ipv4(b, seed=r)
    mi.ipv4_finalize(b)
    bs.append(b)
outs = [dict(ip=torch.empty(n, dtype=torch.uint16, device=dev), l4=torch.empty(n, dtype=torch.uint16, device=dev),
             status=torch.empty(n, dtype=torch.uint8, device=dev)) for _ in bs]
torch.cuda.synchronize()
mi.ipv4_verify_repeat(bs, outs, 400, nstreams=2, timing="none")
for rnd in range(2):
    for cap in (0, 512, 1024, 2048, 4096, 8192):
        mi.set_shape(0, 0, cap)
        mi.ipv4_verify_repeat(bs, outs, 20, nstreams=2, timing="none")
        span = mi.ipv4_verify_repeat(bs, outs, 100, nstreams=2, timing="region")
        chk = mi.ipv4_verify(bs[0], bad_count=True)
        torch.cuda.synchronize()
        print(json.dumps(dict(round=rnd, cap=cap, n=n, us_per_launch=round(span / 100, 2),
                              GBps=round((lens.sum() + 5 * n) / (span / 100) / 1e3, 1),
                              ok=int(chk["bad"].item()) == 0)), flush=True)
mi.set_shape(0, 0, 0)
