#!/usr/bin/env python3
"""Zero-copy host path (mi_cksum_ipv4_verify_host on a registered batch): rate
per lane-group shape / grid cap, one JSON line each.  1500 B slots by default.

    python tools/host_sweep.py [--L 1500] [--n 65536]
"""
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

GIB = float(1 << 30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=1500)
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    L, n = args.L, args.n
    stride = 2176 if L <= 2034 else ((L + 142 + 255) // 256) * 256
    first = 142
    buf = torch.empty(first + n * stride + 64, dtype=torch.uint8, device="cuda")
    b = mi.PktBatch(buf, n, stride=stride, first_off=first, fixed_len=L)
    mi.synth_ipv4(b)
    mi.ipv4_finalize(b)
    torch.cuda.synchronize()
    raw = buf.cpu().numpy()
    host = np.zeros(raw.size + 8192, np.uint8)
    s = (-host.ctypes.data) % 4096
    h = host[s:s + raw.size]
    h[:] = raw
    lay = dict(stride=stride, first_off=first, fixed_len=L)
    mi.host_register(h)
    shapes = [(0, 0, 0), (16, 6, 0), (16, 2, 0), (16, 4, 0), (8, 4, 0), (8, 12, 0), (32, 4, 0), (64, 4, 0),
              (16, 6, 256), (16, 6, 1024), (16, 6, 4096), (16, 6, 16384), (16, 2, 16384), (64, 2, 8192)]
    for G, U, B in shapes:
        try:
            mi.set_shape(G, U, B)
        except Exception as e:  # noqa: BLE001
            print(json.dumps(dict(shape=f"{G}x{U}", blocks=B, error=str(e))), flush=True)
            continue
        for staged in (False, True):
            mi.ipv4_verify_host(h, n, staged=staged, **lay)
            t0 = time.perf_counter()
            for _ in range(args.iters):
                _, _, st, bad = mi.ipv4_verify_host(h, n, staged=staged, **lay)
            dt = (time.perf_counter() - t0) / args.iters
            assert bad == 0
            print(json.dumps(dict(L=L, shape=f"{G}x{U}", blocks=B, staged=staged,
                                  GiBps=round(n * L / dt / GIB, 2), ms=round(dt * 1e3, 3))), flush=True)
    mi.set_shape(0, 0, 0)
    mi.host_unregister(h)


if __name__ == "__main__":
    main()
