#!/usr/bin/env python3
"""What TX finalize's in-place stores cost by themselves (tools/libceiling.so,
no checksum code): the bench's slot read pattern alone, plus a 4-byte store
into each slot's header chunk, plus the slot's first 64 B block stored back
whole, plus 4 bytes per slot into a dense side array -- on 1 and 2 streams,
R rotating batches (>= 2 GiB read between reuses).

    python tools/ceiling_writes.py > out.jsonl
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

# "packed288": a packed stand-in for the Pareto batch (4 Mi datagrams, ~288 B apart)
CFG = {"1500": (65536, 1500, 2176, 142), "9000": (65536, 9000, 9216, 142), "packed288": (1 << 22, 284, 288, 2)}
MODES = {0: "read only", 2: "read + 4 B in place per slot", 3: "read + 64 B block in place per slot",
         4: "read + 4 B per slot to a side array", 5: "read + 4 B in place per slot, nt store",
         6: "read + 64 B block in place per slot, nt store", 7: "4 B in place per slot, write only"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="1500,9000")
    ap.add_argument("--modes", default=",".join(str(m) for m in MODES))
    ap.add_argument("--streams", default="2,1")
    a = ap.parse_args()
    lib = C.CDLL(os.path.join(ROOT, "tools", "libceiling.so"))
    lib.ceil_run.restype = C.c_float
    lib.ceil_run.argtypes = [C.POINTER(C.c_void_p), C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                             C.c_uint32, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
    dev = torch.device("cuda", 0)
    K = 400
    for cfg in a.configs.split(","):
        n, L, stride, first = CFG[cfg]
        size = (first + (n - 1) * stride + L + 64 + 255) & ~255
        env_off = first & ~15
        nch = (first + L + 15) // 16 - env_off // 16
        R = 1 + -(-(2 << 30) // (n * nch * 16))
        bufs = [torch.randint(0, 255, (size,), dtype=torch.uint8, device=dev) for _ in range(R)]
        bases = (C.c_void_p * R)(*[b.data_ptr() for b in bufs])
        torch.cuda.synchronize()
        for ns in [int(x) for x in a.streams.split(",")]:
            for mode in [int(x) for x in a.modes.split(",")]:
                lib.ceil_run(bases, R, size, n, stride, env_off, nch, mode, 4, 8192, 200, ns)  # warm
                sp = lib.ceil_run(bases, R, size, n, stride, env_off, nch, mode, 4, 8192, K, ns)
                if sp <= 0:
                    raise SystemExit(f"ceil_run failed: {sp}")
                us = sp / K
                print(json.dumps(dict(config=cfg, streams=ns, mode=MODES[mode], R=R, us_per_launch=round(us, 3),
                                      read_TBps=round(n * nch * 16 / us / 1e6, 3))), flush=True)
        del bufs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
