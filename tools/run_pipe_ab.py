#!/usr/bin/env python3
"""A/B of the flat-run verify's pipelined passes (packed_body PIPE,
MI_CKSUM_RUN_PIPE) on the bench's Pareto batch (and optionally the 64 B
slots): the same rotating batches, the same AQL submission as bench.py,
interleaved rounds, every round's outputs checked (all datagrams verify).

    python tools/run_pipe_ab.py [--configs pareto] [--steps 200] [--rounds 3]
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

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="pareto")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--waves", type=int, default=2)
    args = ap.parse_args()
    import bench
    import libunsod_amd as mi
    from libunsod_amd import shard, synth
    lib = mi.load()
    lib.mi__set_run_pipe.restype = C.c_int
    lib.mi__set_run_pipe.argtypes = [C.c_int]
    lib.mi__set_run_waves.argtypes = [C.c_int]
    lib.mi__set_packed_u.restype = C.c_int
    lib.mi__set_packed_u.argtypes = [C.c_int]
    lib.mi__set_run_occ.restype = C.c_int
    lib.mi__set_run_occ.argtypes = [C.c_int]
    lib.mi__set_run_waves(args.waves)
    mi.set_busy_wait(True)
    dev = torch.device("cuda", 0)
    for cfg in args.configs.split(","):
        wl = bench.build_workload(mi, synth, shard, cfg, 0, False, dev, 0, 1)
        L_sum, n = wl["L_sum"], wl["n"]
        alg = L_sum + 5 * n
        for rnd in range(args.rounds):
            for pu, pipe, occ in ((0, 0, 0), (4, 0, 1), (0, 0, 1), (4, 0, 0)):
                lib.mi__set_run_pipe(pipe)
                lib.mi__set_packed_u(pu)
                lib.mi__set_run_occ(occ)
                plan = bench.repeat_plan(wl["batches"][0])
                rep = mi.VerifyRepeat(wl["batches"], wl["outs"], nstreams=2, engine="aql")
                rep.run(200, timed=True)
                t_end = time.perf_counter() + 0.3
                while time.perf_counter() < t_end:
                    rep.run(200, timed=True)
                bench.poison_outputs(wl["outs"])
                torch.cuda.synchronize()
                rep.run(args.steps, timed=True)
                torch.cuda.synchronize()
                span = rep.span()
                rep.close()
                chk = bench.check_timed_outputs(wl["outs"], args.steps)
                us = span / args.steps
                print(json.dumps(dict(config=cfg, round=rnd, pipe=pipe, occ=occ, packed_u=pu or "auto", plan=plan, us_per_launch=round(us, 2),
                                      frac=round(alg / us / 1e3 / bench.HBM_PEAK_GBS, 4),
                                      outputs_checked=chk["checked"])), flush=True)
        lib.mi__set_run_pipe(0)
        lib.mi__set_packed_u(0)
        lib.mi__set_run_occ(0)
        del wl
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
