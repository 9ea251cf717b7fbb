#!/usr/bin/env python3
"""Interleaved A/B of the fused TX copy kernels on the bench's TX workload
(bench.py config_tx: 65536 x 1514 B frames, socket-layout chains, 2176 B
rte_mbuf slots) and on single-segment frames: k_tx_copy 8x2 with the loads
after / before the stores (MI_CKSUM_TX_EARLY=0 / 1) and the LDS-staged
gather k_tx_lds (MI_CKSUM_TX_KERNEL=lds, MI_CKSUM_TX_LDS=UxR).  HIP launches
over two streams, span from events on the launch streams; each variant's
output checked byte for byte against the first variant's.

    python tools/tx_ab.py [--steps 200] [--rounds 3] [--variants el0,el1,lds2x3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

VARIANTS = {
    "el0": dict(MI_CKSUM_TX_KERNEL="pair", MI_CKSUM_TX_EARLY="0"),
    "el1": dict(MI_CKSUM_TX_KERNEL="pair", MI_CKSUM_TX_EARLY="1"),
    "lds2x2": dict(MI_CKSUM_TX_KERNEL="lds", MI_CKSUM_TX_LDS="2x2"),
    "lds2x3": dict(MI_CKSUM_TX_KERNEL="lds", MI_CKSUM_TX_LDS="2x3"),
    "lds2x4": dict(MI_CKSUM_TX_KERNEL="lds", MI_CKSUM_TX_LDS="2x4"),
    "lds1x4": dict(MI_CKSUM_TX_KERNEL="lds", MI_CKSUM_TX_LDS="1x4"),
    "lds1x3": dict(MI_CKSUM_TX_KERNEL="lds", MI_CKSUM_TX_LDS="1x3"),  # 5 waves per SIMD
    "lds2x2c": dict(MI_CKSUM_TX_KERNEL="lds", MI_CKSUM_TX_LDS="2x2c"),  # cut cache
    "lds2x2g16": dict(MI_CKSUM_TX_KERNEL="lds", MI_CKSUM_TX_LDS="2x2g16"),  # 16 lanes per frame
    # the 2x2 ring with a smaller grid (mi_cksum_set_shape(0, 0, cap): cap
    # 4-wave workgroups' worth, i.e. 4 cap one-wave workgroups; 2048 = default)
    "lds2x2c1024": dict(MI_CKSUM_TX_KERNEL="lds", MI_CKSUM_TX_LDS="2x2", _cap=1024),
    "lds2x2c1536": dict(MI_CKSUM_TX_KERNEL="lds", MI_CKSUM_TX_LDS="2x2", _cap=1536),
    # the wave-per-frame kernel (k_tx_wave<2>, 4 waves per workgroup) at larger
    # grids: 16384 workgroups = one frame per wave, one-shot
    "wave": dict(MI_CKSUM_TX_KERNEL="wave"),
    "wave4k": dict(MI_CKSUM_TX_KERNEL="wave", _cap=4096),
    "wave8k": dict(MI_CKSUM_TX_KERNEL="wave", _cap=8192),
    "wave16k": dict(MI_CKSUM_TX_KERNEL="wave", _cap=16384),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="el0,el1,lds2x2,lds2x3,lds2x4,lds1x4")
    ap.add_argument("--layouts", default="socket,single")
    args = ap.parse_args()
    import libunsod_amd as mi
    from libunsod_amd import synth
    dev = torch.device("cuda", 0)
    n, L, stride, first, l3 = 65536, 1500, 2176, 128, 14
    frame = L + l3
    alg = n * (2 * frame + 1)
    for layout in args.layouts.split(","):
        d = synth.build_tx_chains(n, L, layout=layout, seed=0x7E57, l3_off=l3)
        R = 1 + -(-(2 << 30) // (2 * n * frame))
        src_h = torch.from_numpy(d["src"])
        batches = []
        for _ in range(R):
            src = src_h.to(dev)
            dst = torch.zeros(first + n * stride + 64, dtype=torch.uint8, device=dev)
            tb = mi.TxBatch(src, d["seg_off"], d["seg_len"], d["pkt_seg"], d["pkt_len"], dst, dst_stride=stride,
                            dst_first=first, room=stride - first, l3_off=l3, max_len=frame)
            batches.append((tb, torch.empty(n, dtype=torch.uint8, device=dev)))
        streams = [torch.cuda.Stream(dev) for _ in range(2)]
        ref = None
        for rnd in range(args.rounds):
            for v in args.variants.split(","):
                spec = dict(VARIANTS[v])
                mi.set_shape(0, 0, spec.pop("_cap", 0))
                os.environ.update(spec)

                def run(k):
                    for j in range(k):
                        tb, st = batches[j % R]
                        mi.tx_copy(tb, status=st, stream=streams[j % 2])
                run(20)
                torch.cuda.synchronize()
                t_end = time.perf_counter() + 0.2
                while time.perf_counter() < t_end:
                    run(40)
                    torch.cuda.synchronize()
                batches[0][0].dst.zero_()
                torch.cuda.synchronize()
                e0 = [torch.cuda.Event(enable_timing=True) for _ in streams]
                e1 = [torch.cuda.Event(enable_timing=True) for _ in streams]
                g = torch.cuda.Event()
                g.record(streams[0])
                streams[1].wait_event(g)
                for e, s_ in zip(e0, streams):
                    e.record(s_)
                run(args.steps)
                for e, s_ in zip(e1, streams):
                    e.record(s_)
                torch.cuda.synchronize()
                us = max(e0[0].elapsed_time(e) for e in e1) * 1e3 / args.steps
                out = batches[0][0].dst.cpu()
                st_ok = bool((batches[0][1] == 0).all())
                if ref is None:
                    ref = out
                same = bool(torch.equal(out, ref))
                print(json.dumps(dict(layout=layout, round=rnd, variant=v, us_per_launch=round(us, 2),
                                      frac=round(alg / us / 1e3 / 8000.0, 4), status_ok=st_ok,
                                      bytes_equal_first=same)), flush=True)
        del batches
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
