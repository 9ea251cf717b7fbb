#!/usr/bin/env python3
"""Which extra HSA queue a resident wave sits on, and what it costs the batch.

tools/service_idle_probe.py (round 5): a one-wave resident kernel that
touches no memory cost the 1500 B batch path nothing on a HIP stream or on
the library's service queue, and 0.65x of its rate on the library's dispatch
queue -- the same kernel, another queue.  Here 8 extra queues are created in
order after the batch side's two AQL queues; a resident wave sits on queue k
(k = 0..7) for 2 s while the batch rate is measured; then again at low and
high queue priority.  One JSON line per case.

--foreign N first creates N queues the library does not know of (raw HSA,
as another component of the process would) between the batch pair and the
extras.  Every line carries the HSA queue ids (ROCr numbers the process's
queues in creation order, HIP's included) and whether (id - batch queue 0's
id) mod 4 puts the queue on a batch queue's pipe, the rule the library's
placement is meant to follow.

    python tools/queue_place_probe.py [--foreign N]
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import libunsod_amd as mi  # noqa: E402
from libunsod_amd import synth  # noqa: E402


class Agent(C.Structure):
    _fields_ = [("handle", C.c_uint64)]


def foreign_queues(n: int) -> list:
    """n HSA queues created straight through the runtime (kept alive)."""
    hsa = C.CDLL("libhsa-runtime64.so.1")
    assert hsa.hsa_init() == 0
    agents = []
    CB = C.CFUNCTYPE(C.c_int, Agent, C.c_void_p)

    def cb(a, _):
        t = C.c_uint32(0)
        hsa.hsa_agent_get_info(a, 17, C.byref(t))  # HSA_AGENT_INFO_DEVICE
        if t.value == 1:
            agents.append(Agent(a.handle))
        return 0

    keep = CB(cb)
    hsa.hsa_iterate_agents(keep, None)
    qs = []
    for _ in range(n):
        q = C.c_void_p()
        assert hsa.hsa_queue_create(agents[0], 64, 0, None, None, C.c_uint32(0xFFFFFFFF), C.c_uint32(0xFFFFFFFF),
                                    C.byref(q)) == 0
        qs.append(q)
    return qs


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--foreign", type=int, default=0)
    ap.add_argument("--priorities", default="-1,0,2")
    a = ap.parse_args()
    lib = mi.load()
    lib.mi__spin_queue_id.restype = C.c_longlong
    lib.mi__repeat_queue_id.restype = C.c_longlong
    lib.mi__repeat_queue_id.argtypes = [C.c_void_p, C.c_int]
    lib.mi__spin_queue.argtypes = [C.c_uint32, C.c_int, C.c_int]
    lib.mi__set_dropin_service.argtypes = [C.c_int]
    lib.mi__set_dropin_service(0)
    lib.mi_cksum_hsa_queues.restype = C.c_int
    n, L, stride, first = 65536, 1500, synth.STRIDE_1500, synth.IP_OFF
    bs, outs = [], []
    for r in range(23):
        buf = torch.empty(first + (n - 1) * stride + L + 64, dtype=torch.uint8, device="cuda")
        b = mi.PktBatch(buf, n, stride=stride, first_off=first, fixed_len=L)
        mi.synth_ipv4(b, seed=0x5EED + r)
        mi.ipv4_finalize(b)
        bs.append(b)
        outs.append(dict(status=torch.empty(n, dtype=torch.uint8, device="cuda")))
    torch.cuda.synchronize()
    rep = mi.VerifyRepeat(bs, outs, nstreams=2, engine="aql")
    rep.run(400)

    def rate(seconds=1.2):
        t0, passes = time.perf_counter(), 0
        while time.perf_counter() - t0 < seconds:
            rep.run(200)
            passes += 200
        return round(float(n) * L * passes / (time.perf_counter() - t0) / 2**30, 1)

    base = rate()
    ida = lib.mi__repeat_queue_id(rep._h, 0)
    idb = lib.mi__repeat_queue_id(rep._h, 1)
    fq = foreign_queues(a.foreign) if a.foreign else []
    print(json.dumps(dict(case="none", batch_gib_s=base, library_queues=lib.mi_cksum_hsa_queues(),
                          batch_queue_ids=[ida, idb], foreign_queues=len(fq))), flush=True)
    for prio in [int(x) for x in a.priorities.split(",")]:
        for k in range(8):
            assert lib.mi__spin_queue(1_600_000, k, prio) == 0
            time.sleep(0.1)
            r = rate()
            qid = lib.mi__spin_queue_id(k)
            print(json.dumps(dict(case="resident wave", queue=k, queue_id=qid, priority=prio, batch_gib_s=r,
                                  batch_vs_none=round(r / base, 3),
                                  id_rule_shared_pipe=(qid - ida) % 4 in (0, 1))), flush=True)
            time.sleep(0.5)
    rep.close()


if __name__ == "__main__":
    main()
