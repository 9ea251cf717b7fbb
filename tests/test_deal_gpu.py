"""Dealt units (round 5, cksum_kernels.hip verify_dyn_body): the prepared
submissions run the lane-group verify as one resident generation of waves
that deal themselves units from per-workgroup-group counters.  Every
datagram must still be verified exactly once -- bit-exact against the
oracle -- through HIP launches and the AQL engine, one and two streams /
queues, and run after run: each launch must leave its counters at zero for
the next pass on the same stream (a counter left dirty would skip or repeat
units, which the poisoned outputs below would show)."""
import ctypes as C

import numpy as np
import pytest
import torch

import libunsod_amd as mi
from libunsod_amd import synth
from libunsod_amd._lib import load
from oracle.pyoracle import Oracle

pytestmark = pytest.mark.gpu
ORC = Oracle("port")


def _lib():
    lib = load()
    lib.mi__set_deal.restype = C.c_int
    lib.mi__set_deal.argtypes = [C.c_int]
    return lib


def _batch(L, n, stride, first, seed):
    buf = torch.zeros(first + (n - 1) * stride + L + 64, dtype=torch.uint8, device="cuda")
    b = mi.PktBatch(buf, n, stride=stride, first_off=first, fixed_len=L)
    mi.synth_ipv4(b, seed=seed)
    mi.ipv4_finalize(b)
    torch.cuda.synchronize()
    host = buf.cpu().numpy()
    rng = np.random.default_rng(seed)
    hit = rng.choice(n, n // 97, replace=False)
    host[first + hit * stride + rng.integers(0, L, hit.size)] ^= 0x21
    buf.copy_(torch.from_numpy(host))
    want = ORC.ipv4_verify_batch(host, n, stride=stride, first_off=first, fixed_flen=L)
    return b, want


@pytest.mark.parametrize("cfg", ["1500", "9000"])
@pytest.mark.parametrize("engine,nst", [("hip", 1), ("hip", 2), ("aql", 1), ("aql", 2)])
def test_dealt_units_bit_exact_run_after_run(cfg, engine, nst):
    lib = _lib()
    was = lib.mi__set_deal(1)
    try:
        L, n, stride, first = {"1500": (1500, 65536, synth.STRIDE_1500, synth.IP_OFF),
                               "9000": (9000, 32768, 9216, synth.IP_OFF)}[cfg]
        b0, want0 = _batch(L, n, stride, first, 5)
        b1, want1 = _batch(L, n, stride, first, 6)
        outs = [dict(ip=torch.empty(n, dtype=torch.uint16, device="cuda"),
                     l4=torch.empty(n, dtype=torch.uint16, device="cuda"),
                     status=torch.empty(n, dtype=torch.uint8, device="cuda")) for _ in range(2)]
        rep = mi.VerifyRepeat([b0, b1], outs, nstreams=nst, engine=engine)
        try:
            for steps in (1, 2, 5, 2):
                for o in outs:
                    o["ip"].fill_(0x7777)
                    o["l4"].fill_(0x7777)
                    o["status"].fill_(0xEE)
                torch.cuda.synchronize()
                rep.run(steps)
                torch.cuda.synchronize()
                for k, (o, w) in enumerate(zip(outs, (want0, want1))):
                    if steps == 1 and k == 1 and rep is not None:
                        continue  # (a 1-step run covers one batch; the rotation continues)
                    assert np.array_equal(o["ip"].cpu().numpy(), w[0]), (cfg, engine, nst, steps, k)
                    assert np.array_equal(o["l4"].cpu().numpy(), w[1]), (cfg, engine, nst, steps, k)
                    assert np.array_equal(o["status"].cpu().numpy(), w[2]), (cfg, engine, nst, steps, k)
        finally:
            rep.close()
    finally:
        lib.mi__set_deal(was)


def test_dealt_units_isolated_passes():
    """mi_cksum_ipv4_verify_repeat per-pass timing (the bench's isolated
    launch): dealt and static grids give the same outputs."""
    lib = _lib()
    n = 65536
    b, want = _batch(1500, n, synth.STRIDE_1500, synth.IP_OFF, 9)
    res = {}
    for on in (1, 0):
        was = lib.mi__set_deal(on)
        try:
            o = dict(ip=torch.empty(n, dtype=torch.uint16, device="cuda"),
                     l4=torch.empty(n, dtype=torch.uint16, device="cuda"),
                     status=torch.empty(n, dtype=torch.uint8, device="cuda"))
            us, span = mi.ipv4_verify_repeat([b], [o], 6, nstreams=1, timing="pass")
            res[on] = float(np.median(us))
            assert np.array_equal(o["ip"].cpu().numpy(), want[0])
            assert np.array_equal(o["l4"].cpu().numpy(), want[1])
            assert np.array_equal(o["status"].cpu().numpy(), want[2])
        finally:
            lib.mi__set_deal(was)
    print("isolated 1500 B launch, median us: dealt %.2f static %.2f" % (res[1], res[0]))
