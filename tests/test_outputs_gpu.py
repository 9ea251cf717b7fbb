"""Status-only RX verify (ip = l4 = NULL: the drop decision alone) against the
full call, per kernel family: the lane-group kernel (1500 B slots), the
64-byte-slot kernel (minimum frames), the flat-run kernel (packed Pareto) and
its LDS-DMA form, through a direct call and through the AQL engine.  1 % of the
datagrams are corrupted so the status bytes carry verdicts; the bad counter
must agree too.  (bench.py --outputs status times this call.)
"""
import numpy as np
import pytest
import torch

import libunsod_amd as mi
from libunsod_amd import synth

pytestmark = pytest.mark.gpu


def _batch(kind):
    if kind == "pareto":
        n = 1 << 16
        lens = synth.pareto_lengths(n, seed=5)
        offs = synth.packed_offsets(lens, first_off=2)
        buf = torch.zeros(int(offs[-1] + lens[-1]) + 256, dtype=torch.uint8, device="cuda")
        b = mi.PktBatch(buf, n, offs=torch.from_numpy(offs.astype(np.int64)).cuda(),
                        lens=torch.from_numpy(lens.astype(np.int32)).cuda(), max_len=int(lens.max()), packed=True,
                        offs32=True)
        starts, sizes = offs.astype(np.int64), lens.astype(np.int64)
    else:
        n, L, stride, first = {"1500": (8192, 1500, synth.STRIDE_1500, synth.IP_OFF),
                               "64": (1 << 16, synth.MIN_FRAME_IP_LEN, synth.STRIDE_64, synth.ETH_HLEN)}[kind]
        buf = torch.zeros(first + (n - 1) * stride + L + 64, dtype=torch.uint8, device="cuda")
        b = mi.PktBatch(buf, n, stride=stride, first_off=first, fixed_len=L)
        starts = first + np.arange(n, dtype=np.int64) * stride
        sizes = np.full(n, L, dtype=np.int64)
    mi.synth_ipv4(b, seed=77)
    mi.ipv4_finalize(b)
    torch.cuda.synchronize()
    rng = np.random.default_rng(3)
    hit = np.sort(rng.choice(n, n // 100, replace=False))
    pos = starts[hit] + rng.integers(0, 1 << 30, hit.size) % sizes[hit]
    host = b.buf.cpu().numpy()
    host[pos] ^= (1 << rng.integers(0, 8, hit.size)).astype(np.uint8)
    b.buf.copy_(torch.from_numpy(host))
    return b, hit


@pytest.mark.parametrize("kind,dma", [("1500", None), ("64", None), ("pareto", None), ("pareto", (2, 4))])
def test_status_only_matches_full(kind, dma):
    if dma:
        mi.set_run_kernel(*dma)
    try:
        b, hit = _batch(kind)
        full = mi.ipv4_verify(b, bad_count=True)
        only = mi.ipv4_verify(b, ip=False, l4=False, bad_count=True)
        assert "ip" not in only and "l4" not in only
        st = full["status"].cpu().numpy()
        assert np.array_equal(np.nonzero(st)[0], hit)
        assert np.array_equal(only["status"].cpu().numpy(), st), mi.verify_plan(b)
        assert int(only["bad"].item()) == int(full["bad"].item()) == hit.size
        # the AQL engine with status-only outputs
        o = dict(status=torch.empty(b.n, dtype=torch.uint8, device="cuda"))
        rep = mi.VerifyRepeat([b], [o], nstreams=1, engine="aql")
        try:
            rep.run(2)
        finally:
            rep.close()
        assert np.array_equal(o["status"].cpu().numpy(), st)
    finally:
        mi.set_run_kernel(0, 0)
