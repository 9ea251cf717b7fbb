"""MI_BATCH_DEMUX on the GPU (the small-header callers):
each datagram's L4 checksum taken the way ip_input's protocol switch hands it
on -- TCP / UDP (pseudo header, UDP length and no-checksum rules), ICMP, IGMP,
CARP (plain in_cksum), fragments and other protocols none -- bit-exact against
the reference's golden vectors (tests/golden/demux_golden.npz) and the oracle,
through every verify kernel and the TX finalize.
"""
import numpy as np
import pytest
import torch

from conftest import aligned
from demux_cases import build_demux_batch, to_rx
from oracle.pyoracle import Oracle

import libunsod_amd as mi

pytestmark = pytest.mark.gpu
ORC = Oracle("port")


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def batch(buf, offs, flen, **kw):
    return mi.PktBatch(buf, len(offs), offs=dev(offs.astype(np.int64)), lens=dev(flen.astype(np.int32)),
                       demux=True, **kw)


# lane-group kernel (automatic, forced small / wide shapes) and the flat-run kernel
KERNELS = ["auto", "g4x2", "g16x6", "g64x4", "packed"]


def _run_verify(kernel, buf, offs, flen):
    if kernel.startswith("g"):
        G, U = (int(x) for x in kernel[1:].split("x"))
        mi.set_shape(G, U, 61)
    try:
        b = batch(buf, offs, flen, packed=kernel == "packed")
        r = mi.ipv4_verify(b, bad_count=True)
        return (r["ip"].cpu().numpy(), r["l4"].cpu().numpy(), r["status"].cpu().numpy(),
                int(r["bad"].item()), mi.verify_plan(b))
    finally:
        mi.set_shape(0, 0, 0)


@pytest.mark.parametrize("kernel", KERNELS)
def test_demux_verify_golden(demux_golden, kernel):
    g = demux_golden
    ip, l4, st, bad, plan = _run_verify(kernel, dev(g["ver_in"]), g["offs"], g["flen"])
    if kernel == "packed":
        assert "packed" in plan or "run_dma" in plan  # a flat-run kernel
    assert np.array_equal(ip, g["ip"]), plan
    assert np.array_equal(l4, g["l4"]), plan
    assert np.array_equal(st, g["st"]), plan
    assert bad == int(((g["st"] & ~np.uint8(8)) != 0).sum())


@pytest.mark.parametrize("shape", [None, (4, 2), (16, 6), (64, 4), "packed"])
def test_demux_finalize_golden(demux_golden, shape):
    """Lane-group shapes and the flat-run finalize (packed hint)."""
    g = demux_golden
    if shape and shape != "packed":
        mi.set_shape(shape[0], shape[1], 61)
    try:
        buf = dev(g["fin_in"])
        mi.ipv4_finalize(batch(buf, g["offs"], g["flen"], packed=shape == "packed"))
        got = buf.cpu().numpy()
    finally:
        mi.set_shape(0, 0, 0)
    diff = np.nonzero(got != g["fin_out"])[0]
    assert diff.size == 0, f"{diff.size} bytes differ, first at {diff[:8]}"


def test_demux_off_is_unchanged(demux_golden):
    """Without the flag verify keeps the plain in_cksum_pseudo_header contract
    for every protocol (no L4_NONE bit ever)."""
    g = demux_golden
    n = len(g["offs"])
    _, h = aligned(g["ver_in"])
    want = ORC.ipv4_verify_batch(h, n, offs=g["offs"], flen=g["flen"])
    b = mi.PktBatch(dev(g["ver_in"]), n, offs=dev(g["offs"].astype(np.int64)), lens=dev(g["flen"].astype(np.int32)))
    r = mi.ipv4_verify(b)
    for k, w in zip(("ip", "l4", "status"), want):
        assert np.array_equal(r[k].cpu().numpy(), w), k
    assert not (want[2] & 8).any()


@pytest.mark.parametrize("kernel", ["auto", "packed"])
def test_demux_large_mixed(kernel):
    """20 000 mixed-protocol datagrams up to 9000 B: finalize on the GPU ==
    oracle finalize (bytes), then verify of the received copy == oracle."""
    d = build_demux_batch(20000, seed=77, max_len=9000)
    n = len(d["offs"])
    _, h = aligned(d["buf"])
    ORC.ipv4_finalize_batch(h, n, offs=d["offs"], flen=d["flen"], demux=True, nthreads=8)
    buf = dev(d["buf"])
    mi.ipv4_finalize(batch(buf, d["offs"], d["flen"], packed=kernel == "packed"))
    assert np.array_equal(buf.cpu().numpy(), h)
    rx = to_rx(h, d, seed=78)
    _, hr = aligned(rx)
    want = ORC.ipv4_verify_batch(hr, n, offs=d["offs"], flen=d["flen"], demux=True, nthreads=8)
    ip, l4, st, bad, plan = _run_verify(kernel, dev(rx), d["offs"], d["flen"])
    assert np.array_equal(ip, want[0]), plan
    assert np.array_equal(l4, want[1]), plan
    assert np.array_equal(st, want[2]), plan
    assert (st == 0).sum() > n // 2
