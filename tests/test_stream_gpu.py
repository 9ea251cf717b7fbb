"""The per-wave streaming verify kernel (k_ipv4_verify_stream, MI_CKSUM_STREAM=1)
bit-exact against the reference's golden vectors and the oracle: the golden
RX batch, the mixed-protocol demux batch, full-size 1500 / 9000 B configs with
1 % corruption, RX offload flags, multi-batch launches, and a batch of edge
cases (every address phase, IP options, runts, zero lengths, ip_len beyond
the frame, datagrams ending exactly on 1 KiB row boundaries, 65535-byte
datagrams)."""
import numpy as np
import pytest
import torch

import libunsod_amd as mi
import test_demux_gpu as DM
import test_gpu_parity as P
from libunsod_amd import synth
from oracle.pyoracle import Oracle

pytestmark = pytest.mark.gpu
ORC = Oracle("port")


@pytest.fixture(autouse=True)
def stream(monkeypatch):
    monkeypatch.setenv("MI_CKSUM_STREAM", "1")


def test_plan_names_stream():
    buf = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    assert mi.verify_plan(mi.PktBatch(buf, 100, stride=2176, first_off=142, fixed_len=1500)).startswith(
        "k_ipv4_verify_stream")


def test_verify_golden(golden):
    P.test_verify_golden(golden)


def test_demux_golden(demux_golden):
    DM.test_demux_verify_golden(demux_golden, "auto")


@pytest.mark.parametrize("name", ["1500", "9000"])
def test_full_size_config(name):
    P.test_full_size_config(name)


def test_rx_offload_flags():
    P.test_rx_offload_flags("unpacked")


def test_verify_multi_matches_single():
    P.test_verify_multi_matches_single("")


SPECS = [  # n, L, stride, first_off, hl, proto
    (3000, 1500, 2176, 142, 20, 6), (500, 1009, 1040, 7, 24, 17), (300, 2033, 2048, 15, 60, 6),
    (64, 65535, 65552, 1, 20, 6), (1000, 20, 32, 3, 20, 6), (100, 19, 32, 0, 20, 6),
    (700, 9000, 9216, 142, 40, 17), (400, 1024, 1088, 16, 20, 1), (257, 1023, 1040, 1, 28, 6)]


def _slot_batch(k, n, L, stride, first, hl, proto, rng):
    b0 = synth.build_ipv4_batch(n, L, stride=stride, first_off=first, proto=proto, hl=min(hl, max(20, L // 4 * 4)),
                                seed=k + 1)
    h = b0["buf"]
    ORC.ipv4_finalize_batch(h, n, stride=stride, first_off=first, fixed_flen=L)
    for i in rng.choice(n, max(1, n // 40), replace=False):       # corrupted bytes
        h[first + int(i) * stride + int(rng.integers(0, L))] ^= 0x10
    if L >= 20:
        for i in rng.choice(n, max(1, n // 100), replace=False):  # ip_len beyond the frame
            h[first + int(i) * stride + 2:first + int(i) * stride + 4] = [0xFF, 0xF0]
        for i in rng.choice(n, max(1, n // 100), replace=False):  # hl 12
            h[first + int(i) * stride] = 0x43
    return h, ORC.ipv4_verify_batch(h, n, stride=stride, first_off=first, fixed_flen=L)


def test_edge_slots_single_and_multi():
    """Fixed-slot batches at every address phase, IP options, runts, header-only
    datagrams, lengths on and around 1 KiB row boundaries, 65535-byte datagrams,
    corrupted / malformed headers: one launch per batch, then all of them in
    ONE multi-batch launch."""
    rng = np.random.default_rng(2024)
    hosts, wants, batches = [], [], []
    for k, (n, L, stride, first, hl, proto) in enumerate(SPECS):
        h, w = _slot_batch(k, n, L, stride, first, hl, proto, rng)
        hosts.append(h)
        wants.append(w)
        b = mi.PktBatch(P.dev_tensor(h), n, stride=stride, first_off=first, fixed_len=L)
        assert "stream" in mi.verify_plan(b), mi.verify_plan(b)
        batches.append(b)
        r = mi.ipv4_verify(b, bad_count=True)
        assert np.array_equal(P.cpu(r["ip"]), w[0]), (L, stride, first)
        assert np.array_equal(P.cpu(r["l4"]), w[1]), (L, stride, first)
        assert np.array_equal(P.cpu(r["status"]), w[2]), (L, stride, first)
        assert int(r["bad"].item()) == int((w[2] != 0).sum())
    outs = [dict(ip=torch.zeros(b.n, dtype=torch.uint16, device="cuda"),
                 l4=torch.zeros(b.n, dtype=torch.uint16, device="cuda"),
                 status=torch.full((b.n,), 0xEE, dtype=torch.uint8, device="cuda")) for b in batches]
    bad = torch.zeros(1, dtype=torch.int32, device="cuda")
    mi.ipv4_verify_multi(batches, outs, bad=bad)
    torch.cuda.synchronize()
    for w, o in zip(wants, outs):
        assert np.array_equal(P.cpu(o["ip"]), w[0]) and np.array_equal(P.cpu(o["l4"]), w[1])
        assert np.array_equal(P.cpu(o["status"]), w[2])
    assert int(bad.item()) == sum(int((w[2] != 0).sum()) for w in wants)


@pytest.mark.parametrize("blocks", [1, 7, 64])
def test_small_grids(blocks):
    """Few waves, many datagrams each (the cursors cross batches many times)."""
    mi.set_shape(0, 0, blocks)
    try:
        test_edge_slots_single_and_multi()
    finally:
        mi.set_shape(0, 0, 0)
