"""TX copy + checksum offload on the GPU (mi_cksum_tx_copy) vs the oracle:
the destination slots byte for byte (including bytes no frame may touch) and
the per-frame status, on every edge case, every TX shape, and the full-size
65536 x 1514 B batch (then RX-verified on the GPU)."""
import numpy as np
import pytest
import torch

import libunsod_amd as mi
from oracle.pyoracle import Oracle
from tx_cases import edge_cases, make_case, run_oracle

pytestmark = pytest.mark.gpu
ORC = Oracle("port")


def run_gpu(c):
    src = torch.from_numpy(c["src"]).cuda()
    dst = torch.from_numpy(c["dst"].copy()).cuda()
    tb = mi.TxBatch(src, c["seg_off"], c["seg_len"], c["pkt_seg"], c["pkt_len"], dst, dst_stride=c["stride"],
                    dst_first=c["dst_first"], room=c["room"], l3_off=c["l3"], csum_flags=c["flags"],
                    csum_data=c["data"], max_len=int(c["pkt_len"].max()))
    st = mi.tx_copy(tb)
    torch.cuda.synchronize()
    return dst.cpu().numpy(), st.cpu().numpy()


CASES = edge_cases(ORC)


@pytest.mark.parametrize("name", [n for n, _ in CASES])
def test_tx_copy_matches_oracle(name):
    c = dict(CASES)[name]
    want_dst, want_st = run_oracle(ORC, c)
    got_dst, got_st = run_gpu(c)
    assert np.array_equal(got_st, want_st), (np.nonzero(got_st != want_st)[0][:8], got_st[:16], want_st[:16])
    bad = np.nonzero(got_dst != want_dst)[0]
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:8]} (frame {(bad[0] - c['dst_first']) // c['stride']})"


@pytest.mark.parametrize("shape", [(8, 2), (8, 4), (8, 8), (16, 2), (16, 4), (16, 6), (16, 8), (32, 2), (32, 4), (64, 2), (64, 4)])
def test_tx_every_shape(shape):
    try:
        mi.set_shape(*shape)
        for name in ("socket-1514", "random-udp-opts", "many-segments", "single-9014"):
            c = dict(CASES)[name]
            want_dst, want_st = run_oracle(ORC, c)
            got_dst, got_st = run_gpu(c)
            assert np.array_equal(got_st, want_st), (shape, name)
            assert np.array_equal(got_dst, want_dst), (shape, name)
    finally:
        mi.set_shape(0, 0, 0)


@pytest.mark.parametrize("shape", ["8x2", "16x4", "64x2"])
def test_tx_every_case_per_shape(shape, monkeypatch):
    """Every edge case (padding, far headers, ragged counts included) through
    a narrow, a middle and a whole-wave group shape (MI_CKSUM_TX_SHAPE)."""
    monkeypatch.setenv("MI_CKSUM_TX_SHAPE", shape)
    for name, c in CASES:
        want_dst, want_st = run_oracle(ORC, c)
        got_dst, got_st = run_gpu(c)
        assert np.array_equal(got_st, want_st), (shape, name, np.nonzero(got_st != want_st)[0][:8])
        bad = np.nonzero(got_dst != want_dst)[0]
        assert bad.size == 0, (shape, name, bad.size, bad[:8])


def test_tx_full_size_then_rx_verify():
    """65536 x 1514 B frames in socket-buffer chains -> rte_mbuf slots; the
    slots then verify to 0/0 on the GPU RX path."""
    n = 65536
    c = make_case(n, 1500, layout="socket", seed=31)
    want_dst, want_st = run_oracle(ORC, c)
    got_dst, got_st = run_gpu(c)
    assert not want_st.any() and np.array_equal(got_st, want_st)
    assert np.array_equal(got_dst, want_dst)
    d = torch.from_numpy(got_dst).cuda()
    pb = mi.PktBatch(d, n, stride=c["stride"], first_off=c["dst_first"] + c["l3"], fixed_len=1500)
    r = mi.ipv4_verify(pb, bad_count=True)
    assert int(r["bad"].item()) == 0


def _host_buf(a: np.ndarray) -> np.ndarray:
    """a copy of ``a`` in a 4 KiB-aligned, whole-page numpy buffer (registrable)."""
    n = (a.size + 4095) & ~4095
    out = mi.page_buffer(n)  # registrable: pages of its own
    out[:a.size] = a
    return out


@pytest.mark.parametrize("mode", ["zero_copy", "staged"])
def test_tx_copy_host_matches_oracle(mode):
    """mi_cksum_tx_copy_host -- the chains and the rte_mbuf slots in host
    memory, as if_dpdk_transmit has them (uinet_if_dpdk.c:583-597): every edge
    case, zero-copy (both buffers registered, the kernel reads and writes them
    over PCIe) and staged, byte for byte against the oracle, bytes no frame
    may touch included."""
    for name, c in CASES:
        want_dst, want_st = run_oracle(ORC, c)
        src, dst = _host_buf(c["src"]), _host_buf(c["dst"])
        if mode == "zero_copy":
            mi.host_register(src)
            mi.host_register(dst)
        try:
            st = mi.tx_copy_host(src, c["seg_off"], c["seg_len"], c["pkt_seg"], c["pkt_len"], dst,
                                 dst_stride=c["stride"], dst_first=c["dst_first"], room=c["room"], l3_off=c["l3"],
                                 csum_flags=c["flags"], csum_data=c["data"], max_len=int(c["pkt_len"].max()),
                                 staged=mode == "staged")
        finally:
            if mode == "zero_copy":
                mi.host_unregister(src)
                mi.host_unregister(dst)
        got = dst[:c["dst"].size]
        assert np.array_equal(st, want_st), (name, np.nonzero(st != want_st)[0][:8])
        bad = np.nonzero(got != want_dst)[0]
        assert bad.size == 0, (name, bad.size, bad[:8])
        assert np.array_equal(dst[c["dst"].size:], np.zeros(dst.size - c["dst"].size, np.uint8)), name


@pytest.mark.parametrize("kernel", ["wave", "pair", "lds", "lds1x3", "lds2x2c", "lds2x2g16"])
def test_tx_kernel_every_case(kernel, monkeypatch):
    """The wave-per-frame TX kernel (k_tx_wave, MI_CKSUM_TX_KERNEL=wave), the
    lane-group gather through VGPRs (k_tx_copy, =pair) and through an LDS ring
    (k_tx_lds, =lds, the default) on every
    edge case (socket / single / random / 40-segment chains, padding, far
    headers, short / nobufs / malformed frames, flags and data, UDP 0 ->
    0xffff), byte for byte against the oracle."""
    monkeypatch.setenv("MI_CKSUM_TX_KERNEL", kernel[:3] if kernel.startswith("lds") else kernel)
    if kernel in ("lds1x3", "lds2x2c", "lds2x2g16"):
        monkeypatch.setenv("MI_CKSUM_TX_LDS", kernel[3:])
    for name, c in CASES:
        want_dst, want_st = run_oracle(ORC, c)
        got_dst, got_st = run_gpu(c)
        assert np.array_equal(got_st, want_st), (kernel, name, np.nonzero(got_st != want_st)[0][:8])
        bad = np.nonzero(got_dst != want_dst)[0]
        assert bad.size == 0, (kernel, name, bad.size, bad[:8])


@pytest.mark.parametrize("kernel", ["wave", "pair", "lds"])
def test_tx_kernel_full_size(kernel, monkeypatch):
    monkeypatch.setenv("MI_CKSUM_TX_KERNEL", kernel)
    for layout in ("socket", "single"):
        c = make_case(65536, 1500, layout=layout, seed=32)
        want_dst, want_st = run_oracle(ORC, c)
        got_dst, got_st = run_gpu(c)
        assert not want_st.any() and np.array_equal(got_st, want_st), layout
        assert np.array_equal(got_dst, want_dst), layout


def test_tx_lds_many_frames_per_wave():
    """The LDS-staged gather (the default TX kernel) with a grid far smaller
    than the batch: every wave walks many frames through its ring (the
    grid-stride loop, the ring reused across frames), byte for byte against
    the oracle on every edge case."""
    mi.set_shape(0, 0, 3)
    try:
        for name, c in CASES:
            want_dst, want_st = run_oracle(ORC, c)
            got_dst, got_st = run_gpu(c)
            assert np.array_equal(got_st, want_st), (name, np.nonzero(got_st != want_st)[0][:8])
            bad = np.nonzero(got_dst != want_dst)[0]
            assert bad.size == 0, (name, bad.size, bad[:8])
    finally:
        mi.set_shape(0, 0, 0)


def _tx_batch(c):
    src = torch.from_numpy(c["src"]).cuda()
    dst = torch.from_numpy(c["dst"].copy()).cuda()
    tb = mi.TxBatch(src, c["seg_off"], c["seg_len"], c["pkt_seg"], c["pkt_len"], dst, dst_stride=c["stride"],
                    dst_first=c["dst_first"], room=c["room"], l3_off=c["l3"], csum_flags=c["flags"],
                    csum_data=c["data"], max_len=int(c["pkt_len"].max()))
    st = torch.full((tb.n,), 0xEE, dtype=torch.uint8, device="cuda")
    return tb, st


@pytest.mark.parametrize("engine", ["hip", "aql"])
def test_tx_repeat_every_case(engine):
    """The prepared TX handle (mi_cksum_tx_repeat_create; the bench's TX leg)
    through HIP launches and as AQL packets of mi_aql_tx_lds: every edge case,
    two batches per handle rotating over five passes on two queues, each
    batch's slots and status byte for byte against the oracle."""
    cases = [(n, c) for n, c in CASES if c["pkt_len"].size]
    for k in range(0, len(cases), 2):
        pair = cases[k:k + 2]
        made = [_tx_batch(c) for _, c in pair]
        torch.cuda.synchronize()
        rep = mi.TxRepeat([tb for tb, _ in made], [st for _, st in made], nstreams=2, engine=engine)
        try:
            rep.run(5, timed=True)
            assert rep.span() > 0
        finally:
            rep.close()
        for (name, c), (tb, st) in zip(pair, made):
            want_dst, want_st = run_oracle(ORC, c)
            got_st = st.cpu().numpy()
            assert np.array_equal(got_st, want_st), (engine, name, np.nonzero(got_st != want_st)[0][:8])
            bad = np.nonzero(tb.dst.cpu().numpy() != want_dst)[0]
            assert bad.size == 0, (engine, name, bad.size, bad[:8])


def test_tx_repeat_full_size_aql_equals_launch():
    """65536 x 1514 B socket chains, three batches rotating over 7 passes of
    the AQL engine: the slots and status equal mi_cksum_tx_copy's and the
    oracle's."""
    c = make_case(65536, 1500, layout="socket", seed=33)
    want_dst, want_st = run_oracle(ORC, c)
    made = [_tx_batch(c) for _ in range(3)]
    torch.cuda.synchronize()
    rep = mi.TxRepeat([tb for tb, _ in made], [st for _, st in made], nstreams=2, engine="aql")
    try:
        rep.run(7, timed=True)
        us = rep.span() / 7
    finally:
        rep.close()
    assert us > 0
    for tb, st in made:
        assert np.array_equal(st.cpu().numpy(), want_st)
        assert np.array_equal(tb.dst.cpu().numpy(), want_dst)


def test_tx_repeat_aql_needs_the_default_kernel(monkeypatch):
    """The AQL engine carries the default TX kernel only: with another ring
    selected it refuses (-ENOTSUP) instead of running something else; HIP
    launches still honour the override."""
    c = dict(CASES)["socket-1514"]
    tb, st = _tx_batch(c)
    torch.cuda.synchronize()
    monkeypatch.setenv("MI_CKSUM_TX_LDS", "2x3")
    with pytest.raises(mi.MiCksumError):
        mi.TxRepeat([tb], [st], engine="aql")
    rep = mi.TxRepeat([tb], [st], engine="hip")
    try:
        rep.run(2)
    finally:
        rep.close()
    want_dst, want_st = run_oracle(ORC, c)
    assert np.array_equal(st.cpu().numpy(), want_st)
    assert np.array_equal(tb.dst.cpu().numpy(), want_dst)


@pytest.mark.parametrize("seed", range(24))
def test_tx_random_sweep(seed):
    """Seeded random batches beyond the named edge cases: frame count, lengths
    (20-9000 B), chain layout, protocol, IP header length, L3 offset and
    destination alignment all drawn at random; the default TX kernel (and,
    for every third seed, the AQL engine's entry point through the prepared
    handle) byte for byte against the oracle, slots and status."""
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.integers(1, 200))
    hi = int(rng.choice([1500, 4000, 9000]))
    lens = rng.integers(20, hi + 1, n)
    layout = str(rng.choice(["socket", "single", "random"]))
    proto = int(rng.choice([6, 17, 1]))
    hl = rng.choice([20, 20, 20, 24, 40, 60], n)
    l3 = int(rng.choice([0, 14, 18, 64]))
    first = int(rng.integers(0, 256))
    c = make_case(n, lens, layout=layout, seed=2000 + seed, proto=proto, hl=hl, l3=l3, dst_first=first,
                  stride=9216 + 256)
    want_dst, want_st = run_oracle(ORC, c)
    got_dst, got_st = run_gpu(c)
    assert np.array_equal(got_st, want_st), (seed, layout, np.nonzero(got_st != want_st)[0][:8])
    bad = np.nonzero(got_dst != want_dst)[0]
    assert bad.size == 0, (seed, layout, bad.size, bad[:8])
    if seed % 3 == 0:
        tb, st = _tx_batch(c)
        torch.cuda.synchronize()
        rep = mi.TxRepeat([tb], [st], nstreams=1, engine="aql")
        try:
            rep.run(2)
        finally:
            rep.close()
        assert np.array_equal(st.cpu().numpy(), want_st), seed
        assert np.array_equal(tb.dst.cpu().numpy(), want_dst), seed
