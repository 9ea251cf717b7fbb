"""Parity of the HIP path against the oracle and the reference's golden vectors.

Every comparison is bit-exact (integer work).  All calls go through
libmicksum.so's C ABI: the drop-in in_cksum* symbols over real mbuf chains, and
the batch kernels over device tensors.
"""
import numpy as np
import pytest
import torch

from conftest import aligned, chain_segments
from oracle.pyoracle import Oracle

import libunsod_amd as mi
from libunsod_amd import synth

pytestmark = pytest.mark.gpu
ORC = Oracle("port")


def dev_tensor(a: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def cpu(t):
    return t.cpu().numpy()


# ------------------------------------------------- (b1) drop-ins vs golden
def test_dropin_skip_golden(golden, dropin_mode):
    g = golden
    bad = []
    for k in range(len(g["sk_result"])):
        segs = chain_segments(g, int(g["sk_seg0"][k]), int(g["sk_nseg"][k]))
        r = mi.in_cksum_skip(mi.MbufChain(segs), int(g["sk_len"][k]), int(g["sk_skip"][k]))
        if r != int(g["sk_result"][k]):
            bad.append(k)
    assert not bad, f"{len(bad)} mismatches, first {bad[:5]}"


def test_dropin_pseudo_golden(golden, dropin_mode):
    g = golden
    bad = []
    for k in range(len(g["ps_result"])):
        segs = chain_segments(g, int(g["ps_seg0"][k]), int(g["ps_nseg"][k]))
        r = mi.in_cksum_pseudo_header(mi.MbufChain(segs), int(g["ps_plen"][k]), int(g["ps_off0"][k]),
                                      int(g["ps_src"][k]), int(g["ps_dst"][k]), int(g["ps_proto"][k]))
        if r != int(g["ps_result"][k]):
            bad.append(k)
    assert not bad, f"{len(bad)} mismatches, first {bad[:5]}"


def test_dropin_hdr_golden(golden, dropin_mode):
    g = golden
    for k in range(len(g["hd_result"])):
        off = int(g["hd_off"][k])
        assert mi.in_cksum_hdr(g["blob"][off:off + 20].tobytes(), int(g["hd_mod"][k])) == int(g["hd_result"][k])


# -------------------------------------------------- (b2) batch vs golden
def test_verify_golden(golden):
    g = golden
    n = len(g["vb_offs"])
    buf = dev_tensor(g["ver_in"])
    b = mi.PktBatch(buf, n, offs=dev_tensor(g["vb_offs"].astype(np.int64)),
                    lens=dev_tensor(g["vb_flen"].astype(np.int32)))
    r = mi.ipv4_verify(b, bad_count=True)
    assert np.array_equal(cpu(r["ip"]), g["ver_ip"])
    assert np.array_equal(cpu(r["l4"]), g["ver_l4"])
    assert np.array_equal(cpu(r["status"]), g["ver_st"])
    assert int(r["bad"].item()) == int((g["ver_st"] != 0).sum())


def test_finalize_golden(golden):
    g = golden
    n = len(g["vb_offs"])
    buf = dev_tensor(g["fin_in"])
    b = mi.PktBatch(buf, n, offs=dev_tensor(g["vb_offs"].astype(np.int64)),
                    lens=dev_tensor(g["vb_flen"].astype(np.int32)))
    mi.ipv4_finalize(b)
    assert np.array_equal(cpu(buf), g["fin_out"])
    sl = dev_tensor(g["slot_in"])
    mi.ipv4_finalize(mi.PktBatch(sl, 64, stride=2176, first_off=142, fixed_len=1500))
    assert np.array_equal(cpu(sl), g["slot_out"])


# ------------------------------------------------------- spans vs oracle
@pytest.mark.parametrize("max_len", [0, 64, 300, 1500, 9100, 70000])
def test_span_batch_random(max_len):
    rng = np.random.default_rng(max_len + 5)
    n = 400
    hi = max(max_len, 64) if max_len else 2000
    lens = rng.integers(0, hi + 1, n)
    lens[:5] = [0, 1, 2, 3, hi]
    offs = synth.packed_offsets(lens, first_off=int(rng.integers(0, 16)), align=1) + \
        np.arange(n, dtype=np.uint64) * 3  # every alignment / parity
    size = int(offs[-1] + lens[-1]) + 64
    host = rng.integers(0, 256, size, dtype=np.uint8)
    host[int(offs[7]):int(offs[7] + lens[7])] = 0       # all-zero span
    host[int(offs[8]):int(offs[8] + lens[8])] = 0xFF    # all-ones span
    buf = dev_tensor(host)
    b = mi.PktBatch(buf, n, offs=dev_tensor(offs.astype(np.int64)), lens=dev_tensor(lens.astype(np.int32)),
                    max_len=max_len)
    _, h = aligned(host)
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    src = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    dst = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    proto = rng.integers(0, 256, n).astype(np.uint8)
    plens = (lens + rng.integers(0, 3, n) * 65536).astype(np.uint32)  # plen truncates to 16 bits in the seed

    got_skip = cpu(mi.span_batch(b))
    got_abs = cpu(mi.span_batch(b, mi.MI_SPAN_ABS))
    got_ps = cpu(mi.span_batch(b, src=dev_tensor(src), dst=dev_tensor(dst), proto=dev_tensor(proto),
                               plens=dev_tensor(plens)))
    got_seed = cpu(mi.span_batch(b, seeds=dev_tensor(seeds)))
    for i in range(n):
        o, L = int(offs[i]), int(lens[i])
        seg = h[o:o + L].tobytes()
        want = ORC.chain_skip([(seg, o % 64)], L, 0)
        assert got_skip[i] == want, (i, L, o)
        # absolute lanes: byte-swapped at odd addresses (in_cksum.c:278-285)
        wa = want if o % 2 == 0 else ((want & 0xFF) << 8) | (want >> 8)
        assert got_abs[i] == wa, (i, L, o)
        # pseudo-header: a one-mbuf chain with the span at off0 = 0; plen beyond the
        # chain truncates the walk silently but still seeds (uint16_t)plen
        wp = ORC.chain_pseudo([(seg, o % 64)], int(plens[i]), 0, int(src[i]), int(dst[i]), int(proto[i]))
        assert got_ps[i] == wp, (i, L)
        # explicit seed == complement of fold(seed + S)
        s = (~want & 0xFFFF) + int(seeds[i])
        f = 0 if s == 0 else 1 + (s - 1) % 65535
        assert got_seed[i] == (~f & 0xFFFF)


def test_span_pseudo_plen_truncation():
    """in_cksum_pseudo_header uses (uint16_t)plen in the seed (in_cksum.c:252-253)."""
    rng = np.random.default_rng(3)
    for L in (65515, 65536, 65536 + 20):
        data = rng.integers(0, 256, L, dtype=np.uint8)
        buf = dev_tensor(np.concatenate([data, np.zeros(64, np.uint8)]))
        b = mi.PktBatch(buf, 1, first_off=0, stride=0, fixed_len=L)
        src = np.array([0x0101A8C0], np.uint32); dst = np.array([0x0201A8C0], np.uint32); pr = np.array([6], np.uint8)
        got = cpu(mi.span_batch(b, src=dev_tensor(src), dst=dev_tensor(dst), proto=dev_tensor(pr)))[0]
        want = ORC.chain_pseudo([(data.tobytes(), 0)], L, 0, int(src[0]), int(dst[0]), 6)
        assert got == want


# --------------------------------------------- full-size configs (properties)
CONFIGS = {
    "1500": dict(n=65536, L=1500, stride=synth.STRIDE_1500, first=synth.IP_OFF),
    "9000": dict(n=65536, L=9000, stride=synth.STRIDE_9000, first=synth.IP_OFF),
    "64": dict(n=1 << 20, L=synth.MIN_FRAME_IP_LEN, stride=synth.STRIDE_64, first=synth.ETH_HLEN),
}


@pytest.mark.parametrize("name", list(CONFIGS))
def test_full_size_config(name):
    """BASELINE configs at full size: device-generated batch -> TX finalize ->
    RX verify must be all-valid; 1 % corrupted packets must be exactly the ones
    flagged; finalize output and verify outputs are compared bit-for-bit with the
    oracle over the whole batch."""
    c = CONFIGS[name]
    n, L, stride, first = c["n"], c["L"], c["stride"], c["first"]
    size = first + (n - 1) * stride + L + 64
    buf = torch.empty(size, dtype=torch.uint8, device="cuda")
    b = mi.PktBatch(buf, n, stride=stride, first_off=first, fixed_len=L)
    mi.synth_ipv4(b, seed=0x5EED5EED)
    raw = cpu(buf).copy()
    mi.ipv4_finalize(b)
    fin = cpu(buf)
    _, ref = aligned(raw)
    ORC.ipv4_finalize_batch(ref, n, stride=stride, first_off=first, fixed_flen=L, nthreads=8)
    assert np.array_equal(fin, ref)
    r = mi.ipv4_verify(b, bad_count=True)
    assert int(r["bad"].item()) == 0
    assert not cpu(r["ip"]).any() and not cpu(r["l4"]).any() and not cpu(r["status"]).any()
    # corrupt 1 %
    rng = np.random.default_rng(11)
    bad = np.sort(rng.choice(n, n // 100, replace=False))
    pos = first + bad.astype(np.int64) * stride + rng.integers(0, L, bad.size)
    flip = (1 << rng.integers(0, 8, bad.size)).astype(np.uint8)
    fin[pos] ^= flip
    buf.copy_(torch.from_numpy(fin))
    r = mi.ipv4_verify(b, bad_count=True)
    st = cpu(r["status"])
    assert np.array_equal(np.nonzero(st)[0], bad)
    assert int(r["bad"].item()) == bad.size
    ip, l4, st_o = ORC.ipv4_verify_batch(fin, n, stride=stride, first_off=first, fixed_flen=L, nthreads=8)
    assert np.array_equal(cpu(r["ip"]), ip) and np.array_equal(cpu(r["l4"]), l4)
    assert np.array_equal(st, st_o)


@pytest.mark.parametrize("packed", [False, True])
def test_pareto_mixed(packed):
    """Mixed 64-9000 B (Pareto) batch packed at 8-byte offsets."""
    n = 1 << 16
    lens = synth.pareto_lengths(n)
    offs = synth.packed_offsets(lens, first_off=2)
    b0 = synth.build_ipv4_batch(n, lens, offs=offs.astype(np.int64), payload="pattern")
    host = b0["buf"]
    _, ref = aligned(host)
    ORC.ipv4_finalize_batch(ref, n, offs=offs, flen=lens.astype(np.uint32), nthreads=8)
    buf = dev_tensor(host)
    b = mi.PktBatch(buf, n, offs=dev_tensor(offs.astype(np.int64)), lens=dev_tensor(lens.astype(np.int32)),
                    packed=packed)
    mi.ipv4_finalize(b)
    assert np.array_equal(cpu(buf), ref)
    r = mi.ipv4_verify(b)
    assert not cpu(r["status"]).any()
    fin = cpu(buf)
    fin[offs[::101].astype(np.int64) + 25] ^= 0x80
    buf.copy_(torch.from_numpy(fin))
    r = mi.ipv4_verify(b, bad_count=True)
    ip_o, l4_o, st_o = ORC.ipv4_verify_batch(fin, n, offs=offs, flen=lens.astype(np.uint32), nthreads=8)
    assert np.array_equal(cpu(r["ip"]), ip_o) and np.array_equal(cpu(r["l4"]), l4_o)
    assert np.array_equal(cpu(r["status"]), st_o) and int(r["bad"].item()) == len(offs[::101])


def test_host_path_matches_device():
    n, L, stride, first = 4096, 1500, 2176, 142
    b0 = synth.build_ipv4_batch(n, L, stride=stride, first_off=first, seed=5)
    host = b0["buf"]
    ORC.ipv4_finalize_batch(host, n, stride=stride, first_off=first, fixed_flen=L)
    host[first + 5 * stride + 100] ^= 1
    ip, l4, st, bad = mi.ipv4_verify_host(host, n, stride=stride, first_off=first, fixed_len=L)
    ip_o, l4_o, st_o = ORC.ipv4_verify_batch(host, n, stride=stride, first_off=first, fixed_flen=L)
    assert np.array_equal(ip, ip_o) and np.array_equal(l4, l4_o) and np.array_equal(st, st_o) and bad == 1
    # variable layout through the host path
    lens = synth.pareto_lengths(3000, seed=9)
    offs = synth.packed_offsets(lens, first_off=6)
    b1 = synth.build_ipv4_batch(3000, lens, offs=offs.astype(np.int64), seed=6)
    h1 = b1["buf"]
    ORC.ipv4_finalize_batch(h1, 3000, offs=offs, flen=lens.astype(np.uint32))
    ip, l4, st, bad = mi.ipv4_verify_host(h1, 3000, offs=offs, lens=lens)
    assert bad == 0 and not st.any()


@pytest.mark.parametrize("layout", ["slots", "packed"])
def test_host_zero_copy(layout):
    """Registered host batches are read in place over PCIe (zero-copy) and
    give the same results as the staged copy path and the oracle; an
    unregistered sub-range falls back to staging."""
    if layout == "slots":
        n, L, stride, first = 3000, 1500, 2176, 142
        b0 = synth.build_ipv4_batch(n, L, stride=stride, first_off=first, seed=15)
        lay = dict(stride=stride, first_off=first, fixed_len=L)
        olay = dict(stride=stride, first_off=first, fixed_flen=L)
        fin = dict(stride=stride, first_off=first, fixed_flen=L)
    else:
        n = 4000
        lens = synth.pareto_lengths(n, seed=19)
        offs = synth.packed_offsets(lens, first_off=6)
        b0 = synth.build_ipv4_batch(n, lens, offs=offs.astype(np.int64), seed=16)
        lay = dict(offs=offs, lens=lens)
        olay = fin = dict(offs=offs, flen=lens.astype(np.uint32))
    host = mi.page_buffer(b0["buf"].size)  # registrable: pages of its own
    host[:] = b0["buf"]
    ORC.ipv4_finalize_batch(host, n, **fin)
    rng = np.random.default_rng(3)
    host[rng.choice(host.size, 25, replace=False)] ^= 0x40
    want = ORC.ipv4_verify_batch(host, n, **olay)
    mi.host_register(host)
    try:
        for staged in (False, True):
            ip, l4, st, bad = mi.ipv4_verify_host(host, n, staged=staged, **lay)
            assert np.array_equal(ip, want[0]) and np.array_equal(l4, want[1]), staged
            assert np.array_equal(st, want[2]) and bad == int((want[2] != 0).sum()), staged
    finally:
        mi.host_unregister(host)
    ip, l4, st, bad = mi.ipv4_verify_host(host, n, **lay)  # no longer registered: staged
    assert np.array_equal(st, want[2])


def test_deterministic_and_stream_async():
    n, L = 8192, 1500
    buf = torch.empty(142 + n * 2176 + 64, dtype=torch.uint8, device="cuda")
    b = mi.PktBatch(buf, n, stride=2176, first_off=142, fixed_len=L)
    mi.synth_ipv4(b, seed=1)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        mi.ipv4_finalize(b)
        r1 = mi.ipv4_verify(b)
        r2 = mi.ipv4_verify(b)
    s.synchronize()
    for k in ("ip", "l4", "status"):
        assert np.array_equal(cpu(r1[k]), cpu(r2[k]))
    assert not cpu(r1["status"]).any()
    # the native back-to-back launcher writes the same outputs, on two streams
    outs = [dict(ip=torch.full((n,), 7, dtype=torch.int16, device="cuda").view(torch.uint16),
                 l4=torch.full((n,), 7, dtype=torch.int16, device="cuda").view(torch.uint16),
                 status=torch.full((n,), 9, dtype=torch.uint8, device="cuda"))]
    us, span = mi.ipv4_verify_repeat([b], outs, 6, nstreams=2, timing="pass")
    assert us.shape == (6,) and (us > 0).all() and span >= us.max() * 0.99
    assert mi.ipv4_verify_repeat([b], outs, 6, nstreams=3, timing="region") > 0
    for k in ("ip", "l4", "status"):
        assert np.array_equal(cpu(outs[0][k]), cpu(r1[k]))
    # the same passes as a cached hipGraph (MI_REPEAT_GRAPH): same outputs, replayable
    for k in ("ip", "l4", "status"):
        outs[0][k].fill_(3)
    assert mi.ipv4_verify_repeat([b], outs, 10, nstreams=2, timing="region", graph=True) > 0
    for k in ("ip", "l4", "status"):
        assert np.array_equal(cpu(outs[0][k]), cpu(r1[k]))
    buf[142 + 5 * 2176 + 700] ^= 1  # the graph reads the batch afresh on every replay
    assert mi.ipv4_verify_repeat([b], outs, 10, nstreams=2, timing="none", graph=True) is None
    assert int((outs[0]["status"] != 0).sum().item()) == 1


SHAPES = [(1, 4), (1, 8), (4, 1), (4, 2), (4, 4), (8, 2), (8, 4), (8, 8), (8, 12), (16, 2), (16, 4), (16, 6),
          (16, 8), (32, 2), (32, 3), (32, 4), (32, 6), (64, 2), (64, 3), (64, 4), (64, 6), (64, 9)]


@pytest.mark.parametrize("shape", SHAPES)
def test_every_shape_bit_exact(golden, shape):
    """The lane-group shape (and grid cap) changes speed only: every compiled
    shape reproduces the reference's verify / finalize / span results."""
    g = golden
    n = len(g["vb_offs"])
    offs = dev_tensor(g["vb_offs"].astype(np.int64))
    lens = dev_tensor(g["vb_flen"].astype(np.int32))
    mi.set_shape(shape[0], shape[1], 97)  # odd grid cap: many packets per group
    try:
        buf = dev_tensor(g["ver_in"])
        r = mi.ipv4_verify(mi.PktBatch(buf, n, offs=offs, lens=lens))
        assert np.array_equal(cpu(r["ip"]), g["ver_ip"])
        assert np.array_equal(cpu(r["l4"]), g["ver_l4"])
        assert np.array_equal(cpu(r["status"]), g["ver_st"])
        fin = dev_tensor(g["fin_in"])
        mi.ipv4_finalize(mi.PktBatch(fin, n, offs=offs, lens=lens))
        assert np.array_equal(cpu(fin), g["fin_out"])
        # spans: in_cksum_skip over every datagram region of the verify buffer
        sp = cpu(mi.span_batch(mi.PktBatch(buf, n, offs=offs, lens=lens)))
        _, h = aligned(g["ver_in"])
        for i in range(0, n, 7):
            o, L = int(g["vb_offs"][i]), int(g["vb_flen"][i])
            assert sp[i] == ORC.chain_skip([(h[o:o + L].tobytes(), o % 64)], L, 0)
    finally:
        mi.set_shape(0, 0, 0)


def test_packed_layout_golden(golden):
    """MI_BATCH_PACKED (flat ranges of 64 datagrams) on the reference's golden
    RX batch: runts, options, malformed headers, corrupted packets, odd starts."""
    g = golden
    n = len(g["vb_offs"])
    buf = dev_tensor(g["ver_in"])
    b = mi.PktBatch(buf, n, offs=dev_tensor(g["vb_offs"].astype(np.int64)),
                    lens=dev_tensor(g["vb_flen"].astype(np.int32)), packed=True)
    r = mi.ipv4_verify(b, bad_count=True)
    assert np.array_equal(cpu(r["ip"]), g["ver_ip"])
    assert np.array_equal(cpu(r["l4"]), g["ver_l4"])
    assert np.array_equal(cpu(r["status"]), g["ver_st"])
    assert int(r["bad"].item()) == int((g["ver_st"] != 0).sum())


@pytest.mark.parametrize("variant", [(4, 0, 0), (8, 1, 0), (4, 1, 0), (8, 0, 1), (4, 0, 1)])
def test_packed_variants_golden(golden, variant):
    """The flat-run kernel's round-6 variants -- chunks per pass U, pipelined
    passes (mi__set_run_pipe), header windows reloaded at a tighter register
    budget (mi__set_run_occ) -- on the golden RX batch (HIP launches) and on a
    Pareto batch through the AQL engine, bit-exact."""
    import ctypes as C
    lib = mi.load()
    for f in ("mi__set_packed_u", "mi__set_run_pipe", "mi__set_run_occ"):
        getattr(lib, f).restype = C.c_int
        getattr(lib, f).argtypes = [C.c_int]
    u, pipe, occ = variant
    was = (lib.mi__set_packed_u(u), lib.mi__set_run_pipe(pipe), lib.mi__set_run_occ(occ))
    try:
        test_packed_layout_golden(golden)
        n = 20000
        lens = synth.pareto_lengths(n, seed=23)
        offs = synth.packed_offsets(lens, first_off=2)
        b0 = synth.build_ipv4_batch(n, lens, offs=offs.astype(np.int64), seed=24)
        _, ref = aligned(b0["buf"])
        ORC.ipv4_finalize_batch(ref, n, offs=offs, flen=lens.astype(np.uint32), nthreads=8)
        ref[offs[::97].astype(np.int64) + 33] ^= 0x21
        ip_o, l4_o, st_o = ORC.ipv4_verify_batch(ref, n, offs=offs, flen=lens.astype(np.uint32), nthreads=8)
        b = mi.PktBatch(dev_tensor(ref), n, offs=dev_tensor(offs.astype(np.int64)), lens=dev_tensor(lens.astype(np.int32)),
                        packed=True, offs32=True)
        outs = [dict(ip=torch.zeros(n, dtype=torch.uint16, device="cuda"), l4=torch.zeros(n, dtype=torch.uint16, device="cuda"),
                     status=torch.zeros(n, dtype=torch.uint8, device="cuda"))]
        rep = mi.VerifyRepeat([b], outs, nstreams=2, engine="aql")
        rep.run(3)
        rep.close()
        assert np.array_equal(cpu(outs[0]["ip"]), ip_o) and np.array_equal(cpu(outs[0]["l4"]), l4_o)
        assert np.array_equal(cpu(outs[0]["status"]), st_o)
    finally:
        lib.mi__set_packed_u(was[0])
        lib.mi__set_run_pipe(was[1])
        lib.mi__set_run_occ(was[2])


@pytest.mark.parametrize("layout", ["packed", "shuffled", "gappy"])
def test_packed_hint_any_layout(layout):
    """The packed kernel is exact on real packed batches and falls back (still
    exact) when the hint is wrong: descending offsets, large gaps."""
    rng = np.random.default_rng(41)
    n = 5000
    lens = synth.pareto_lengths(n, seed=8)
    offs = synth.packed_offsets(lens, first_off=6)
    if layout == "gappy":
        offs = offs + np.arange(n, dtype=np.uint64) * 200
    b0 = synth.build_ipv4_batch(n, lens, offs=offs.astype(np.int64), seed=9, proto=rng.choice([6, 17], n))
    host = b0["buf"]
    _, ref = aligned(host)
    ORC.ipv4_finalize_batch(ref, n, offs=offs, flen=lens.astype(np.uint32))
    bad = rng.choice(n, 40, replace=False)
    ref[offs[bad].astype(np.int64) + rng.integers(0, 40, 40)] ^= 0x11
    perm = np.arange(n)
    if layout == "shuffled":
        perm = rng.permutation(n)
    o2, l2 = offs[perm], lens[perm]
    ip_o, l4_o, st_o = ORC.ipv4_verify_batch(ref, n, offs=o2, flen=l2.astype(np.uint32))
    buf = dev_tensor(ref)
    b = mi.PktBatch(buf, n, offs=dev_tensor(o2.astype(np.int64)), lens=dev_tensor(l2.astype(np.int32)),
                    packed=True)
    r = mi.ipv4_verify(b, bad_count=True)
    assert np.array_equal(cpu(r["ip"]), ip_o)
    assert np.array_equal(cpu(r["l4"]), l4_o)
    assert np.array_equal(cpu(r["status"]), st_o)
    assert int(r["bad"].item()) == int((st_o != 0).sum()) >= 40


# ------------------------------------------- (f) scatter-gather chain batches
def _golden_chains(g, pfx):
    return [chain_segments(g, int(g[pfx + "_seg0"][k]), int(g[pfx + "_nseg"][k])) for k in range(len(g[pfx + "_result"]))]


def test_chain_batch_skip_golden(golden):
    g = golden
    cb = mi.ChainBatch(_golden_chains(g, "sk"))
    out = mi.chain_batch(cb, dev_tensor(g["sk_len"].astype(np.int32)), dev_tensor(g["sk_skip"].astype(np.int32)))
    np.testing.assert_array_equal(cpu(out).astype(np.int64), g["sk_result"].astype(np.int64))


def test_chain_batch_pseudo_golden(golden):
    g = golden
    cb = mi.ChainBatch(_golden_chains(g, "ps"))
    out = mi.chain_batch(cb, dev_tensor(g["ps_plen"].astype(np.int32)), dev_tensor(g["ps_off0"].astype(np.int32)),
                         src=dev_tensor(g["ps_src"].astype(np.int64)), dst=dev_tensor(g["ps_dst"].astype(np.int64)),
                         proto=dev_tensor(g["ps_proto"].astype(np.uint8)))
    np.testing.assert_array_equal(cpu(out).astype(np.int64), g["ps_result"].astype(np.int64))


def test_chain_batch_walk_edges():
    """Zero-length mbufs, skips ending exactly on / past a segment boundary,
    short chains, 64 KiB TSO chains of 2 KiB clusters -- against the port."""
    rng = np.random.default_rng(0xC4A1)
    chains, lens, skips = [], [], []
    for i in range(600):
        nseg = int(rng.integers(1, 40 if i % 50 == 0 else 6))
        segs = []
        for _ in range(nseg):
            L = 0 if rng.random() < 0.15 else int(rng.choice([1, 2, 3, 15, 16, 17, 2048, int(rng.integers(1, 3000))]))
            segs.append((rng.integers(0, 256, L, dtype=np.uint8).tobytes(), int(rng.integers(64))))
        total = sum(len(s) for s, _ in segs)
        bounds = np.cumsum([len(s) for s, _ in segs])
        c = rng.random()
        skip = 0 if c < 0.3 else int(rng.choice(bounds)) if c < 0.6 else int(rng.integers(0, total + 3))
        length = max(skip, total if rng.random() < 0.5 else int(rng.integers(0, total + 40)))
        chains.append(segs), lens.append(length), skips.append(skip)
    for _ in range(8):  # TSO send: 64 KiB in 2 KiB clusters, odd placements
        segs = [(rng.integers(0, 256, 2048, dtype=np.uint8).tobytes(), int(rng.integers(64))) for _ in range(32)]
        chains.append(segs), lens.append(65536), skips.append(int(rng.integers(0, 60)))
    want = np.array([ORC.chain_skip(c, L, s) for c, L, s in zip(chains, lens, skips)], np.int64)
    cb = mi.ChainBatch(chains)
    out = mi.chain_batch(cb, dev_tensor(np.array(lens, np.int32)), dev_tensor(np.array(skips, np.int32)))
    np.testing.assert_array_equal(cpu(out).astype(np.int64), want)
    # pseudo over the same chains (off0 inside the first mbuf, as tcp_output guarantees)
    off0 = np.array([min(20, len(c[0][0])) for c in chains], np.int32)
    plen = np.array([max(0, sum(len(s) for s, _ in c) - o - int(rng.integers(0, 5))) for c, o in zip(chains, off0)],
                    np.int32)
    src = rng.integers(0, 2**32, len(chains)); dst = rng.integers(0, 2**32, len(chains))
    proto = rng.choice([6, 17], len(chains)).astype(np.uint8)
    want = np.array([ORC.chain_pseudo(c, int(p), int(o), int(s), int(d), int(pr))
                     for c, p, o, s, d, pr in zip(chains, plen, off0, src, dst, proto)], np.int64)
    out = mi.chain_batch(cb, dev_tensor(plen), dev_tensor(off0), src=dev_tensor(src.astype(np.int64)),
                         dst=dev_tensor(dst.astype(np.int64)), proto=dev_tensor(proto))
    np.testing.assert_array_equal(cpu(out).astype(np.int64), want)


# --------------------------------------------- (f) RX offload csum_flags / csum_data
def _rx_mix(n, seed):
    """A received burst with everything the flag rules distinguish: TCP, UDP,
    ICMP and other protocols, IP options, fragments, UDP ulen != ip_len - hl,
    bad checksums, Ethernet padding, ip_len past the frame, hl < 20."""
    from oracle.pyoracle import rx_offload_flags  # noqa: F401  (checker)
    rng = np.random.default_rng(seed)
    lens = np.where(rng.random(n) < 0.3, rng.integers(28, 200, n), rng.integers(200, 9001, n)).astype(np.int64)
    proto = rng.choice([6, 6, 6, 17, 17, 1, 47], n)
    hl = np.where(rng.random(n) < 0.1, rng.choice([24, 40, 60], n), 20)
    hl = np.minimum(hl, (lens // 4) * 4)
    offs = synth.packed_offsets(lens + 8, first_off=2)
    b0 = synth.build_ipv4_batch(n, lens, offs=offs, proto=proto, hl=hl, seed=seed, payload="random")
    h = mi.page_buffer(b0["buf"].size)  # registrable (test_host_paths_offsets): pages of its own
    h[:] = b0["buf"]
    keep = h
    o = offs.astype(np.int64)
    frag = rng.random(n) < 0.05
    for i in np.nonzero(frag)[0]:
        h[o[i] + 6] = int(rng.choice([0x20, 0x00, 0x21]))  # MF, offset only, both
        h[o[i] + 7] = int(rng.integers(1, 256)) if h[o[i] + 6] != 0x20 else 0
    udp_bad = (proto == 17) & (rng.random(n) < 0.2) & (lens - hl >= 8)
    for i in np.nonzero(udp_bad)[0]:
        h[o[i] + hl[i] + 5] ^= int(rng.integers(1, 8))
    ORC.ipv4_finalize_batch(h, n, offs=offs, flen=lens.astype(np.uint32))
    flen = lens.copy()
    pad = rng.random(n) < 0.05  # Ethernet padding after ip_len
    flen[pad] += 8
    for i in np.nonzero((rng.random(n) < 0.05) & (lens > hl))[0]:  # corrupt a payload byte
        h[o[i] + int(rng.integers(hl[i], lens[i]))] ^= 0x10
    for i in np.nonzero(rng.random(n) < 0.03)[0]:  # corrupt the header checksum
        h[o[i] + 10] ^= 1
    for i in np.nonzero(rng.random(n) < 0.02)[0]:  # ip_len past the frame
        h[o[i] + 2] = 0xFF
    for i in np.nonzero(rng.random(n) < 0.01)[0]:  # hl < 20
        h[o[i]] = 0x44
    return keep, h, o, flen.astype(np.uint32)


@pytest.mark.parametrize("layout", ["unpacked", "packed"])
def test_rx_offload_flags(layout):
    from oracle.pyoracle import CSUM_DATA_VALID, CSUM_IP_CHECKED, CSUM_IP_VALID, rx_offload_flags
    n = 20000
    keep, h, o, flen = _rx_mix(n, 0x0FF1 + (layout == "packed"))
    ip_o, l4_o, st_o = ORC.ipv4_verify_batch(h, n, offs=o.astype(np.uint64), flen=flen, nthreads=8)
    want_fl, want_cd = rx_offload_flags(h, o, flen, ip_o, l4_o, st_o)
    # every rule is exercised
    chk, val, dv = (want_fl & CSUM_IP_CHECKED) != 0, (want_fl & CSUM_IP_VALID) != 0, (want_fl & CSUM_DATA_VALID) != 0
    assert dv.any() and (chk & ~dv).any() and (chk & ~val).any() and (want_fl == 0).any()
    buf = dev_tensor(h)
    b = mi.PktBatch(buf, n, offs=dev_tensor(o), lens=dev_tensor(flen.astype(np.int32)), packed=layout == "packed")
    r = mi.rx_offload(b, bad_count=True)
    fl = cpu(r["flags"]).astype(np.uint32)
    cd = cpu(r["data"]).astype(np.uint32)
    np.testing.assert_array_equal(fl, want_fl)
    np.testing.assert_array_equal(cd, want_cd)
    assert int(r["bad"].item()) == int((st_o != 0).sum())
    # the stack's decisions through the offload branch equal its own sums
    chk = (fl & CSUM_IP_CHECKED) != 0
    assert np.array_equal(((fl & CSUM_IP_VALID) == 0)[chk], (ip_o != 0)[chk])
    dv = (fl & CSUM_DATA_VALID) != 0
    assert np.array_equal((cd ^ 0xFFFF)[dv], l4_o[dv].astype(np.uint32))


@pytest.mark.parametrize("first", [14, 2, 7, 30])
def test_slot64_edge_cases(first):
    """Minimum-size frames in 64-byte slots (k_ipv4_verify_slot64): malformed
    headers, IP options, Ethernet padding past ip_len, UDP / ICMP / IGMP,
    fragments and corrupted bytes at odd and even starts -- verify, demux
    verify and RX offload flags all equal the oracle."""
    rng = np.random.default_rng(first)
    n, L, stride = 6000, 46, 64
    proto = rng.choice([6, 17, 1, 2], n)
    hl = rng.choice([20, 20, 20, 24], n)
    b0 = synth.build_ipv4_batch(n, L, stride=stride, first_off=first, proto=proto, hl=hl, seed=first + 1)
    host = b0["buf"]
    _, h = aligned(host)
    ORC.ipv4_finalize_batch(h, n, stride=stride, first_off=first, fixed_flen=L)
    for i in rng.choice(n, 600, replace=False):
        p = first + int(i) * stride
        k = int(rng.integers(0, 6))
        if k == 0:
            h[p] = 0x40 | int(rng.integers(0, 16))                 # any hl, incl. < 20 and > flen
        elif k == 1:
            v = int(rng.integers(0, 80))                          # ip_len below, at or past the frame
            h[p + 2], h[p + 3] = v >> 8, v & 0xFF
        elif k == 2:
            h[p + 6] = 0x20                                       # a fragment
        else:
            h[p + int(rng.integers(0, L))] ^= np.uint8(1 << int(rng.integers(8)))
    buf = dev_tensor(h)
    b = mi.PktBatch(buf, n, stride=stride, first_off=first, fixed_len=L)
    assert mi.verify_plan(b) == ("k_ipv4_verify_slot64" if first < 16 else "k_ipv4_verify_packed<4,2 waves>")
    r = mi.ipv4_verify(b, bad_count=True)
    ip, l4, st = ORC.ipv4_verify_batch(h, n, stride=stride, first_off=first, fixed_flen=L)
    assert np.array_equal(cpu(r["ip"]), ip) and np.array_equal(cpu(r["l4"]), l4)
    assert np.array_equal(cpu(r["status"]), st) and int(r["bad"].item()) == int((st != 0).sum())
    bd = mi.PktBatch(buf, n, stride=stride, first_off=first, fixed_len=L, demux=True)
    rd = mi.ipv4_verify(bd)
    ipd, l4d, std = ORC.ipv4_verify_batch(h, n, stride=stride, first_off=first, fixed_flen=L, demux=True)
    assert np.array_equal(cpu(rd["l4"]), l4d) and np.array_equal(cpu(rd["status"]), std)
    from oracle.pyoracle import rx_offload_flags
    offs = first + np.arange(n, dtype=np.int64) * stride
    fl, cd = rx_offload_flags(h, offs, np.full(n, L), ip, l4, st)
    ro = mi.rx_offload(b)
    assert np.array_equal(cpu(ro["flags"]).view(np.uint32), fl)
    assert np.array_equal(cpu(ro["data"]).view(np.uint32), cd)


def test_full_size_pareto_and_shards():
    """BASELINE configs[4] at full size (2^22 Pareto datagrams, 1.19 GB, packed):
    device-generated -> TX finalize -> RX verify all valid; 1 % corrupted
    datagrams are exactly the ones flagged, bit-exact with the oracle; and the
    8 byte-balanced shards a node would get (shard.shard_by_bytes) verify to the
    same outputs as the whole batch."""
    from libunsod_amd import shard
    n = 1 << 22
    lens = synth.pareto_lengths(n)
    offs = synth.packed_offsets(lens, first_off=2)
    size = (int(offs[-1] + lens[-1]) + 64 + 255) & ~255
    buf = torch.empty(size, dtype=torch.uint8, device="cuda")
    d_offs = dev_tensor(offs.astype(np.int64))
    d_lens = dev_tensor(lens.astype(np.int32))
    b = mi.PktBatch(buf, n, offs=d_offs, lens=d_lens, max_len=int(lens.max()), packed=True)
    mi.synth_ipv4(b, seed=0x9A7E70)
    mi.ipv4_finalize(b)
    r = mi.ipv4_verify(b, bad_count=True)
    assert int(r["bad"].item()) == 0
    rng = np.random.default_rng(5)
    bad = np.sort(rng.choice(n, n // 100, replace=False))
    pos = offs[bad].astype(np.int64) + rng.integers(0, lens[bad])
    host = cpu(buf)
    host[pos] ^= (1 << rng.integers(0, 8, bad.size)).astype(np.uint8)
    buf.copy_(torch.from_numpy(host))
    r = mi.ipv4_verify(b, bad_count=True)
    st = cpu(r["status"])
    assert np.array_equal(np.nonzero(st)[0], bad) and int(r["bad"].item()) == bad.size
    _, h = aligned(host)
    ip, l4, st_o = ORC.ipv4_verify_batch(h, n, offs=offs, flen=lens.astype(np.uint32), nthreads=16)
    assert np.array_equal(cpu(r["ip"]), ip) and np.array_equal(cpu(r["l4"]), l4) and np.array_equal(st, st_o)
    # the 8-GPU partition: contiguous byte-balanced ranges, each verified as its own batch
    for rank in range(8):
        lo, hi = shard.shard_by_bytes(lens, 8, rank)
        bs = mi.PktBatch(buf, hi - lo, offs=d_offs[lo:hi], lens=d_lens[lo:hi], max_len=int(lens.max()), packed=True)
        rs = mi.ipv4_verify(bs)
        assert np.array_equal(cpu(rs["status"]), st[lo:hi]) and np.array_equal(cpu(rs["l4"]), l4[lo:hi])


@pytest.mark.parametrize("hint", [True, False])
def test_finalize_golden_flat_run(golden, hint):
    """TX finalize through the flat-run kernel (packed hint) on the reference's
    golden batch: runts, options, malformed headers, odd starts, UDP / ICMP --
    byte-identical to the reference's output either way."""
    g = golden
    n = len(g["vb_offs"])
    buf = dev_tensor(g["fin_in"])
    b = mi.PktBatch(buf, n, offs=dev_tensor(g["vb_offs"].astype(np.int64)),
                    lens=dev_tensor(g["vb_flen"].astype(np.int32)), packed=hint)
    mi.ipv4_finalize(b)
    assert np.array_equal(cpu(buf), g["fin_out"])


@pytest.mark.parametrize("layout", ["packed", "shuffled"])
def test_span_batch_flat_run(layout):
    """mi_cksum_span_batch with the packed hint (flat-run span mode): stream and
    absolute lanes, pseudo-header seeds, empty / odd / long spans (> 65535 B
    take the per-span fallback) -- equal to the oracle's chains."""
    rng = np.random.default_rng(9 if layout == "packed" else 10)
    n = 3000
    lens = synth.pareto_lengths(n, seed=4)
    lens[:6] = [0, 1, 2, 3, 65535, 70000]
    offs = synth.packed_offsets(lens, first_off=3, align=1) + np.arange(n, dtype=np.uint64) % 3
    if layout == "shuffled":
        perm = rng.permutation(n)
        offs, lens = offs[perm], lens[perm]
    size = int((offs + lens).max()) + 64
    host = rng.integers(0, 256, size, dtype=np.uint8)
    buf = dev_tensor(host)
    b = mi.PktBatch(buf, n, offs=dev_tensor(offs.astype(np.int64)), lens=dev_tensor(lens.astype(np.int32)),
                    packed=True)
    src = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    dst = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    proto = rng.integers(0, 256, n).astype(np.uint8)
    got = cpu(mi.span_batch(b))
    got_abs = cpu(mi.span_batch(b, mi.MI_SPAN_ABS))
    got_ps = cpu(mi.span_batch(b, src=dev_tensor(src), dst=dev_tensor(dst), proto=dev_tensor(proto)))
    _, h = aligned(host)
    for i in range(n):
        o, L = int(offs[i]), int(lens[i])
        seg = h[o:o + L].tobytes()
        want = ORC.chain_skip([(seg, o % 64)], L, 0)
        assert got[i] == want, (i, L, o)
        assert got_abs[i] == (want if o % 2 == 0 else ((want & 0xFF) << 8) | (want >> 8)), (i, L, o)
        assert got_ps[i] == ORC.chain_pseudo([(seg, o % 64)], L, 0, int(src[i]), int(dst[i]), int(proto[i])), i


# ------------------------------------------- MI_BATCH_OFFS32 (u32 offsets)
@pytest.mark.parametrize("layout", ["packed", "shuffled", "gappy"])
def test_offs32_same_results(golden, layout):
    """u32 packet offsets (MI_BATCH_OFFS32) give exactly what u64 offsets give:
    RX verify, RX offload flags, span folds and TX finalize, on a mixed-length
    batch (packed, shuffled, gappy) and on the reference's golden RX batch."""
    rng = np.random.default_rng(77)
    n = 6000
    lens = synth.pareto_lengths(n, seed=12)
    offs = synth.packed_offsets(lens, first_off=2)
    if layout == "gappy":
        offs = offs + np.arange(n, dtype=np.uint64) * 130
    b0 = synth.build_ipv4_batch(n, lens, offs=offs.astype(np.int64), seed=13, proto=rng.choice([6, 17], n))
    _, ref = aligned(b0["buf"])
    ORC.ipv4_finalize_batch(ref, n, offs=offs, flen=lens.astype(np.uint32))
    fin_in = ref.copy()
    bad = rng.choice(n, 50, replace=False)
    ref[offs[bad].astype(np.int64) + rng.integers(0, 40, 50)] ^= 0x21
    perm = rng.permutation(n) if layout == "shuffled" else np.arange(n)
    o2, l2 = offs[perm], lens[perm]
    ip_o, l4_o, st_o = ORC.ipv4_verify_batch(ref, n, offs=o2, flen=l2.astype(np.uint32))
    buf = dev_tensor(ref)
    d_lens = dev_tensor(l2.astype(np.int32))
    b64 = mi.PktBatch(buf, n, offs=dev_tensor(o2.astype(np.int64)), lens=d_lens, packed=True)
    b32 = mi.PktBatch(buf, n, offs=dev_tensor(o2.astype(np.int64)), lens=d_lens, packed=True, offs32=True)
    assert b32.offs.dtype == torch.int32 and b32.c.flags & 8
    r = mi.ipv4_verify(b32, bad_count=True)
    assert np.array_equal(cpu(r["ip"]), ip_o) and np.array_equal(cpu(r["l4"]), l4_o)
    assert np.array_equal(cpu(r["status"]), st_o) and int(r["bad"].item()) == int((st_o != 0).sum()) >= 50
    ro32, ro64 = mi.rx_offload(b32), mi.rx_offload(b64)
    assert all(torch.equal(ro32[k], ro64[k]) for k in ro64 if torch.is_tensor(ro64[k]))
    assert torch.equal(mi.span_batch(b32), mi.span_batch(b64))
    # TX finalize in place, u32 offsets (shuffled order included) == the oracle's finalize
    _, fsrc = aligned(b0["buf"])
    fbuf = dev_tensor(fsrc)
    bf = mi.PktBatch(fbuf, n, offs=dev_tensor(o2.astype(np.int64)), lens=d_lens, packed=True, offs32=True)
    mi.ipv4_finalize(bf)
    assert np.array_equal(cpu(fbuf), fin_in)
    g = golden
    gn = len(g["vb_offs"])
    gb = mi.PktBatch(dev_tensor(g["ver_in"]), gn, offs=dev_tensor(g["vb_offs"].astype(np.int64)),
                     lens=dev_tensor(g["vb_flen"].astype(np.int32)), packed=True, offs32=True)
    gr = mi.ipv4_verify(gb)
    assert np.array_equal(cpu(gr["ip"]), g["ver_ip"]) and np.array_equal(cpu(gr["l4"]), g["ver_l4"])
    assert np.array_equal(cpu(gr["status"]), g["ver_st"])
    gbuf = dev_tensor(g["fin_in"])
    gf = mi.PktBatch(gbuf, gn, offs=dev_tensor(g["vb_offs"].astype(np.int64)),
                     lens=dev_tensor(g["vb_flen"].astype(np.int32)), packed=True, offs32=True)
    mi.ipv4_finalize(gf)
    assert np.array_equal(cpu(gbuf), g["fin_out"])


@pytest.mark.parametrize("shape", ["", "8x12"])
def test_verify_multi_matches_single(shape):
    """mi_cksum_ipv4_verify_multi == mi_cksum_ipv4_verify per batch: slot
    batches of several lengths (merged into one launch), a packed batch (its
    own launch), empty and one-packet batches, corrupted datagrams."""
    if shape:
        mi.set_shape(*[int(x) for x in shape.split("x")])
    try:
        rng = np.random.default_rng(404)
        batches, outs, want = [], [], []
        specs = [(3000, 1500, 2176, 142), (1, 1500, 2176, 142), (0, 1500, 2176, 142), (777, 9000, 9216, 142),
                 (2500, 600, 640, 2), (4096, 1500, 2176, 143)]
        for n, L, stride, first in specs:
            b0 = synth.build_ipv4_batch(n, L, stride=stride, first_off=first, seed=n + L, payload="pattern")
            h = b0["buf"] if n else np.zeros(4096, np.uint8)
            if n:
                ORC.ipv4_finalize_batch(h, n, stride=stride, first_off=first, fixed_flen=L)
                for i in rng.choice(n, max(1, n // 50), replace=False):
                    h[first + int(i) * stride + int(rng.integers(0, L))] ^= 0x22
            want.append(ORC.ipv4_verify_batch(h, n, stride=stride, first_off=first, fixed_flen=L) if n else None)
            batches.append(mi.PktBatch(dev_tensor(h), n, stride=stride, first_off=first, fixed_len=L))
            outs.append(dict(ip=torch.zeros(max(n, 1), dtype=torch.uint16, device="cuda"),
                             l4=torch.zeros(max(n, 1), dtype=torch.uint16, device="cuda"),
                             status=torch.zeros(max(n, 1), dtype=torch.uint8, device="cuda")))
        lens = synth.pareto_lengths(3000, seed=5)
        offs = synth.packed_offsets(lens, first_off=2)
        bp = synth.build_ipv4_batch(3000, lens, offs=offs.astype(np.int64), seed=6)
        hp = bp["buf"]
        ORC.ipv4_finalize_batch(hp, 3000, offs=offs, flen=lens.astype(np.uint32))
        hp[offs[::37].astype(np.int64) + 21] ^= 1
        want.append(ORC.ipv4_verify_batch(hp, 3000, offs=offs, flen=lens.astype(np.uint32)))
        batches.append(mi.PktBatch(dev_tensor(hp), 3000, offs=dev_tensor(offs.astype(np.int64)),
                                   lens=dev_tensor(lens.astype(np.int32)), packed=True))
        outs.append(dict(ip=torch.zeros(3000, dtype=torch.uint16, device="cuda"),
                         l4=torch.zeros(3000, dtype=torch.uint16, device="cuda"),
                         status=torch.zeros(3000, dtype=torch.uint8, device="cuda")))
        bad = torch.zeros(1, dtype=torch.int32, device="cuda")
        mi.ipv4_verify_multi(batches, outs, bad=bad)
        torch.cuda.synchronize()
        nbad = 0
        for w, o, b in zip(want, outs, batches):
            if w is None:
                continue
            assert np.array_equal(cpu(o["ip"])[:b.n], w[0]) and np.array_equal(cpu(o["l4"])[:b.n], w[1])
            assert np.array_equal(cpu(o["status"])[:b.n], w[2])
            nbad += int((w[2] != 0).sum())
        assert int(bad.item()) == nbad
    finally:
        mi.set_shape(0, 0, 0)


@pytest.mark.parametrize("offs32", [False, True])
def test_verify_multi_offset_arrays(offs32):
    """The multi-batch launch over batches described by offset arrays with a
    fixed length (the descriptor of a wave's next unit is prefetched inside a
    batch, never across one): offsets in shuffled slot order, batch sizes that
    end mid-unit, one launch; every output == the oracle's for its slot."""
    rng = np.random.default_rng(808)
    batches, outs, want = [], [], []
    for n, L, stride, first in [(5000, 1500, 2176, 142), (33, 1500, 2176, 142), (4099, 600, 640, 2),
                                (1, 1500, 2176, 142), (2500, 9000, 9216, 142)]:
        b0 = synth.build_ipv4_batch(n, L, stride=stride, first_off=first, seed=n + 3 * L, payload="pattern")
        h = b0["buf"]
        ORC.ipv4_finalize_batch(h, n, stride=stride, first_off=first, fixed_flen=L)
        for i in rng.choice(n, max(1, n // 40), replace=False):
            h[first + int(i) * stride + int(rng.integers(0, L))] ^= 0x41
        offs = first + rng.permutation(n).astype(np.int64) * stride
        want.append(ORC.ipv4_verify_batch(h, n, offs=offs, fixed_flen=L))
        batches.append(mi.PktBatch(dev_tensor(h), n, offs=dev_tensor(offs), fixed_len=L, offs32=offs32))
        outs.append(dict(ip=torch.zeros(n, dtype=torch.uint16, device="cuda"),
                         l4=torch.zeros(n, dtype=torch.uint16, device="cuda"),
                         status=torch.zeros(n, dtype=torch.uint8, device="cuda")))
    bad = torch.zeros(1, dtype=torch.int32, device="cuda")
    mi.ipv4_verify_multi(batches, outs, bad=bad)
    torch.cuda.synchronize()
    for w, o in zip(want, outs):
        assert np.array_equal(cpu(o["ip"]), w[0]) and np.array_equal(cpu(o["l4"]), w[1])
        assert np.array_equal(cpu(o["status"]), w[2])
    assert int(bad.item()) == sum(int((w[2] != 0).sum()) for w in want)


def test_repeat_handle_outputs_and_rotation():
    """mi_cksum_repeat_*: every pass writes exactly what mi_cksum_ipv4_verify
    writes for its batch; runs continue the batch rotation; timed runs give a
    positive span; the finalize op equals mi_cksum_ipv4_finalize; busy-wait
    mode changes nothing but the wait."""
    n, L, stride, first = 2048, 1500, 2176, 142
    bs, outs, want = [], [], []
    for r in range(3):
        b0 = synth.build_ipv4_batch(n, L, stride=stride, first_off=first, seed=90 + r)
        h = b0["buf"]
        ORC.ipv4_finalize_batch(h, n, stride=stride, first_off=first, fixed_flen=L)
        h[first + (7 * r + 3) * stride + 200] ^= 0x80
        want.append(ORC.ipv4_verify_batch(h, n, stride=stride, first_off=first, fixed_flen=L))
        bs.append(mi.PktBatch(dev_tensor(h), n, stride=stride, first_off=first, fixed_len=L))
        outs.append(dict(ip=torch.zeros(n, dtype=torch.uint16, device="cuda"),
                         l4=torch.zeros(n, dtype=torch.uint16, device="cuda"),
                         status=torch.zeros(n, dtype=torch.uint8, device="cuda")))
    mi.set_busy_wait(True)
    try:
        for ns in (1, 2, 3):
            rep = mi.VerifyRepeat(bs, outs, nstreams=ns)
            for o in outs:
                for t in o.values():
                    t.zero_()
            torch.cuda.synchronize()
            rep.run(2)  # batches 0, 1
            assert not cpu(outs[2]["status"]).any() and not cpu(outs[2]["ip"]).any()
            rep.run(1, timed=True)  # batch 2: the rotation continues
            assert rep.span() > 0
            rep.close()
            for w, o in zip(want, outs):
                assert np.array_equal(cpu(o["ip"]), w[0]) and np.array_equal(cpu(o["l4"]), w[1])
                assert np.array_equal(cpu(o["status"]), w[2])
    finally:
        mi.set_busy_wait(False)
    # finalize op: one pass per batch over fresh TX seeds == the oracle's finalize
    b1 = synth.build_ipv4_batch(n, L, stride=stride, first_off=first, seed=77)
    ref = b1["buf"].copy()
    ORC.ipv4_finalize_batch(ref, n, stride=stride, first_off=first, fixed_flen=L)
    buf = dev_tensor(b1["buf"])
    fb = mi.PktBatch(buf, n, stride=stride, first_off=first, fixed_len=L)
    rep = mi.VerifyRepeat([fb], None, nstreams=2, op="finalize")
    rep.run(1)
    rep.close()
    assert np.array_equal(cpu(buf), ref)


@pytest.mark.parametrize("seed", range(24))
def test_verify_random_sweep(seed):
    """Seeded random RX batches beyond the golden vectors: packet count,
    lengths (uniform 20-9000 B or heavy-tailed), placement (fixed slots at a
    random first offset, packed, shuffled, gappy), protocol and IP header
    length per packet, then random single-byte corruptions and truncated
    lengths.  ipv4_verify (and for every third seed the repeat handle's AQL
    engine when the plan is one launch per pass, for every fourth u32
    offsets) against the oracle: ip / l4 / status bit for bit."""
    rng = np.random.default_rng(5000 + seed)
    n = int(rng.integers(1, 3000))
    if rng.random() < 0.5:
        lens = rng.integers(20, int(rng.choice([128, 1500, 9000])) + 1, n)
    else:
        lens = np.minimum(synth.pareto_lengths(n, seed=seed + 1), 9000)
    lens = np.maximum(lens, 20).astype(np.int64)
    proto = rng.choice([6, 17, 6, 17, 1], n)
    hl = np.minimum(rng.choice([20, 20, 20, 24, 40, 60], n), lens & ~3)
    layout = str(rng.choice(["slots", "packed", "shuffled", "gappy"]))
    if layout == "slots":
        stride = int(lens.max()) + int(rng.integers(0, 300))
        first = int(rng.integers(0, 200))
        b0 = synth.build_ipv4_batch(n, lens, stride=stride, first_off=first, seed=seed, proto=proto, hl=hl)
        offs = (first + np.arange(n, dtype=np.int64) * stride).astype(np.uint64)
    else:
        offs = synth.packed_offsets(lens, first_off=int(rng.integers(0, 64)))
        if layout == "gappy":
            offs = offs + np.cumsum(rng.integers(0, 400, n)).astype(np.uint64)
        b0 = synth.build_ipv4_batch(n, lens, offs=offs.astype(np.int64), seed=seed, proto=proto, hl=hl)
    _, ref = aligned(b0["buf"])
    ORC.ipv4_finalize_batch(ref, n, offs=offs, flen=lens.astype(np.uint32))
    k = int(rng.integers(0, max(1, n // 10) + 1))
    if k:
        bad = rng.choice(n, k, replace=False)
        at = offs[bad].astype(np.int64) + rng.integers(0, 1 << 30, k) % lens[bad]
        ref[at] ^= rng.integers(1, 256, k).astype(np.uint8)
    flen = lens.astype(np.uint32).copy()
    cut = rng.choice(n, int(rng.integers(0, max(1, n // 20) + 1)), replace=False)
    flen[cut] = rng.integers(0, 40, cut.size).astype(np.uint32) % np.maximum(flen[cut], 1)  # truncated frames
    perm = rng.permutation(n) if layout == "shuffled" else np.arange(n)
    o2, l2 = offs[perm], flen[perm]
    ip_o, l4_o, st_o = ORC.ipv4_verify_batch(ref, n, offs=o2, flen=l2)
    buf = dev_tensor(ref)
    use32 = seed % 4 == 0 and int(o2.max()) < (1 << 32)
    b = mi.PktBatch(buf, n, offs=dev_tensor(o2.astype(np.int64)),
                    lens=dev_tensor(l2.astype(np.int32)), packed=layout != "slots", offs32=use32)
    r = mi.ipv4_verify(b, bad_count=True)
    assert np.array_equal(cpu(r["ip"]), ip_o), (seed, layout)
    assert np.array_equal(cpu(r["l4"]), l4_o), (seed, layout)
    assert np.array_equal(cpu(r["status"]), st_o), (seed, layout)
    assert int(r["bad"].item()) == int((st_o != 0).sum()), (seed, layout)
    # (length-class plans take several launches per pass: HIP engine only, -ENOTSUP by design)
    if seed % 3 == 0 and "length classes" not in mi.verify_plan(b):
        out = dict(ip=torch.zeros(n, dtype=torch.uint16, device="cuda"), l4=torch.zeros(n, dtype=torch.uint16, device="cuda"),
                   status=torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda"))
        torch.cuda.synchronize()
        rep = mi.VerifyRepeat([b], [out], nstreams=1, engine="aql")
        try:
            rep.run(2)
        finally:
            rep.close()
        assert np.array_equal(cpu(out["ip"]), ip_o), seed
        assert np.array_equal(cpu(out["l4"]), l4_o), seed
        assert np.array_equal(cpu(out["status"]), st_o), seed


@pytest.mark.parametrize("seed", range(12))
def test_finalize_random_sweep(seed):
    """TX finalize in place (in_delayed_cksum + ip_sum) on seeded random
    batches: slots or packed / gappy offsets, lengths 20-9000 B, TCP / UDP /
    ICMP / others, IP options, truncated available lengths, with and without
    MI_BATCH_DEMUX (the small-header senders and fragments).  The whole
    buffer after the GPU pass equals the oracle's, bytes between datagrams
    included."""
    rng = np.random.default_rng(7000 + seed)
    n = int(rng.integers(1, 2000))
    lens = np.maximum(rng.integers(20, int(rng.choice([200, 1500, 9000])) + 1, n), 20).astype(np.int64)
    proto = rng.choice([6, 17, 6, 17, 1, 2, 112, 47], n)
    hl = np.minimum(rng.choice([20, 20, 20, 24, 40, 60], n), lens & ~3)
    demux = bool(seed % 2)
    layout = str(rng.choice(["slots", "packed", "gappy"]))
    if layout == "slots":
        stride = int(lens.max()) + int(rng.integers(0, 200))
        first = int(rng.integers(0, 100))
        b0 = synth.build_ipv4_batch(n, lens, stride=stride, first_off=first, seed=seed, proto=proto, hl=hl)
        offs = (first + np.arange(n, dtype=np.int64) * stride).astype(np.uint64)
    else:
        offs = synth.packed_offsets(lens, first_off=int(rng.integers(0, 64)))
        if layout == "gappy":
            offs = offs + np.cumsum(rng.integers(0, 300, n)).astype(np.uint64)
        b0 = synth.build_ipv4_batch(n, lens, offs=offs.astype(np.int64), seed=seed, proto=proto, hl=hl)
    frag = rng.random(n) < 0.05  # fragments: MF or an offset
    for i in np.nonzero(frag)[0]:
        b0["buf"][int(offs[i]) + 6] = int(rng.choice([0x20, 0x00, 0x21]))
        b0["buf"][int(offs[i]) + 7] = int(rng.integers(1, 256))
    flen = lens.astype(np.uint32).copy()
    cut = rng.choice(n, int(rng.integers(0, max(1, n // 20) + 1)), replace=False)
    flen[cut] = (flen[cut] * rng.random(cut.size)).astype(np.uint32)
    _, want = aligned(b0["buf"])
    ORC.ipv4_finalize_batch(want, n, offs=offs, flen=flen, demux=demux)
    buf = dev_tensor(b0["buf"])
    b = mi.PktBatch(buf, n, offs=dev_tensor(offs.astype(np.int64)), lens=dev_tensor(flen.astype(np.int32)),
                    packed=layout == "packed", demux=demux)
    mi.ipv4_finalize(b)
    got = cpu(buf)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (seed, layout, demux, bad.size, bad[:8])
