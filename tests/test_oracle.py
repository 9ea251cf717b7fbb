"""The CPU oracle is pinned before it is trusted (CPU-only tests).

* tests/golden/cksum_golden.npz was produced by the reference's own compiled
  in_cksum.c (tests/golden/make_golden.py); the restatement
  (oracle/cksum_oracle.c) must reproduce every vector bit for bit.
* SURVEY.md 8(a) known answers.
* A third, numpy statement of the closed-form contract (SURVEY.md 8 "Contract").
* When oracle/_ref/libref.so is present (built from /root/reference), fresh
  random cases restatement-vs-reference.
"""
import numpy as np
import pytest

from conftest import aligned, chain_segments
from oracle.pyoracle import Oracle, available

PORT = Oracle("port")


def contract_stream(data: bytes, seed: int = 0) -> int:
    """~fold(seed + sum b[i] << 8*(i&1)) -- SURVEY.md 8 Contract, in numpy."""
    b = np.frombuffer(data, np.uint8).astype(np.uint64)
    s = int(b[0::2].sum()) + (int(b[1::2].sum()) << 8) + seed
    if s == 0:
        f = 0
    else:
        f = 1 + (s - 1) % 65535
    return ~f & 0xFFFF


# ------------------------------------------------------------------ KATs
RFC = bytes([0x00, 0x01, 0xF2, 0x03, 0xF4, 0xF5, 0xF6, 0xF7])
HDR = bytes.fromhex("450000730000400040110000c0a80001c0a800c7")
PAT = bytes(i & 0xFF for i in range(65536 + 64))


def le32(b):
    return int.from_bytes(bytes(b), "little")


@pytest.mark.parametrize("kind", ["port", "reference"])
def test_kats(kind):
    if not available(kind):
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    o = PORT if kind == "port" else Oracle(kind)
    assert o.chain_skip([(RFC, 0)], 8, 0) == 0x0D22                            # KAT1
    assert o.in_cksum_hdr(HDR, 0) == 0x61B8                                     # KAT2
    assert o.in_cksum_hdr(HDR, 2) == 0x61B8                                     # KAT3
    assert o.in_cksum_hdr(HDR, 1) == 0xB861                                     # KAT4 quirk
    assert o.chain_skip([(HDR, 1)], 20, 0) == 0x61B8
    assert o.chain_skip([(bytes(1500), 0)], 1500, 0) == 0xFFFF                 # KAT5
    assert o.chain_skip([(b"\xff" * 1500, 0)], 1500, 0) == 0x0000              # KAT6
    for L, r in [(1, 0xFFFF), (2, 0xFEFF), (3, 0xFEFD), (63, 0x3B1C), (64, 0xFC1B), (1500, 0x4E39),
                 (1501, 0x4D5D), (9000, 0xB739), (65535, 0x3EC1), (65536, 0x3FC0)]:   # KAT7
        assert o.chain_skip([(PAT[:L], 0)], L, 0) == r, L
    for L, r in [(1, 0xFFFE), (64, 0xDBFB), (1500, 0x5D4D), (9000, 0x11B7), (65536, 0xC03F)]:  # KAT7b
        assert o.chain_skip([(PAT[1:L + 1], 1)], L, 0) == r, L
    src, dst = le32([192, 168, 1, 1]), le32([192, 168, 1, 2])
    assert o.chain_pseudo([(PAT[:1500], 0)], 1480, 20, src, dst, 6) == 0x900A    # KAT8
    assert o.chain_pseudo([(PAT[:9000], 0)], 8980, 20, src, dst, 17) == 0xA1ED   # KAT9
    assert o.in_pseudo(src, dst, le32((20 + 6 + 1460).to_bytes(4, "big"))) == 0x2289  # KAT10
    assert o.chain_skip([(PAT[:701], 0), (PAT[701:1500], 1)], 1500, 0) == 0x4E39      # KAT11
    assert o.chain_skip([(PAT[:1500], 0)], 1500, 20) == 0xB293                   # KAT12


# ------------------------------------------------------- golden vectors (port)
def test_golden_skip(golden):
    g = golden
    bad = []
    for k in range(len(g["sk_result"])):
        segs = chain_segments(g, int(g["sk_seg0"][k]), int(g["sk_nseg"][k]))
        r = PORT.chain_skip(segs, int(g["sk_len"][k]), int(g["sk_skip"][k]))
        if r != int(g["sk_result"][k]):
            bad.append(k)
    assert not bad, f"{len(bad)} skip mismatches, first {bad[:5]}"


def test_golden_pseudo(golden):
    g = golden
    bad = []
    for k in range(len(g["ps_result"])):
        segs = chain_segments(g, int(g["ps_seg0"][k]), int(g["ps_nseg"][k]))
        r = PORT.chain_pseudo(segs, int(g["ps_plen"][k]), int(g["ps_off0"][k]), int(g["ps_src"][k]),
                              int(g["ps_dst"][k]), int(g["ps_proto"][k]))
        if r != int(g["ps_result"][k]):
            bad.append(k)
    assert not bad, f"{len(bad)} pseudo mismatches, first {bad[:5]}"


def test_golden_hdr(golden):
    g = golden
    for k in range(len(g["hd_result"])):
        off = int(g["hd_off"][k])
        assert PORT.in_cksum_hdr(g["blob"][off:off + 20].tobytes(), int(g["hd_mod"][k])) == int(g["hd_result"][k])


def test_golden_scalars(golden):
    g = golden
    for a, b, c, r in zip(g["ip_a"], g["ip_b"], g["ip_c"], g["ip_result"]):
        assert PORT.in_pseudo(int(a), int(b), int(c)) == int(r)
    for a, b, r in zip(g["aw_a"], g["aw_b"], g["aw_result"]):
        assert PORT.in_addword(int(a), int(b)) == int(r)


def test_golden_verify_finalize(golden):
    g = golden
    n = len(g["vb_offs"])
    _, fin = aligned(g["fin_in"])
    PORT.ipv4_finalize_batch(fin, n, offs=g["vb_offs"], flen=g["vb_flen"])
    assert np.array_equal(fin, g["fin_out"])
    _, ver = aligned(g["ver_in"])
    ip, l4, st = PORT.ipv4_verify_batch(ver, n, offs=g["vb_offs"], flen=g["vb_flen"], nthreads=4)
    assert np.array_equal(ip, g["ver_ip"]) and np.array_equal(l4, g["ver_l4"]) and np.array_equal(st, g["ver_st"])
    assert (st & 4).any() and (st & 1).any() and (st & 2).any() and (st == 0).any()
    _, sl = aligned(g["slot_in"])
    PORT.ipv4_finalize_batch(sl, 64, stride=2176, first_off=142, fixed_flen=1500)
    assert np.array_equal(sl, g["slot_out"])


# --------------------------------------------------- contract (numpy) vs port
def test_contract_statement():
    rng = np.random.default_rng(1)
    for _ in range(300):
        n = int(rng.integers(0, 3000))
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        mod = int(rng.integers(64))
        assert PORT.chain_skip([(data, mod)], n, 0) == contract_stream(data)
        # split anywhere, any parity: still the stream sum (in_cksum.c:222-225)
        cut = int(rng.integers(0, n + 1))
        assert PORT.chain_skip([(data[:cut], mod), (data[cut:], int(rng.integers(64)))], n, 0) == contract_stream(data)
    for mod in range(8):  # in_cksum_hdr: absolute lanes
        h = rng.integers(0, 256, 20, dtype=np.uint8).tobytes()
        want = contract_stream(h)
        if mod & 1:
            want = ((want & 0xFF) << 8) | (want >> 8)
        assert PORT.in_cksum_hdr(h, mod) == want


# ----------------------------------------- restatement vs the reference itself
@pytest.mark.skipif(not available("reference"), reason="oracle/_ref not built (needs /root/reference)")
def test_port_matches_reference_random():
    ref = Oracle("reference")
    rng = np.random.default_rng(99)
    for _ in range(2000):
        nseg = int(rng.integers(1, 6))
        segs = [(rng.integers(0, 256, int(rng.integers(0, 700)), dtype=np.uint8).tobytes(), int(rng.integers(64)))
                for _ in range(nseg)]
        total = sum(len(s) for s, _ in segs)
        skip = int(rng.integers(0, total + 1))
        length = int(rng.integers(skip, total + 30))
        assert PORT.chain_skip(segs, length, skip) == ref.chain_skip(segs, length, skip)
        if len(segs[0][0]) >= 20:
            plen = int(rng.integers(0, total - 20 + 10))
            a, b = int(rng.integers(2**32)), int(rng.integers(2**32))
            p = int(rng.integers(256))
            assert PORT.chain_pseudo(segs, plen, 20, a, b, p) == ref.chain_pseudo(segs, plen, 20, a, b, p)


# ------------------------------- MI_BATCH_DEMUX (small-header callers) golden
def test_golden_demux(demux_golden):
    """tests/golden/demux_golden.npz came from the reference's in_cksum.c
    driven as ip_input's protocol input routines call it; the restatement
    reproduces every datagram (finalize bytes, verify ip / l4 / status)."""
    g = demux_golden
    n = len(g["offs"])
    _, fin = aligned(g["fin_in"])
    PORT.ipv4_finalize_batch(fin, n, offs=g["offs"], flen=g["flen"], demux=True)
    assert np.array_equal(fin, g["fin_out"])
    _, ver = aligned(g["ver_in"])
    ip, l4, st = PORT.ipv4_verify_batch(ver, n, offs=g["offs"], flen=g["flen"], demux=True, nthreads=3)
    assert np.array_equal(ip, g["ip"]) and np.array_equal(l4, g["l4"]) and np.array_equal(st, g["st"])


def test_demux_rules_statement(demux_golden):
    """A second, Python statement of the demux length / protocol rules
    (include/mi_cksum.h) agrees with the golden status bits and with the
    contract sum over each protocol's span."""
    g = demux_golden
    buf, offs, flen = g["ver_in"], g["offs"], g["flen"]
    for i in range(len(offs)):
        p, fl = int(offs[i]), int(flen[i])
        st = int(g["st"][i])
        if fl < 20 or (buf[p] & 15) * 4 < 20 or (buf[p] & 15) * 4 > fl:
            assert st == 4
            continue
        hl = (int(buf[p]) & 15) * 4
        iplen = (int(buf[p + 2]) << 8) | int(buf[p + 3])
        if iplen < hl or iplen > fl:
            assert st & 4 and int(g["l4"][i]) == 0
            continue
        plen, proto = iplen - hl, int(buf[p + 9])
        a = [int(x) for x in buf[p + 12:p + 20]]
        addr = a[0] + a[2] + a[4] + a[6] + ((a[1] + a[3] + a[5] + a[7]) << 8)
        frag = ((int(buf[p + 6]) << 8) | int(buf[p + 7])) & 0x3FFF
        d = bytes(buf[p + hl:p + iplen])
        want_l4, want_st = 0, 0
        if frag or proto not in (6, 17, 1, 2, 112):
            want_st = 8
        elif plen < {6: 20, 17: 8, 1: 36, 2: 8, 112: 36}[proto]:
            want_st = 4
        elif proto == 17:
            ulen = (d[4] << 8) | d[5]
            if ulen != plen and (ulen > plen or ulen < 8):
                want_st = 4
            elif (d[6] << 8 | d[7]) == 0:
                want_st = 8
            else:
                seed = addr + (17 << 8) + (((ulen & 0xFF) << 8) | (ulen >> 8))
                want_l4 = contract_stream(d[:ulen], seed)
        elif proto == 6:
            seed = addr + (6 << 8) + (((plen & 0xFF) << 8) | (plen >> 8))
            want_l4 = contract_stream(d, seed)
        else:
            want_l4 = contract_stream(d[:36] if proto == 112 else d)
        assert int(g["l4"][i]) == want_l4, i
        ip_bad = 1 if int(g["ip"][i]) else 0
        assert st == want_st | ip_bad | (2 if want_l4 else 0), i
