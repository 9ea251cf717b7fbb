"""TX copy + checksum offload: the CPU oracle.

The restatement (oracle/_build) must agree with the reference's own in_cksum.c
(oracle/_ref) on every case, and a frame it produces must verify to 0/0 with
the RX path (ip_input + tcp_input sums over the copy)."""
import numpy as np
import pytest

from oracle.pyoracle import Oracle, available
from tx_cases import edge_cases, make_case, run_oracle

PORT = Oracle("port")


@pytest.mark.skipif(not available("reference"), reason="oracle/_ref/libref.so not built")
def test_tx_port_equals_reference():
    ref = Oracle("reference")
    for name, c in edge_cases(PORT):
        d1, s1 = run_oracle(PORT, c)
        d2, s2 = run_oracle(ref, c)
        assert np.array_equal(s1, s2), name
        assert np.array_equal(d1, d2), name


def test_tx_frames_verify():
    c = make_case(64, np.random.default_rng(3).integers(40, 1500, 64), layout="random", seed=3)
    dst, st = run_oracle(PORT, c)
    assert set(np.unique(st)) <= {0, 8}  # 8: the IP mbuf was cut short of the L4 sum field
    ip, l4, vs = PORT.ipv4_verify_batch(dst, 64, stride=c["stride"], first_off=c["dst_first"] + c["l3"],
                                        flen=c["pkt_len"] - c["l3"])
    assert not ip.any()
    assert np.array_equal(vs != 0, st == 8) and (st == 0).sum() > 32


def test_tx_status_rules():
    cases = dict(edge_cases(PORT))
    _, st = run_oracle(PORT, cases["short-nobufs-malformed"])
    assert st[3] == 2 and st[5] == 1 and st[7] == 4 and st[9] == 4
    assert not np.delete(st, [3, 5, 7, 9]).any()
    c = cases["flags-and-data"]
    _, st = run_oracle(PORT, c)
    big = (c["data"] + 20 + 2 > 40) & ((c["flags"] & 6) != 0)  # the header mbuf holds IP + TCP = 40 B
    assert np.array_equal(st == 8, big)  # the sum field beyond the IP mbuf: "delayed m_pullup"


@pytest.mark.parametrize("name", ["eth-padding", "eth-padding-socket", "l3-64-hl-60", "ragged-count-mixed"])
def test_tx_new_cases_verify(name):
    """The padded / far-header / ragged cases are summed (status 0 where the
    IP mbuf holds the L4 field) and their frames verify to 0/0."""
    c = dict(edge_cases(PORT))[name]
    dst, st = run_oracle(PORT, c)
    n = len(c["pkt_len"])
    assert set(np.unique(st)) <= {0, 8} and (st == 0).sum() >= n // 2
    flen = c["pkt_len"].astype(np.int64) - c["l3"]
    ip, l4, vs = PORT.ipv4_verify_batch(dst, n, stride=c["stride"], first_off=c["dst_first"] + c["l3"], flen=flen)
    assert not ip.any()
    assert np.array_equal(vs != 0, st == 8)
    if name.startswith("eth-padding"):
        ip_len = np.array([int(f[c["l3"] + 2]) << 8 | int(f[c["l3"] + 3]) for f in c["frames"]])
        assert (ip_len < flen).sum() >= n // 2  # padding really follows most datagrams


def test_tx_zero_udp_sum_stored_as_ffff():
    c = dict(edge_cases(PORT))["zero-udp-sum"]
    dst, st = run_oracle(PORT, c)
    assert not st.any()
    for i in range(len(c["pkt_len"])):
        p = c["dst_first"] + i * c["stride"] + c["l3"] + 20 + 6
        assert dst[p] == 0xFF and dst[p + 1] == 0xFF
