"""Host-resident batches -- the path's real start and end (DPDK mbufs in host
memory): mi_cksum_ipv4_verify_host and the driver-side RX
offload hook mi_cksum_rx_offload_host (uinet_if_dpdk.c:854-879), over both
transports (registered memory read in place over PCIe, and the staged copy
ring), with u64 and u32 (MI_BATCH_OFFS32) offsets, against the oracle and the
restated offload rules."""
import numpy as np
import pytest

import libunsod_amd as mi
from oracle.pyoracle import Oracle, rx_offload_flags
from test_gpu_parity import _rx_mix

pytestmark = pytest.mark.gpu
ORC = Oracle("port")


@pytest.mark.parametrize("offs32", [False, True])
def test_host_paths_offsets(offs32):
    n = 8000
    keep, h, o, flen = _rx_mix(n, 0x5151 + offs32)
    want = ORC.ipv4_verify_batch(h, n, offs=o.astype(np.uint64), flen=flen, nthreads=8)
    want_fl, want_cd = rx_offload_flags(h, o, flen, *want)
    nbad = int((want[2] != 0).sum())
    for registered in (True, False):
        if registered:
            mi.host_register(h)
        try:
            for staged in ((False, True) if registered else (False,)):
                ip, l4, st, bad = mi.ipv4_verify_host(h, n, offs=o, lens=flen, staged=staged, offs32=offs32)
                tag = (registered, staged, offs32)
                assert np.array_equal(ip, want[0]) and np.array_equal(l4, want[1]), tag
                assert np.array_equal(st, want[2]) and bad == nbad, tag
                fl, cd, bad = mi.rx_offload_host(h, n, offs=o, lens=flen, staged=staged, offs32=offs32)
                np.testing.assert_array_equal(fl, want_fl)
                np.testing.assert_array_equal(cd, want_cd)
                assert bad == nbad, tag
        finally:
            if registered:
                mi.host_unregister(h)


@pytest.mark.parametrize("n", [1, 64, 512, 4096])
def test_rx_offload_host_bursts(n):
    """rte_eth_rx_burst-sized bursts (<= 512, dpdk_helper.h:20; ring of 4096,
    uinet_api.c:1983) in 2176 B rte_mbuf slots, registered and staged."""
    from libunsod_amd import synth
    stride, first, L = 2176, 142, 1500
    b0 = synth.build_ipv4_batch(n, L, stride=stride, first_off=first, seed=n)
    h = mi.page_buffer(b0["buf"].size)  # registrable: pages of its own
    h[:] = b0["buf"]
    ORC.ipv4_finalize_batch(h, n, stride=stride, first_off=first, fixed_flen=L)
    h[first + (n // 2) * stride + 700] ^= 4
    want = ORC.ipv4_verify_batch(h, n, stride=stride, first_off=first, fixed_flen=L)
    o = (first + np.arange(n) * stride).astype(np.int64)
    want_fl, want_cd = rx_offload_flags(h, o, np.full(n, L), *want)
    mi.host_register(h)
    try:
        for staged in (False, True):
            fl, cd, bad = mi.rx_offload_host(h, n, stride=stride, first_off=first, fixed_len=L, staged=staged)
            np.testing.assert_array_equal(fl, want_fl)
            np.testing.assert_array_equal(cd, want_cd)
            assert bad == 1
    finally:
        mi.host_unregister(h)


def test_offs32_rejects_wide_offsets():
    import torch
    buf = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    offs = torch.tensor([0, 1 << 32], dtype=torch.int64, device="cuda")
    lens = torch.tensor([20, 20], dtype=torch.int32, device="cuda")
    with pytest.raises(ValueError):
        mi.PktBatch(buf, 2, offs=offs, lens=lens, offs32=True)
    with pytest.raises(ValueError):
        mi.ipv4_verify_host(np.zeros(4096, np.uint8), 2, offs=np.array([0, 1 << 32]), lens=np.array([20, 20]),
                            offs32=True)
