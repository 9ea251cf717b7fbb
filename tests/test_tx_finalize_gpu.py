"""TX finalize in place (in_delayed_cksum ip_output.c:958-983 + ip_sum
:667-672) through the whole-64-byte-block store path (k_ipv4_finalize<BLOCKS>):
every slot phase (first_off % 64), IP options up to hl 60 (L4 field beyond
chunk G: byte-store fallback), TCP / UDP / other protocols, short datagrams
whose blocks run past the envelope, per-packet lens under a max_len hint and
lens beyond it, MI_BATCH_DEMUX small-header senders.  The whole buffer must
equal the oracle's finalize byte for byte -- which also proves that the
rewritten bytes around each datagram are unchanged."""
import os

import numpy as np
import pytest
import torch


import libunsod_amd as mi
from conftest import aligned
from libunsod_amd import synth
from oracle.pyoracle import Oracle

pytestmark = pytest.mark.gpu
ORC = Oracle("port")


@pytest.fixture(autouse=True, params=["blocks", "bytes"])
def tx_store_mode(request, monkeypatch):
    """Both store schemes (the library reads MI_CKSUM_TX_BLOCKS per launch)."""
    monkeypatch.setenv("MI_CKSUM_TX_BLOCKS", "1" if request.param == "blocks" else "0")
    return request.param


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def finalize_both(host, n, *, stride, first_off, flen, fixed, max_len=0, demux=False):
    _, ref = aligned(host.copy())
    if fixed:
        ORC.ipv4_finalize_batch(ref, n, stride=stride, first_off=first_off, fixed_flen=int(flen[0]), demux=demux)
    else:
        offs = (first_off + np.arange(n, dtype=np.uint64) * stride).astype(np.uint64)
        ORC.ipv4_finalize_batch(ref, n, offs=offs, flen=flen.astype(np.uint32), demux=demux)
    buf = dev(host)
    if fixed:
        b = mi.PktBatch(buf, n, stride=stride, first_off=first_off, fixed_len=int(flen[0]), demux=demux)
    else:
        b = mi.PktBatch(buf, n, stride=stride, first_off=first_off, lens=dev(flen.astype(np.int32)),
                        max_len=max_len, demux=demux)
    mi.ipv4_finalize(b)
    torch.cuda.synchronize()
    return buf.cpu().numpy(), ref


@pytest.mark.parametrize("phase", [0, 2, 6, 13, 14, 15, 16, 30, 47, 63])
@pytest.mark.parametrize("L", [1500, 333])
def test_blocks_every_phase(phase, L):
    n, stride = 512, 2176
    first = 128 + phase
    rng = np.random.default_rng(phase * 7 + L)
    proto = rng.choice([6, 17, 6, 1], n)
    hl = rng.choice([20, 20, 20, 24, 40, 60], n)
    b0 = synth.build_ipv4_batch(n, L, stride=stride, first_off=first, proto=proto, hl=hl, seed=phase + 3)
    host = b0["buf"]
    # non-zero bytes around the datagrams (the blocks' outside bytes must survive)
    gap = np.ones(host.size, bool)
    for i in range(n):
        gap[first + i * stride:first + i * stride + L] = False
    host[gap] = rng.integers(0, 256, int(gap.sum()), dtype=np.uint8)
    got, ref = finalize_both(host, n, stride=stride, first_off=first, flen=np.full(n, L), fixed=True)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("demux", [False, True])
def test_blocks_mixed_lens(demux):
    """Per-packet lens in 9216 B slots: short datagrams (blocks past the
    envelope), runts, malformed headers; max_len hint exact and too small."""
    n, stride, first = 700, 9216, 142
    rng = np.random.default_rng(5 + demux)
    lens = rng.integers(20, 9001, n)
    lens[:40] = rng.integers(20, 120, 40)
    proto = rng.choice([6, 17, 1, 2, 112, 50], n)
    hl = rng.choice([20, 20, 28, 60], n)
    b0 = synth.build_ipv4_batch(n, lens, stride=stride, first_off=first, proto=proto, hl=hl, seed=11)
    host = b0["buf"]
    host[first + 3 * stride] = 0x43  # hl 12: malformed
    host[first + 4 * stride + 2:first + 4 * stride + 4] = [0xFF, 0xFF]  # ip_len > flen
    for max_len in (int(lens.max()), 64):
        got, ref = finalize_both(host, n, stride=stride, first_off=first, flen=lens, fixed=False,
                                 max_len=max_len, demux=demux)
        assert np.array_equal(got, ref), max_len


def test_blocks_off_for_tight_layouts():
    """Layouts the block condition rejects (stride not a multiple of 64, slots
    too tight) still finalize exactly (byte stores)."""
    for stride, L, first in ((1504, 1500, 2), (1600, 1540, 70), (128, 96, 14)):
        n = 300
        b0 = synth.build_ipv4_batch(n, L, stride=stride, first_off=first, seed=stride)
        got, ref = finalize_both(b0["buf"], n, stride=stride, first_off=first, flen=np.full(n, L), fixed=True)
        assert np.array_equal(got, ref), stride
