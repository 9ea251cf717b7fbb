"""The LDS-DMA flat-run kernel (k_ipv4_verify_run_dma<U, R>) against the oracle.

The packed-layout parity cases of test_gpu_parity / test_demux_gpu /
test_aql_gpu run again with each compiled ring shape chosen through
mi_cksum_set_run_kernel (the register flat-run kernel is the default), so every
shape is bit-exact on the golden vectors, on gappy / shuffled / u32-offset
layouts, on RX offload flags, under the AQL engine, and on the full 2^22
Pareto batch.  The shapes differ in how far ahead the ring runs (R - 1 passes
of 64 U chunks), so the small golden batches and the big one between them
cover the ring's wrap, its stall when the next range's descriptors are late,
and ranges shorter than the lookahead.
"""
import pytest

import libunsod_amd as mi

import test_aql_gpu as aql
import test_demux_gpu as demux
import test_gpu_parity as par

pytestmark = pytest.mark.gpu

SHAPES = [(2, 3), (2, 4), (4, 2), (4, 3)]


@pytest.fixture(params=SHAPES, ids=lambda s: "%dx%d" % s)
def dma_shape(request):
    mi.set_run_kernel(*request.param)
    try:
        yield request.param
    finally:
        mi.set_run_kernel(0, 0)


def test_plan_names_the_dma_kernel(dma_shape):
    import torch
    buf = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    offs = torch.arange(100, dtype=torch.int64, device="cuda") * 300
    lens = torch.full((100,), 280, dtype=torch.int32, device="cuda")
    assert mi.verify_plan(mi.PktBatch(buf, 100, offs=offs, lens=lens, packed=True)) == \
        "k_ipv4_verify_run_dma<%d,%d>" % dma_shape


def test_packed_golden(golden, dma_shape):
    par.test_packed_layout_golden(golden)


@pytest.mark.parametrize("layout", ["packed", "shuffled", "gappy"])
def test_any_layout(layout, dma_shape):
    par.test_packed_hint_any_layout(layout)


@pytest.mark.parametrize("layout", ["packed", "shuffled", "gappy"])
def test_offs32(golden, layout, dma_shape):
    par.test_offs32_same_results(golden, layout)


def test_pareto_mixed(dma_shape):
    par.test_pareto_mixed(True)


def test_rx_offload(dma_shape):
    par.test_rx_offload_flags("packed")


def test_demux_golden(demux_golden, dma_shape):
    demux.test_demux_verify_golden(demux_golden, "packed")


def test_aql_engine(dma_shape):
    aql.test_aql_every_plan_bit_exact("packed")


def test_full_size_pareto(dma_shape):
    par.test_full_size_pareto_and_shards()
