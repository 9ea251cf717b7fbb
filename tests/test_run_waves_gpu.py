"""The flat-run verify kernel with 1- and 2-wave workgroups
(k_ipv4_verify_packed<U, 0, NW>, MI_CKSUM_RUN_WAVES) against the oracle.

Each wave owns its own 64-datagram ranges whatever the workgroup size, so the
results must not move; the packed / dense-slot parity cases of
test_gpu_parity, test_demux_gpu and test_aql_gpu run again with every
workgroup size (the AQL engine dispatches the mi_aql_run<U>w<NW> entry points
with 64- and 128-lane workgroups), and the full 2^22 Pareto batch too.
"""
import ctypes as C

import pytest

import libunsod_amd as mi

import test_aql_gpu as aql
import test_demux_gpu as demux
import test_gpu_parity as par

pytestmark = pytest.mark.gpu


def _set_waves(w):
    lib = mi.load()
    lib.mi__set_run_waves.restype = C.c_int
    lib.mi__set_run_waves.argtypes = [C.c_int]
    assert lib.mi__set_run_waves(w) == 0


@pytest.fixture(params=[1, 4], ids=lambda w: f"{w}wave")
def run_waves(request):
    _set_waves(request.param)
    try:
        yield request.param
    finally:
        _set_waves(2)


def test_plan_names_the_workgroup(run_waves):
    import torch
    buf = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    offs = torch.arange(100, dtype=torch.int64, device="cuda") * 300
    lens = torch.full((100,), 280, dtype=torch.int32, device="cuda")
    want = "k_ipv4_verify_packed<8>" if run_waves == 4 else "k_ipv4_verify_packed<8,%d waves>" % run_waves
    assert mi.verify_plan(mi.PktBatch(buf, 100, offs=offs, lens=lens, packed=True)) == want


def test_packed_golden(golden, run_waves):
    par.test_packed_layout_golden(golden)


@pytest.mark.parametrize("layout", ["packed", "shuffled", "gappy"])
def test_any_layout(layout, run_waves):
    par.test_packed_hint_any_layout(layout)


@pytest.mark.parametrize("layout", ["packed", "shuffled", "gappy"])
def test_offs32(golden, layout, run_waves):
    par.test_offs32_same_results(golden, layout)


def test_pareto_mixed(run_waves):
    par.test_pareto_mixed(True)


def test_rx_offload(run_waves):
    par.test_rx_offload_flags("packed")


def test_demux_golden(demux_golden, run_waves):
    demux.test_demux_verify_golden(demux_golden, "packed")


def test_aql_engine(run_waves):
    aql.test_aql_every_plan_bit_exact("packed")


def test_full_size_pareto(run_waves):
    par.test_full_size_pareto_and_shards()
