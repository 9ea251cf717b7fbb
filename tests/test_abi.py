"""The C-ABI boundary, without a GPU: libmicksum.so loads, exports every symbol
include/mi_cksum.h declares, the integer-only drop-ins match the golden
vectors, and the batch calls refuse to run without a gfx950 device (no CPU
fallback; the (b1) drop-ins' host mode is tests/test_dropin_host.py)."""
import ctypes as C
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

import libunsod_amd as mi
from libunsod_amd._lib import LIB_PATH, SIGNATURES, PktBatchC, load

HEADER = os.path.join(ROOT, "include", "mi_cksum.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"^\s*#.*$", "", src, flags=re.M)
    names = re.findall(r"\b([a-z_][a-z0-9_]*)\s*\([^;{()]*\)\s*;", src)
    return sorted(set(n for n in names if n not in ("defined",)))


def test_header_declares_reference_abi():
    names = declared_functions()
    for ref in ("in_cksum_skip", "in_cksum_pseudo_header", "in_cksum_hdr", "in_pseudo", "in_addword"):
        assert ref in names
    assert set(names) == set(SIGNATURES), set(names) ^ set(SIGNATURES)


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, missing
    lib = load()
    for n in declared_functions():
        assert getattr(lib, n) is not None


def test_struct_layouts():
    assert C.sizeof(PktBatchC) == 64
    assert PktBatchC.n.offset == 52 and PktBatchC.lens.offset == 40


def test_integer_dropins_match_golden(golden):
    g = golden
    for a, b, c, r in zip(g["ip_a"], g["ip_b"], g["ip_c"], g["ip_result"]):
        assert mi.in_pseudo(int(a), int(b), int(c)) == int(r)
    for a, b, r in zip(g["aw_a"], g["aw_b"], g["aw_result"]):
        assert mi.in_addword(int(a), int(b)) == int(r)


def test_version():
    assert "gfx950" in mi.version()


@pytest.mark.skipif(mi.device_count() > 0, reason="a GPU is present")
def test_no_cpu_fallback_batch():
    buf = np.zeros(4096, np.uint8)
    b = PktBatchC(buf.ctypes.data, buf.nbytes, None, 2176, 0, None, 64, 1, 64, 0)
    rc = load().mi_cksum_ipv4_verify(C.byref(b), None, None, None, None, None)
    assert rc == -19  # -ENODEV: never silently computed on the CPU
    assert load().mi_cksum_init(0) == -19


def test_verify_plan_needs_no_gpu():
    """The kernel choice is host logic: dense minimum-size slots and hinted
    packed layouts take the flat-run kernel (packed ones its LDS-DMA form when
    mi_cksum_set_run_kernel picks it), roomy slots the lane-group one."""
    import torch
    import libunsod_amd as mi
    buf = torch.zeros(1 << 20, dtype=torch.uint8)
    assert mi.verify_plan(mi.PktBatch(buf, 100, stride=2176, first_off=142, fixed_len=1500)).startswith("k_ipv4_verify<")
    assert mi.verify_plan(mi.PktBatch(buf, 100, stride=64, first_off=14, fixed_len=46)) == "k_ipv4_verify_slot64"
    assert mi.verify_plan(mi.PktBatch(buf, 100, stride=64, first_off=30, fixed_len=46)) == "k_ipv4_verify_packed<4,2 waves>"
    offs = torch.arange(100, dtype=torch.int64) * 300
    lens = torch.full((100,), 280, dtype=torch.int32)
    assert mi.verify_plan(mi.PktBatch(buf, 100, offs=offs, lens=lens, packed=True)) == "k_ipv4_verify_packed<8,2 waves>"
    mi.set_run_kernel(2, 4)
    try:
        assert mi.verify_plan(mi.PktBatch(buf, 100, offs=offs, lens=lens, packed=True)) == "k_ipv4_verify_run_dma<2,4>"
        with pytest.raises(Exception):
            mi.set_run_kernel(3, 3)
    finally:
        mi.set_run_kernel(0, 0)
    assert mi.verify_plan(mi.PktBatch(buf, 100, offs=offs, lens=lens)) == "k_ipv4_verify x length classes"
    assert mi.verify_plan(mi.PktBatch(buf, 100, offs=offs, lens=lens // 4)) == "k_ipv4_verify<1,8>"
