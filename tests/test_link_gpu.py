"""Link-time substitution.

oracle/_ref/linktest is a kernel-side caller compiled with the reference's own
headers and kernel flags (-nostdinc -D_KERNEL, <machine/in_cksum.h>
src/sys/amd64/include/in_cksum.h:77-83; recipe in oracle/Makefile) and linked
against libmicksum.so where libuinet links in_cksum.o (MACHINE_SRCS,
src/lib/libuinet/Makefile:275-276).  Built in the dev container (it needs
/root/reference); the prebuilt binary travels to the GPU box.
"""
import json
import os
import subprocess

import pytest

from conftest import ROOT

BIN = os.path.join(ROOT, "oracle", "_ref", "linktest")
OBJ = os.path.join(ROOT, "oracle", "_ref", "kat_kernel.o")
ABI = {"in_cksum_skip", "in_cksum_pseudo_header", "in_cksum_hdr", "in_pseudo", "in_addword"}


@pytest.mark.skipif(not os.path.exists(OBJ), reason="kernel-side caller not built (needs /root/reference)")
def test_kernel_side_object_needs_only_the_abi():
    """The kernel-side object's only external references are the five
    checksum entry points: exactly what in_cksum.o resolved for it."""
    out = subprocess.run(["nm", "-u", OBJ], capture_output=True, text=True, check=True).stdout
    undef = {ln.split()[-1] for ln in out.splitlines() if ln.strip()} - {"_GLOBAL_OFFSET_TABLE_"}
    assert undef == ABI


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(BIN), reason="linktest not built (needs /root/reference at build time)")
def test_linked_kernel_caller_kats():
    p = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    res = json.loads(p.stdout)
    assert res["failed"] == 0 and res["kats"] == 28
