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


OFFLOAD_BIN = os.path.join(ROOT, "oracle", "_ref", "offload_test")
OFFLOAD_OBJ = os.path.join(ROOT, "oracle", "_ref", "offload_kernel.o")


@pytest.mark.skipif(not os.path.exists(OFFLOAD_OBJ), reason="offload contract object not built (needs /root/reference)")
def test_offload_contract_object():
    """oracle/linktest/offload_kernel.c compiled with the reference's headers
    and kernel flags -- its static asserts pin include/mi_cksum_flags.h (the
    CSUM_* values, m_pkthdr.csum_flags / csum_data offsets and widths) to
    src/sys/sys/mbuf.h -- and its only checksum calls go to the reference's own
    in_cksum.c (ref_*): the software branch the offload is compared with."""
    out = subprocess.run(["nm", "-u", OFFLOAD_OBJ], capture_output=True, text=True, check=True).stdout
    undef = {ln.split()[-1] for ln in out.splitlines() if ln.strip()} - {"_GLOBAL_OFFSET_TABLE_", "bzero"}
    assert undef == {"ref_in_cksum_hdr", "ref_in_cksum_pseudo_header", "ref_in_cksum_skip", "ref_in_pseudo"}


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(OFFLOAD_BIN), reason="offload_test not built (needs /root/reference at build time)")
def test_offload_decisions_match_reference(tmp_path, demux_golden):
    """VERDICT r2 "do this" 2: a GPU burst of the 720 mixed-protocol golden
    datagrams (TCP / UDP / ICMP / IGMP / CARP / other, IP options, fragments,
    bad sums, short and malformed headers) through mi_cksum_rx_offload_host;
    INTEGRATION.md section 2's hook stores the flags into real struct mbufs of
    the reference's definition; ip_input / tcp_input / udp_input's consume
    expressions (th_sum = csum_data ^ 0xffff) give the same accept/drop
    decision, and the same tested sum, as the reference's own
    in_cksum_hdr / in_cksum / in_cksum_pseudo_header on the same mbufs --
    zero-copy and staged transports both."""
    import numpy as np
    g = demux_golden
    buf, offs, flen = g["ver_in"], g["offs"].astype(np.uint64), g["flen"].astype(np.uint32)
    p = tmp_path / "burst.bin"
    with open(p, "wb") as f:
        f.write(np.array([0x424F494D, len(offs)], np.uint32).tobytes())
        f.write(np.array([buf.size], np.uint64).tobytes())
        f.write(buf.tobytes())
        f.write(offs.tobytes())
        f.write(flen.tobytes())
    r = subprocess.run([OFFLOAD_BIN, str(p)], capture_output=True, text=True, timeout=120)
    assert r.stdout.strip(), r.stderr
    res = json.loads(r.stdout)
    print(json.dumps(res))
    assert r.returncode == 0, res
    for leg in ("zero_copy", "staged"):
        x = res[leg]
        assert x["datagrams"] == 720
        assert x["decision_mismatch"] == 0 and x["l4_value_mismatch"] == 0, x
        assert x["ip_from_flags"] == 720 and x["l4_from_csum_data"] > 250, x
        # the burst exercises accepts and both kinds of checksum drop
        assert x["decisions"][0] > 0 and x["decisions"][4] > 0 and x["decisions"][8] > 0, x
