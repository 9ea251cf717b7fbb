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
@pytest.mark.parametrize("mode", ["host", "gpu"])
def test_linked_kernel_caller_kats(mode):
    """All 28 SURVEY.md 8(a) known answers through the kernel-side caller, served
    by the host fold (the default) and by the GPU drop-in service -- in GPU mode
    none of them by the host fold after a GPU error (degraded == 0)."""
    p = subprocess.run([BIN], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, MI_CKSUM_DROPIN=mode))
    assert p.returncode == 0, p.stdout + p.stderr
    res = json.loads(p.stdout)
    assert res["failed"] == 0 and res["kats"] == 28
    assert res["mode"] == mode and res["degraded"] == 0


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


# ---------------------------------------------------------------- TX (2b)
TX_BIN = os.path.join(ROOT, "oracle", "_ref", "tx_test")
TX_OBJ = os.path.join(ROOT, "oracle", "_ref", "tx_kernel.o")
TXC_IN, TXC_NOT_IP, TXC_SHORT, TXC_NOBUFS = 0, 1, 2, 3


def _tx_case_file(path, c):
    """tx_main.c's input: a tests/tx_cases.py case (flags given without data
    get the csum_data the library assumes by flag, tcp_output.c:1066 /
    udp_usrreq.c:1240)."""
    import numpy as np
    n = len(c["pkt_len"])
    fl, da = c["flags"], c["data"]
    if fl is not None and da is None:
        da = np.where(np.asarray(fl) & 2, 16, 6).astype(np.uint32)
    with open(path, "wb") as f:
        f.write(np.array([0x5854494D, n, len(c["seg_off"]), c["l3"], c["room"], fl is not None, da is not None, 0],
                         np.uint32).tobytes())
        f.write(np.array([c["src"].size, c["dst"].size, c["stride"], c["dst_first"]], np.uint64).tobytes())
        f.write(c["src"].tobytes())
        f.write(np.asarray(c["seg_off"], np.uint64).tobytes())
        f.write(np.asarray(c["seg_len"], np.int32).tobytes())
        f.write(np.asarray(c["pkt_seg"], np.uint32).tobytes())
        f.write(np.asarray(c["pkt_len"], np.uint32).tobytes())
        if fl is not None:
            f.write(np.asarray(fl, np.uint32).tobytes())
        if da is not None:
            f.write(np.asarray(da, np.uint32).tobytes())
        f.write(c["dst"].tobytes())


def _tx_cases():
    from oracle.pyoracle import Oracle
    from tx_cases import edge_cases
    return edge_cases(Oracle("port"))


@pytest.mark.skipif(not os.path.exists(TX_OBJ), reason="TX contract object not built (needs /root/reference)")
def test_tx_contract_object():
    """oracle/linktest/tx_kernel.c compiled with the reference's headers and
    kernel flags: its static asserts pin include/mi_cksum_flags.h's TX values
    (CSUM_IP / TCP / UDP, CSUM_DELAY_DATA / _IP, and the csum_data defaults =
    offsetof(struct tcphdr, th_sum) / offsetof(struct udphdr, uh_sum)) to
    mbuf.h / tcp.h / udp.h, and its only checksum call goes to the reference's
    own in_cksum.c (ref_in_cksum_skip: in_delayed_cksum and in_cksum(m, hlen))."""
    out = subprocess.run(["nm", "-u", TX_OBJ], capture_output=True, text=True, check=True).stdout
    undef = {ln.split()[-1] for ln in out.splitlines() if ln.strip()} - {"_GLOBAL_OFFSET_TABLE_"}
    assert undef == {"ref_in_cksum_skip", "bcopy", "bzero"}


@pytest.mark.skipif(not os.path.exists(TX_BIN), reason="tx_test not built (needs /root/reference at build time)")
def test_tx_reference_route_pins_the_restatement(tmp_path):
    """CPU: the reference-header software route (real struct mbufs through
    ip_output.c:649-672 + in_delayed_cksum with the reference's in_cksum.c,
    then m_copydata into the slots) against oracle/batch_driver.c's restated
    tx_copy_batch, which test_tx_gpu.py compares the GPU with: identical slot
    bytes for every frame ip_output takes (ip_output always adds CSUM_IP, so the
    restatement gets the flags with it), every case of tests/tx_cases.py."""
    import numpy as np
    from oracle.pyoracle import Oracle
    orc = Oracle("port")
    totals = dict(through_ip_output=0, l4_gave_up=0, udp_zero_to_ffff=0, not_ip_output_input=0)
    for name, c in _tx_cases():
        p, o = tmp_path / f"{name}.bin", tmp_path / f"{name}.out"
        _tx_case_file(p, c)
        r = subprocess.run([TX_BIN, str(p), "--software", str(o)], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr
        res = json.loads(r.stdout)
        for k in totals:
            totals[k] += res[k]
        n = len(c["pkt_len"])
        raw = np.fromfile(o, np.uint8)
        sw = raw[:c["dst"].size]
        cls = raw[c["dst"].size:].view(np.int32)[:n]
        fl = c["flags"]
        if fl is None:
            fl = np.zeros(n, np.uint32)
            for i in range(n):  # the transports' seeding (what tx_kernel.c's default is)
                k = int(c["seg_off"][c["pkt_seg"][i]])
                proto = _frame_byte(c, i, c["l3"] + 9)
                fl[i] = 2 if proto == 6 else 4 if proto == 17 else 0
        cc = dict(c, flags=(np.asarray(fl, np.uint32) | 1))
        from tx_cases import run_oracle
        want, _ = run_oracle(orc, cc)
        keep = np.ones(c["dst"].size, bool)
        for i in np.nonzero(cls == TXC_NOT_IP)[0]:
            a = c["dst_first"] + int(i) * c["stride"]
            keep[a:a + c["room"]] = False
        bad = np.nonzero((sw != want) & keep)[0]
        assert bad.size == 0, (name, bad.size, bad[:8])
    print(totals)
    assert totals["through_ip_output"] > 500 and totals["l4_gave_up"] > 0 and totals["udp_zero_to_ffff"] > 0


def _frame_byte(c, i, q):
    """byte q of frame i, read through its chain"""
    pos = 0
    for k in range(int(c["pkt_seg"][i]), int(c["pkt_seg"][i + 1])):
        ln = int(c["seg_len"][k])
        if pos <= q < pos + ln:
            return int(c["src"][int(c["seg_off"][k]) + q - pos])
        pos += max(ln, 0)
    return -1


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(TX_BIN), reason="tx_test not built (needs /root/reference at build time)")
@pytest.mark.parametrize("kernel", ["pair", "wave", "lds"])
def test_tx_offload_matches_reference_software_route(tmp_path, kernel):
    """VERDICT r3 "do this" 1: every tests/tx_cases.py case goes out twice
    through real struct mbufs of the reference's definition -- if_hwassist = 0
    (ip_output.c:649-672 + in_delayed_cksum :958-983 with the reference's own
    in_cksum.c, then m_copydata into the rte_mbuf slots) and if_hwassist =
    CSUM_IP | CSUM_TCP | CSUM_UDP (the sums left to the device; the frames'
    descriptors read out of the mbufs go to mi_cksum_tx_copy_host on the GPU,
    zero-copy and staged).  0 wire-byte mismatches over all slot bytes, the
    in_delayed_cksum give-up (:971-981, MI_TX_L4_SKIPPED) and UDP 0 -> 0xffff
    (:967-968) exercised, each frame's status the one its route implies."""
    totals = {}
    for name, c in _tx_cases():
        p = tmp_path / f"{name}.bin"
        _tx_case_file(p, c)
        r = subprocess.run([TX_BIN, str(p)], capture_output=True, text=True, timeout=120,
                           env=dict(os.environ, MI_CKSUM_TX_KERNEL=kernel))
        assert r.stdout.strip(), r.stderr
        res = json.loads(r.stdout)
        print(kernel, name, json.dumps(res))
        assert r.returncode == 0, (name, res)
        for k in ("byte_mismatch_zero_copy", "byte_mismatch_staged", "status_mismatch_zero_copy",
                  "status_mismatch_staged"):
            assert res[k] == 0, (name, res)
        for k, v in res.items():
            if k != "first_bad_byte":
                totals[k] = totals.get(k, 0) + v
    print(json.dumps(totals))
    assert totals["through_ip_output"] > 500 and totals["l4_gave_up"] > 0 and totals["udp_zero_to_ffff"] > 0
    assert totals["short_chain"] > 0 and totals["nobufs"] > 0
