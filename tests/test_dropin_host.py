"""The (b1) drop-ins in their default mode, MI_DROPIN_HOST: served on the calling
CPU by libunsod_amd/csrc/host_fold.c ("per-call GPU dispatch is
not viable"), so they run here, without a GPU.  Bit-exact against the golden
vectors the reference's own in_cksum.c produced (tests/golden/make_golden.py),
the SURVEY.md 8(a) known answers through the kernel-side caller built with the
reference's headers, and the degrade path of the GPU mode.  Also the host
registration table's bookkeeping."""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, chain_segments

import libunsod_amd as mi
from libunsod_amd._lib import DROPIN_ERROR_FN, load


@pytest.fixture(autouse=True)
def host_mode():
    was = mi.set_dropin_mode("host")
    yield
    mi.set_dropin_mode(was)


def test_default_mode_is_host():
    code = ("import sys; sys.path.insert(0, %r); import libunsod_amd as mi; "
            "print(mi.set_dropin_mode('host'))") % ROOT
    env = {k: v for k, v in os.environ.items() if k != "MI_CKSUM_DROPIN"}
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env)
    assert p.returncode == 0 and p.stdout.strip() == "host", p.stderr
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                       env=dict(env, MI_CKSUM_DROPIN="gpu"))
    assert p.returncode == 0 and p.stdout.strip() == "gpu", p.stderr
    assert load().mi_cksum_set_dropin_mode(7) == -22


def test_skip_golden(golden):
    g = golden
    bad = [k for k in range(len(g["sk_result"]))
           if mi.in_cksum_skip(mi.MbufChain(chain_segments(g, int(g["sk_seg0"][k]), int(g["sk_nseg"][k]))),
                               int(g["sk_len"][k]), int(g["sk_skip"][k])) != int(g["sk_result"][k])]
    assert not bad, f"{len(bad)} of {len(g['sk_result'])} differ, first {bad[:5]}"


def test_pseudo_golden(golden):
    g = golden
    bad = []
    for k in range(len(g["ps_result"])):
        m = mi.MbufChain(chain_segments(g, int(g["ps_seg0"][k]), int(g["ps_nseg"][k])))
        r = mi.in_cksum_pseudo_header(m, int(g["ps_plen"][k]), int(g["ps_off0"][k]), int(g["ps_src"][k]),
                                      int(g["ps_dst"][k]), int(g["ps_proto"][k]))
        if r != int(g["ps_result"][k]):
            bad.append(k)
    assert not bad, f"{len(bad)} of {len(g['ps_result'])} differ, first {bad[:5]}"


def test_hdr_golden(golden):
    g = golden
    for k in range(len(g["hd_result"])):
        off = int(g["hd_off"][k])
        assert mi.in_cksum_hdr(g["blob"][off:off + 20].tobytes(), int(g["hd_mod"][k])) == int(g["hd_result"][k])


def test_known_answers():
    """SURVEY.md 8(a) KATs 1-12, through the Python mirror."""
    kat7 = bytes(i & 0xFF for i in range(65537))
    assert mi.in_cksum_skip(mi.MbufChain([bytes.fromhex("0001f203f4f5f6f7")]), 8, 0) == 0x0D22
    hdr = bytes.fromhex("450000730000400040110000c0a80001c0a800c7")
    assert [mi.in_cksum_hdr(hdr, m) for m in (0, 2, 1)] == [0x61B8, 0x61B8, 0xB861]
    assert mi.in_cksum_skip(mi.MbufChain([(hdr, 1)]), 20, 0) == 0x61B8
    assert mi.in_cksum_skip(mi.MbufChain([bytes(1500)]), 1500, 0) == 0xFFFF
    assert mi.in_cksum_skip(mi.MbufChain([b"\xff" * 1500]), 1500, 0) == 0x0000
    for n, want in [(1, 0xFFFF), (2, 0xFEFF), (3, 0xFEFD), (63, 0x3B1C), (64, 0xFC1B), (1500, 0x4E39),
                    (1501, 0x4D5D), (9000, 0xB739), (65535, 0x3EC1), (65536, 0x3FC0)]:
        assert mi.in_cksum_skip(mi.MbufChain([kat7[:n]]), n, 0) == want, n
    for n, want in [(1, 0xFFFE), (64, 0xDBFB), (1500, 0x5D4D), (9000, 0x11B7), (65536, 0xC03F)]:
        assert mi.in_cksum_skip(mi.MbufChain([(kat7[1:n + 1], 1)]), n, 0) == want, n
    src, dst = 0x0101A8C0, 0x0201A8C0  # 192.168.1.1 / .2 as loaded from the header
    assert mi.in_cksum_pseudo_header(mi.MbufChain([kat7[:1500]]), 1480, 20, src, dst, 6) == 0x900A
    assert mi.in_cksum_pseudo_header(mi.MbufChain([kat7[:9000]]), 8980, 20, src, dst, 17) == 0xA1ED
    assert mi.in_cksum_skip(mi.MbufChain([kat7[:701], (kat7[701:1500], 1)]), 1500, 0) == 0x4E39
    assert mi.in_cksum_skip(mi.MbufChain([kat7[:1500]]), 1500, 20) == 0xB293


def test_odd_spans_and_truncation():
    """Every split of a buffer into three mbufs at every address parity gives
    the contiguous sum; a chain shorter than len truncates silently."""
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, 257, dtype=np.uint8).tobytes()
    want = mi.in_cksum_skip(mi.MbufChain([data]), 257, 0)
    for a, b in [(1, 2), (3, 100), (128, 129), (0, 256), (255, 256)]:
        for mods in [(0, 1, 2), (1, 1, 1), (3, 0, 7)]:
            segs = [(data[:a], mods[0]), (data[a:b], mods[1]), (data[b:], mods[2])]
            assert mi.in_cksum_skip(mi.MbufChain(segs), 257, 0) == want
    assert mi.in_cksum_skip(mi.MbufChain([data[:100]]), 257, 0) == mi.in_cksum_skip(mi.MbufChain([data[:100]]), 100, 0)


LINKTEST = os.path.join(ROOT, "oracle", "_ref", "linktest")


@pytest.mark.skipif(not os.path.exists(LINKTEST), reason="linktest not built (needs /root/reference at build time)")
def test_linked_kernel_caller_kats_host_mode():
    """The kernel-side caller compiled with the reference's headers and kernel
    flags, linked against libmicksum.so: all 28 known answers from the host fold."""
    env = {k: v for k, v in os.environ.items() if k != "MI_CKSUM_DROPIN"}
    p = subprocess.run([LINKTEST], capture_output=True, text=True, timeout=120, env=dict(env, MI_CKSUM_DROPIN="host"))
    assert p.returncode == 0, p.stdout + p.stderr
    res = json.loads(p.stdout)
    assert res["failed"] == 0 and res["kats"] == 28


@pytest.mark.skipif(mi.device_count() > 0, reason="a GPU is present")
def test_gpu_mode_degrades_to_host_fold(golden):
    """GPU mode with no device: every call is told to the handler, counted, and
    answered by the host fold -- the right sums; nothing aborts."""
    seen = []
    cb = DROPIN_ERROR_FN(lambda what, err: seen.append(what.decode()))
    lib = load()
    lib.mi_cksum_set_dropin_error_handler(C.cast(cb, C.c_void_p))
    mi.set_dropin_mode("gpu")
    d0 = mi.dropin_degraded()
    try:
        hdr = bytes.fromhex("450000730000400040110000c0a80001c0a800c7")
        assert mi.in_cksum_hdr(hdr, 1) == 0xB861
        kat7 = bytes(i & 0xFF for i in range(1500))
        assert mi.in_cksum_skip(mi.MbufChain([kat7]), 1500, 20) == 0xB293
        assert mi.in_cksum_pseudo_header(mi.MbufChain([kat7]), 1480, 20, 0x0101A8C0, 0x0201A8C0, 6) == 0x900A
        assert seen == ["in_cksum_hdr", "in_cksum_skip", "in_cksum_pseudo_header"]
        assert mi.dropin_degraded() == d0 + 3
    finally:
        lib.mi_cksum_set_dropin_error_handler(None)
        mi.set_dropin_mode("host")


# ----------------------------------------------------- host registration table
def _reg():
    lib = load()
    lib.mi__reg_table_insert.restype = C.c_int
    lib.mi__reg_table_insert.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64]
    lib.mi__reg_table_remove.restype = C.c_int
    lib.mi__reg_table_remove.argtypes = [C.c_void_p]
    lib.mi__reg_table_lookup.restype = C.c_uint64
    lib.mi__reg_table_lookup.argtypes = [C.c_void_p, C.c_uint64]
    lib.mi__reg_table_count.restype = C.c_int
    return lib


def test_registration_table_exact_and_disjoint():
    """two ranges that share a page can no longer both be
    registered; unregistration names the exact pointer, so removing one range
    never erases another's entry nor leaves its own (and its cached GPU
    address) behind for a later batch in the freed pages."""
    lib = _reg()
    base = 0x7F0000000000  # made-up addresses: the table is bookkeeping only
    n0 = lib.mi__reg_table_count()
    a, b = base + 0x100, base + 0x1000 + 0x80  # b's first page is a's last
    assert lib.mi__reg_table_insert(a, 0x1000, 0xA000) == 0
    assert lib.mi__reg_table_insert(b, 0x2000, 0xB000) == -17  # -EEXIST: shares page base+0x1000
    c = base + 0x3000
    assert lib.mi__reg_table_insert(c, 0x2000, 0xC000) == 0
    assert lib.mi__reg_table_lookup(a + 0x10, 0x100) == 0xA000 + 0x10
    assert lib.mi__reg_table_lookup(c + 0x10, 0x100) == 0xC000 + 0x10
    assert lib.mi__reg_table_remove(c + 0x10) == -2  # -ENOENT: not the registered pointer
    assert lib.mi__reg_table_remove(c) == 0
    assert lib.mi__reg_table_lookup(c + 0x10, 0x100) == 0  # nothing left in the freed range
    assert lib.mi__reg_table_lookup(a + 0x10, 0x100) == 0xA000 + 0x10  # the other range untouched
    assert lib.mi__reg_table_remove(c) == -2
    assert lib.mi__reg_table_remove(a) == 0
    assert lib.mi__reg_table_count() == n0


def test_page_buffer_is_page_granular():
    a = mi.page_buffer(5000)
    b = mi.page_buffer(100)
    assert a.nbytes == 5000 and a.ctypes.data % 4096 == 0 and b.ctypes.data % 4096 == 0
    a[:] = 1
    pa, pb = a.ctypes.data, b.ctypes.data
    assert pa + 8192 <= pb or pb + 4096 <= pa  # no page shared


from oracle.pyoracle import Oracle, available  # noqa: E402  (the checker)


@pytest.mark.skipif(not available("reference"), reason="oracle/_ref not built")
def test_random_chains_match_the_reference():
    """Property test beyond the golden vectors: 3000 random chains (1-6 mbufs,
    0-4100 bytes each, every address parity, zero-length mbufs, skips and
    lengths past the chain's end) through in_cksum_skip and
    in_cksum_pseudo_header, against the reference's own in_cksum.c
    (oracle/_ref) on the same mbuf layouts.  Long spans take the vector body,
    short ones the word loop; both stream-parity branches are hit."""
    ref = Oracle("reference")
    rng = np.random.default_rng(20260)
    for _ in range(3000):
        k = int(rng.integers(1, 7))
        segs = []
        for _ in range(k):
            ln = int(rng.choice([0, int(rng.integers(1, 64)), int(rng.integers(64, 4100))]))
            segs.append((rng.integers(0, 256, ln, dtype=np.uint8).tobytes(), int(rng.integers(0, 8))))
        total = sum(len(s) for s, _ in segs)
        skip = int(rng.integers(0, min(total, 60) + 1))
        length = int(rng.integers(skip, total + 40 + 1))
        m = mi.MbufChain(segs)
        assert mi.in_cksum_skip(m, length, skip) == ref.chain_skip(segs, length, skip), (segs, length, skip)
        if len(segs[0][0]) >= 20:
            plen = int(rng.integers(0, total + 1))
            src, dst = (int(x) for x in rng.integers(0, 1 << 32, 2, dtype=np.uint64))
            proto = int(rng.choice([6, 17]))
            assert (mi.in_cksum_pseudo_header(m, plen, 20, src, dst, proto)
                    == ref.chain_pseudo(segs, plen, 20, src, dst, proto))
