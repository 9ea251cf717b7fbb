#!/usr/bin/env python3
"""Generate the golden vectors in tests/golden/ from the REFERENCE itself.

Run in the dev container (needs /root/reference): ``make -C oracle`` builds
oracle/_ref/libref.so from the reference's own src/sys/amd64/amd64/in_cksum.c;
this script drives it through oracle/batch_driver.c on seeded inputs and stores
inputs + outputs as data (no reference source is stored).

The reference ships no tests, fixtures or golden vectors for in_cksum*
(SURVEY.md section 4), so these vectors -- plus the KATs from SURVEY.md 8(a),
which are asserted here before anything is written -- are the parity pin.

    python tests/golden/make_golden.py      # writes tests/golden/cksum_golden.npz
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.pyoracle import Oracle  # noqa: E402
from libunsod_amd.synth import build_ipv4_batch  # noqa: E402

OUT = os.path.join(HERE, "cksum_golden.npz")
SEED = 20261015


def _le32(b):
    return int.from_bytes(bytes(b), "little")


def check_kats(o: Oracle) -> None:
    """SURVEY.md 8(a) known answers, from the compiled reference."""
    rfc = bytes([0x00, 0x01, 0xF2, 0x03, 0xF4, 0xF5, 0xF6, 0xF7])
    assert o.chain_skip([(rfc, 0)], 8, 0) == 0x0D22
    hdr = bytes.fromhex("450000730000400040110000c0a80001c0a800c7")
    assert o.in_cksum_hdr(hdr, 0) == 0x61B8 and o.in_cksum_hdr(hdr, 2) == 0x61B8
    assert o.in_cksum_hdr(hdr, 1) == 0xB861 and o.chain_skip([(hdr, 1)], 20, 0) == 0x61B8
    assert o.chain_skip([(bytes(1500), 0)], 1500, 0) == 0xFFFF
    assert o.chain_skip([(b"\xff" * 1500, 0)], 1500, 0) == 0x0000
    pat = bytes(i & 0xFF for i in range(65536 + 64))
    for L, r in [(1, 0xFFFF), (2, 0xFEFF), (3, 0xFEFD), (63, 0x3B1C), (64, 0xFC1B), (1500, 0x4E39),
                 (1501, 0x4D5D), (9000, 0xB739), (65535, 0x3EC1), (65536, 0x3FC0)]:
        assert o.chain_skip([(pat[:L], 0)], L, 0) == r, L
    for L, r in [(1, 0xFFFE), (64, 0xDBFB), (1500, 0x5D4D), (9000, 0x11B7), (65536, 0xC03F)]:
        assert o.chain_skip([(pat[1:L + 1], 1)], L, 0) == r, L
    src, dst = _le32([192, 168, 1, 1]), _le32([192, 168, 1, 2])
    assert o.chain_pseudo([(pat[:1500], 0)], 1480, 20, src, dst, 6) == 0x900A
    assert o.chain_pseudo([(pat[:9000], 0)], 8980, 20, src, dst, 17) == 0xA1ED
    assert o.in_pseudo(src, dst, _le32((20 + 6 + 1460).to_bytes(4, "big"))) == 0x2289
    assert o.chain_skip([(pat[:701], 0), (pat[701:1500], 1)], 1500, 0) == 0x4E39
    assert o.chain_skip([(pat[:1500], 0)], 1500, 20) == 0xB293


class Blob:
    def __init__(self):
        self.parts, self.size = [], 0

    def add(self, data: bytes) -> int:
        off = self.size
        self.parts.append(np.frombuffer(bytes(data), np.uint8))
        self.size += len(data)
        return off

    def array(self):
        return np.concatenate(self.parts) if self.parts else np.zeros(0, np.uint8)


def rand_bytes(rng, n, kind=None):
    kind = kind or rng.choice(["rand", "rand", "rand", "rand", "zero", "ff", "pat"])
    if kind == "zero":
        return bytes(n)
    if kind == "ff":
        return b"\xff" * n
    if kind == "pat":
        return bytes((np.arange(n) + int(rng.integers(256))) & 0xFF)
    return rng.integers(0, 256, n, dtype=np.uint8).tobytes()


def sparse_bytes(rng, n):
    """Large buffers: a byte pattern with ~3 % random bytes (keeps the file small)."""
    b = (np.arange(n) * 7 + int(rng.integers(256))) & 0xFF
    k = rng.integers(0, n, max(1, n // 32))
    b[k] = rng.integers(0, 256, k.size)
    return b.astype(np.uint8).tobytes()


def rand_seglen(rng):
    c = rng.random()
    if c < 0.10:
        return int(rng.integers(0, 4))
    if c < 0.35:
        return int(rng.integers(1, 41))
    if c < 0.90:
        return int(rng.integers(40, 601))
    return int(rng.integers(600, 3001))


def main():
    o = Oracle("reference")
    check_kats(o)
    rng = np.random.default_rng(SEED)
    blob = Blob()
    seg_off, seg_len, seg_mod = [], [], []

    def add_chain(segs):
        start = len(seg_off)
        for data, mod in segs:
            seg_off.append(blob.add(data)); seg_len.append(len(data)); seg_mod.append(mod)
        return start

    # ---- in_cksum_skip over chains -----------------------------------------
    sk = {k: [] for k in ("seg0", "nseg", "len", "skip", "result")}
    def skip_case(segs, length, skip):
        r = o.chain_skip(segs, length, skip)
        sk["seg0"].append(add_chain(segs)); sk["nseg"].append(len(segs))
        sk["len"].append(length); sk["skip"].append(skip); sk["result"].append(r)

    for _ in range(1400):
        nseg = int(rng.choice([1, 1, 1, 2, 2, 3, 4, 5]))
        kind = rng.choice(["rand", "rand", "rand", "zero", "ff", "pat"])
        segs = [(rand_bytes(rng, rand_seglen(rng), kind), int(rng.integers(64))) for _ in range(nseg)]
        total = sum(len(s) for s, _ in segs)
        c = rng.random()
        skip = 0 if c < 0.5 else int(rng.integers(0, 24)) if c < 0.8 else int(rng.integers(0, total + 2))
        c = rng.random()
        length = total if c < 0.6 else int(rng.integers(skip, max(skip, total) + 1)) if c < 0.9 \
            else total + int(rng.integers(1, 64))
        length = max(length, skip)
        skip_case(segs, length, skip)
    for L in (9000, 9001, 9100, 8999, 12345, 65535, 65536, 70001):
        for mod in (0, 1, 2, 3):
            skip_case([(sparse_bytes(rng, L), mod)], L, int(rng.integers(0, 24)) if mod & 2 else 0)

    # ---- in_cksum_pseudo_header ---------------------------------------------
    ps = {k: [] for k in ("seg0", "nseg", "plen", "off0", "src", "dst", "proto", "result")}
    def pseudo_case(segs, plen, off0, src, dst, proto):
        r = o.chain_pseudo(segs, plen, off0, src, dst, proto)
        ps["seg0"].append(add_chain(segs)); ps["nseg"].append(len(segs))
        for k, v in (("plen", plen), ("off0", off0), ("src", src), ("dst", dst), ("proto", proto), ("result", r)):
            ps[k].append(v)

    for _ in range(900):
        nseg = int(rng.choice([1, 1, 1, 2, 2, 3, 4]))
        off0 = int(rng.choice([20, 20, 24, 40, 60, int(rng.integers(0, 65))]))
        kind = rng.choice(["rand", "rand", "rand", "zero", "pat"])
        first = max(off0 + int(rng.integers(0, 3)), rand_seglen(rng))
        segs = [(rand_bytes(rng, first, kind), int(rng.integers(64)))]
        segs += [(rand_bytes(rng, rand_seglen(rng), kind), int(rng.integers(64))) for _ in range(nseg - 1)]
        total = sum(len(s) for s, _ in segs)
        c = rng.random()
        plen = total - off0 if c < 0.6 else int(rng.integers(0, total - off0 + 1)) if c < 0.9 \
            else total - off0 + int(rng.integers(1, 50))
        src, dst = int(rng.integers(0, 2**32)), int(rng.integers(0, 2**32))
        if rng.random() < 0.05:
            src = dst = 0
        proto = int(rng.choice([6, 17, 6, 17, int(rng.integers(0, 256))]))
        pseudo_case(segs, plen, off0, src, dst, proto)
    for plen in (65515, 65516, 65536 - 20, 65536, 65536 + 100, 70000):  # 16-bit truncation of plen
        segs = [(sparse_bytes(rng, plen + 20), int(rng.integers(64)))]
        pseudo_case(segs, plen, 20, int(rng.integers(0, 2**32)), int(rng.integers(0, 2**32)), 6)

    # ---- in_cksum_hdr at every alignment ------------------------------------
    hd_off, hd_mod, hd_res = [], [], []
    for mod in range(64):
        for kind in ("rand", "rand", "rand", "zero", "ff"):
            b = rand_bytes(rng, 20, kind)
            hd_off.append(blob.add(b)); hd_mod.append(mod); hd_res.append(o.in_cksum_hdr(b, mod))

    # ---- in_pseudo / in_addword ---------------------------------------------
    edge32 = [0, 1, 0xFFFF, 0x10000, 0xFFFEFFFF, 0xFFFF0000, 0xFFFFFFFF]
    pa = [int(x) for x in rng.integers(0, 2**32, 600)] + edge32 * 3
    pb = [int(x) for x in rng.integers(0, 2**32, 600)] + edge32[::-1] * 3
    pc = [int(x) for x in rng.integers(0, 2**32, 600)] + edge32[1:] * 3 + edge32[:1] * 3
    ip_res = [o.in_pseudo(a, b, c) for a, b, c in zip(pa, pb, pc)]
    edge16 = [0, 1, 0x7FFF, 0x8000, 0xFFFE, 0xFFFF]
    wa = [int(x) for x in rng.integers(0, 2**16, 600)] + [a for a in edge16 for _ in edge16]
    wb = [int(x) for x in rng.integers(0, 2**16, 600)] + [b for _ in edge16 for b in edge16]
    aw_res = [o.in_addword(a, b) for a, b in zip(wa, wb)]

    # ---- RX verify / TX finalize batches --------------------------------------
    nb = 600
    L = rng.integers(20, 2200, nb)
    L[:40] = rng.integers(0, 24, 40)           # runts / tiny
    L[40:80] = rng.integers(9000, 9100, 40)    # jumbo
    hl = rng.choice([20, 20, 20, 24, 40, 60], nb)
    proto = rng.choice([6, 6, 17, 17, 1], nb)
    sz = (L + 7 + rng.integers(0, 5, nb))
    offs = np.concatenate([[0], np.cumsum(sz)[:-1]]) + 3  # odd and even starts
    b = build_ipv4_batch(nb, np.maximum(L, 0), offs=offs, proto=proto, hl=hl, seed=SEED + 1)
    buf_in = b["buf"].copy()
    flen = b["flen"].copy()
    # some malformed headers: ip_len / hl inconsistent with flen
    bad = rng.choice(np.arange(80, nb), 60, replace=False)
    for k, i in enumerate(bad):
        p = int(offs[i])
        if flen[i] < 20:
            continue
        if k % 3 == 0:
            buf_in[p] = 0x40 | int(rng.integers(0, 5))          # hl < 20
        elif k % 3 == 1:
            v = int(flen[i]) + int(rng.integers(1, 40))          # ip_len > flen
            buf_in[p + 2], buf_in[p + 3] = v >> 8, v & 0xFF
        else:
            buf_in[p + 2], buf_in[p + 3] = 0, int(rng.integers(0, 20))  # ip_len < hl
    fin_in = buf_in.copy()
    base_keep, base_addr = None, None
    # run the reference on a 64-aligned copy so address parity == offset parity
    def aligned_copy(a):
        raw = np.zeros(a.size + 128, np.uint8)
        s = (-raw.ctypes.data) % 64
        v = raw[s:s + a.size]
        v[:] = a
        return raw, v
    keep1, fin = aligned_copy(fin_in)
    o.ipv4_finalize_batch(fin, nb, offs=offs, flen=flen)
    fin_out = fin.copy()
    ver_in = fin_out.copy()
    corrupt = rng.choice(np.arange(nb), 50, replace=False)
    for i in corrupt:
        if flen[i] > 20:
            j = int(offs[i]) + int(rng.integers(0, int(flen[i])))
            ver_in[j] ^= np.uint8(1 << int(rng.integers(8)))
    keep2, ver = aligned_copy(ver_in)
    v_ip, v_l4, v_st = o.ipv4_verify_batch(ver, nb, offs=offs, flen=flen)
    assert (v_st == 0).sum() > nb // 2

    # fixed-stride slot batch (the 1500 B geometry, scaled down): valid packets
    ns = 64
    sb = build_ipv4_batch(ns, 1500, stride=2176, first_off=142, seed=SEED + 2)
    keep3, sbuf = aligned_copy(sb["buf"])
    o.ipv4_finalize_batch(sbuf, ns, stride=2176, first_off=142, fixed_flen=1500)
    s_ip, s_l4, s_st = o.ipv4_verify_batch(sbuf, ns, stride=2176, first_off=142, fixed_flen=1500)
    assert (s_st == 0).all() and (s_ip == 0).all() and (s_l4 == 0).all()

    np.savez_compressed(
        OUT,
        blob=blob.array(),
        seg_off=np.array(seg_off, np.int64), seg_len=np.array(seg_len, np.int32),
        seg_mod=np.array(seg_mod, np.int32),
        **{f"sk_{k}": np.array(v, np.int64) for k, v in sk.items()},
        **{f"ps_{k}": np.array(v, np.int64) for k, v in ps.items()},
        hd_off=np.array(hd_off, np.int64), hd_mod=np.array(hd_mod, np.int32), hd_result=np.array(hd_res, np.int64),
        ip_a=np.array(pa, np.int64), ip_b=np.array(pb, np.int64), ip_c=np.array(pc, np.int64),
        ip_result=np.array(ip_res, np.int64),
        aw_a=np.array(wa, np.int64), aw_b=np.array(wb, np.int64), aw_result=np.array(aw_res, np.int64),
        vb_offs=offs.astype(np.uint64), vb_flen=flen, fin_in=fin_in, fin_out=fin_out,
        ver_in=ver_in, ver_ip=v_ip, ver_l4=v_l4, ver_st=v_st,
        slot_in=sb["buf"], slot_out=sbuf.copy(),
    )
    print(f"wrote {OUT}: {len(sk['result'])} skip, {len(ps['result'])} pseudo, {len(hd_res)} hdr, "
          f"{len(ip_res)} in_pseudo, {len(aw_res)} in_addword, {nb} verify/finalize packets, "
          f"blob {blob.size} B, file {os.path.getsize(OUT)} B")


if __name__ == "__main__":
    main()
