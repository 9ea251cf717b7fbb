"""ctypes front-end for the CPU checker libraries.

TEST INFRASTRUCTURE ONLY.  Imported by tests/, ``__graft_entry__.smoke()`` and
bench.py's ``cpu_baseline`` leg -- never by the product (``libunsod_amd``).

Two implementations share one interface:

* ``Oracle("port")``      -- oracle/_build/liboracle.so, the from-scratch C
  restatement of src/sys/amd64/amd64/in_cksum.c (cksum_oracle.c);
* ``Oracle("reference")`` -- oracle/_ref/libref.so, the reference's own
  in_cksum.c compiled from /root/reference by oracle/Makefile (symbols renamed
  ``ref_*``).  Built in the dev container; the prebuilt .so travels to the GPU
  box, the reference tree does not.

Mbuf chains are built in C (batch_driver.c) over caller segments, so a segment's
*address* is real: ``place()`` puts bytes at a chosen address mod 64, which is
what ``in_cksum_hdr``'s absolute-address lanes and the chain-walk parity swap
(in_cksum.c:222-225) depend on.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATHS = {
    "port": os.path.join(_HERE, "_build", "liboracle.so"),
    "reference": os.path.join(_HERE, "_ref", "libref.so"),
}
_PFX = {"port": "orc_", "reference": "ref_"}

u8p = C.POINTER(C.c_uint8)
u16p = C.POINTER(C.c_uint16)
u32p = C.POINTER(C.c_uint32)
u64p = C.POINTER(C.c_uint64)


def available(kind: str) -> bool:
    return os.path.exists(LIB_PATHS[kind])


def place(data, addr_mod: int, align: int = 64, pad: int = 64) -> tuple[np.ndarray, int]:
    """Copy ``data`` into a fresh buffer so that its first byte sits at an
    address == addr_mod (mod align).  Returns (keepalive_array, address).
    ``pad`` slack bytes surround it (in_cksumdata reads up to 3 B either side)."""
    src = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    n = int(src.size)
    buf = np.zeros(n + 2 * pad + 2 * align, dtype=np.uint8)
    base = buf.ctypes.data
    start = pad + ((addr_mod - (base + pad)) % align)
    buf[start:start + n] = src
    return buf, base + start


def _ptr(a: np.ndarray | None, typ):
    return None if a is None else a.ctypes.data_as(typ)


class Oracle:
    def __init__(self, kind: str = "port"):
        if kind not in LIB_PATHS:
            raise ValueError(kind)
        path = LIB_PATHS[kind]
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle`")
        self.kind = kind
        self.lib = C.CDLL(path)
        p = _PFX[kind]
        g = lambda n: getattr(self.lib, p + n)  # noqa: E731

        self._skip = g("in_cksum_skip")
        self._hdr = g("in_cksum_hdr"); self._hdr.restype = C.c_uint; self._hdr.argtypes = [C.c_void_p]
        self._pseudo = g("in_pseudo"); self._pseudo.restype = C.c_uint16
        self._pseudo.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32]
        self._addword = g("in_addword"); self._addword.restype = C.c_uint16
        self._addword.argtypes = [C.c_uint16, C.c_uint16]

        self._chain_skip = g("chain_skip"); self._chain_skip.restype = C.c_uint16
        self._chain_skip.argtypes = [C.POINTER(C.c_void_p), C.POINTER(C.c_int32), C.c_int, C.c_int, C.c_int]
        self._chain_pseudo = g("chain_pseudo"); self._chain_pseudo.restype = C.c_uint16
        self._chain_pseudo.argtypes = [C.POINTER(C.c_void_p), C.POINTER(C.c_int32), C.c_int, C.c_int,
                                       C.c_int, C.c_uint32, C.c_uint32, C.c_uint8]
        self._verify = g("ipv4_verify_batch"); self._verify.restype = None
        self._verify.argtypes = [C.c_void_p, u64p, C.c_uint64, C.c_uint64, u32p, C.c_uint32,
                                 C.c_uint32, u16p, u16p, u8p, C.c_int]
        self._final = g("ipv4_finalize_batch"); self._final.restype = None
        self._final.argtypes = [C.c_void_p, u64p, C.c_uint64, C.c_uint64, u32p, C.c_uint32,
                                C.c_uint32, C.c_int]
        self._dverify = g("ipv4_demux_verify_batch"); self._dverify.restype = None
        self._dverify.argtypes = self._verify.argtypes
        self._dfinal = g("ipv4_demux_finalize_batch"); self._dfinal.restype = None
        self._dfinal.argtypes = self._final.argtypes
        self._repeat = g("skip_repeat"); self._repeat.restype = C.c_uint64
        self._repeat.argtypes = [C.c_void_p, C.c_int, C.c_int]
        self._tx = g("tx_copy_batch"); self._tx.restype = None
        self._tx.argtypes = [C.c_void_p, u64p, C.POINTER(C.c_int32), u32p, u32p, u32p, u32p, C.c_uint32,
                             C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, u8p]

    # --- scalar reference entry points (in_cksum.h:77-83) -------------------
    def in_pseudo(self, a: int, b: int, c: int) -> int:
        return int(self._pseudo(a & 0xFFFFFFFF, b & 0xFFFFFFFF, c & 0xFFFFFFFF))

    def in_addword(self, a: int, b: int) -> int:
        return int(self._addword(a & 0xFFFF, b & 0xFFFF))

    def in_cksum_hdr_at(self, addr: int) -> int:
        return int(self._hdr(C.c_void_p(addr)))

    def in_cksum_hdr(self, data20, addr_mod: int = 0) -> int:
        keep, addr = place(data20, addr_mod)
        r = self.in_cksum_hdr_at(addr)
        del keep
        return r

    @staticmethod
    def _segs(segs: Sequence[tuple[bytes, int]]):
        keep, addrs, lens = [], [], []
        for data, mod in segs:
            k, a = place(data, mod)
            keep.append(k); addrs.append(a); lens.append(len(data))
        n = len(segs)
        return keep, (C.c_void_p * n)(*addrs), (C.c_int32 * n)(*lens), n

    def chain_skip(self, segs: Sequence[tuple[bytes, int]], length: int, skip: int) -> int:
        keep, a, l, n = self._segs(segs)
        r = int(self._chain_skip(a, l, n, length, skip))
        del keep
        return r

    def chain_pseudo(self, segs, plen: int, off0: int, src: int, dst: int, proto: int) -> int:
        keep, a, l, n = self._segs(segs)
        r = int(self._chain_pseudo(a, l, n, plen, off0, src & 0xFFFFFFFF, dst & 0xFFFFFFFF, proto & 0xFF))
        del keep
        return r

    # --- batch drivers ------------------------------------------------------
    def ipv4_verify_batch(self, buf: np.ndarray, n: int, *, offs=None, stride: int = 0,
                          first_off: int = 0, flen=None, fixed_flen: int = 0, nthreads: int = 1,
                          demux: bool = False):
        """RX verify; ``demux`` = the MI_BATCH_DEMUX protocol dispatch
        (batch_driver.c demux_l4)."""
        ip = np.zeros(n, np.uint16); l4 = np.zeros(n, np.uint16); st = np.zeros(n, np.uint8)
        offs = None if offs is None else np.ascontiguousarray(offs, np.uint64)
        flen = None if flen is None else np.ascontiguousarray(flen, np.uint32)
        (self._dverify if demux else self._verify)(buf.ctypes.data, _ptr(offs, u64p), stride, first_off, _ptr(flen, u32p),
                     fixed_flen, n, _ptr(ip, u16p), _ptr(l4, u16p), _ptr(st, u8p), nthreads)
        return ip, l4, st

    def ipv4_finalize_batch(self, buf: np.ndarray, n: int, *, offs=None, stride: int = 0,
                            first_off: int = 0, flen=None, fixed_flen: int = 0, nthreads: int = 1,
                            demux: bool = False):
        offs = None if offs is None else np.ascontiguousarray(offs, np.uint64)
        flen = None if flen is None else np.ascontiguousarray(flen, np.uint32)
        (self._dfinal if demux else self._final)(buf.ctypes.data, _ptr(offs, u64p), stride, first_off, _ptr(flen, u32p),
                    fixed_flen, n, nthreads)

    def skip_repeat(self, buf: np.ndarray, length: int, iters: int) -> int:
        return int(self._repeat(buf.ctypes.data, length, iters))

    def tx_copy_batch(self, src: np.ndarray, seg_off, seg_len, pkt_seg, pkt_len, dst: np.ndarray, *,
                      dst_stride: int, dst_first: int, room: int, l3_off: int = 14, csum_flags=None,
                      csum_data=None) -> np.ndarray:
        """TX offload fused with the driver's copy (batch_driver.c tx_copy_batch):
        frame i = chain of segments [pkt_seg[i], pkt_seg[i+1]) of ``src`` copied
        into ``dst`` at dst_first + i*dst_stride with in_delayed_cksum / ip_sum
        applied as the software stack would.  ``dst`` is written in place;
        returns the per-frame status (ORC_TX_* bits)."""
        seg_off = np.ascontiguousarray(seg_off, np.uint64)
        seg_len = np.ascontiguousarray(seg_len, np.int32)
        pkt_seg = np.ascontiguousarray(pkt_seg, np.uint32)
        pkt_len = np.ascontiguousarray(pkt_len, np.uint32)
        n = len(pkt_len)
        cf = None if csum_flags is None else np.ascontiguousarray(csum_flags, np.uint32)
        cd = None if csum_data is None else np.ascontiguousarray(csum_data, np.uint32)
        st = np.zeros(n, np.uint8)
        self._tx(src.ctypes.data, _ptr(seg_off, u64p), seg_len.ctypes.data_as(C.POINTER(C.c_int32)),
                 _ptr(pkt_seg, u32p), _ptr(pkt_len, u32p), _ptr(cf, u32p), _ptr(cd, u32p), l3_off,
                 dst.ctypes.data, dst_stride, dst_first, room, n, _ptr(st, u8p))
        return st


TX_NOBUFS, TX_SHORT, TX_NOSUM, TX_L4_SKIPPED = 1, 2, 4, 8
CSUM_IP, CSUM_TCP, CSUM_UDP = 0x1, 0x2, 0x4  # mbuf.h:281-283


# --- RX offload flags -----------------------------------
CSUM_IP_CHECKED, CSUM_IP_VALID, CSUM_DATA_VALID, CSUM_PSEUDO_HDR = 0x100, 0x200, 0x400, 0x800  # mbuf.h:290-293


def rx_offload_flags(buf: np.ndarray, offs, flen, ip, l4, st):
    """(csum_flags, csum_data) per datagram from a verify result, restating what
    makes the stack's offload branches equivalent to its own sums:
    ip_input.c:459-460 (IP_CHECKED / IP_VALID), tcp_input.c:698-709 and
    udp_usrreq.c:431-438 (DATA_VALID | PSEUDO_HDR, th_sum = csum_data ^ 0xffff),
    udp_usrreq.c:406-414 (UDP sums uh_ulen bytes: offload only when it equals
    ip_len - hl), ip_reass (no offload for fragments)."""
    n = len(offs)
    fl = np.zeros(n, np.uint32)
    cd = np.zeros(n, np.uint32)
    for i in range(n):
        if st[i] & 4 and (int(flen[i]) < 20 or not _hdr_ok(buf, int(offs[i]), int(flen[i]))):
            continue
        p = int(offs[i])
        fl[i] = CSUM_IP_CHECKED | (CSUM_IP_VALID if ip[i] == 0 else 0)
        if st[i] & 4:  # header fine, ip_len out of range
            continue
        hl = (int(buf[p]) & 15) * 4
        iplen = (int(buf[p + 2]) << 8) | int(buf[p + 3])
        ip_off = (int(buf[p + 6]) << 8) | int(buf[p + 7])
        proto = int(buf[p + 9])
        if ip_off & 0x3FFF:
            continue
        ok = proto == 6
        if proto == 17 and iplen - hl >= 8:
            ok = ((int(buf[p + hl + 4]) << 8) | int(buf[p + hl + 5])) == iplen - hl
        if ok:
            fl[i] |= CSUM_DATA_VALID | CSUM_PSEUDO_HDR
            cd[i] = int(l4[i]) ^ 0xFFFF
    return fl, cd


def _hdr_ok(buf, p, flen):
    hl = (int(buf[p]) & 15) * 4
    return hl >= 20 and hl <= flen
