"""Python mirror of the reference checksum interface, over the C ABI.

Scalar layer -- same names, argument meaning and (lack of) error behaviour as
src/sys/amd64/include/in_cksum.h:44,77-83.  ``MbufChain`` builds a real
``struct mbuf`` chain in host memory (256 B mbufs; m_next@0, m_data@16,
m_len@24 as in src/sys/sys/mbuf.h:90-98,166-168) so the calls below go through
libmicksum's drop-in C symbols exactly as libuinet's protocol code would.

Batch layer -- ``PktBatch`` describes packets in a device-resident torch uint8
tensor; ``ipv4_verify`` / ``ipv4_finalize`` / ``span_batch`` launch the gfx950
kernels on the current torch stream (asynchronous).
"""
from __future__ import annotations

import ctypes as C
from typing import Iterable

import numpy as np

from ._lib import (MI_BATCH_DEMUX, MI_BATCH_HOST_STAGED, MI_BATCH_OFFS32, MI_BATCH_PACKED, MI_BATCH_MAX_BYTES, MI_CHAIN_PSEUDO,
                   MI_CHAIN_SKIP, MI_REPEAT_AFTER_DEFAULT, MI_REPEAT_ASYNC, MI_REPEAT_GRAPH, MI_SPAN_ABS,
                   MI_SPAN_STREAM, MI_TIME_NONE, MI_TIME_PER_PASS, MI_TIME_REGION, ChainBatchC, PktBatchC,
                   SpanSeedsC, TxBatchC, check, load)

MSIZE = 256  # param.h:159


# ----------------------------------------------------------------- scalar (b1)
class MbufChain:
    """A chain of real mbufs over ``segments``.

    Each segment is ``bytes`` or ``(bytes, addr_mod)``; the data of a segment is
    placed at an address == addr_mod (mod 64) -- address parity is what the
    reference's per-span swap (in_cksum.c:222-225) reacts to.
    """

    def __init__(self, segments: Iterable):
        segs = [(s, 0) if isinstance(s, (bytes, bytearray, memoryview, np.ndarray)) else s for s in segments]
        if not segs:
            raise ValueError("an mbuf chain has at least one mbuf")
        self._keep = []
        self.mbufs = np.zeros(len(segs) * MSIZE + 64, np.uint8)
        mb_base = self.mbufs.ctypes.data + ((-self.mbufs.ctypes.data) % 64)
        addrs = [mb_base + k * MSIZE for k in range(len(segs))]
        for k, (data, mod) in enumerate(segs):
            raw = np.frombuffer(bytes(data), np.uint8)
            buf = np.zeros(raw.size + 192, np.uint8)
            start = 64 + ((mod - (buf.ctypes.data + 64)) % 64)
            buf[start:start + raw.size] = raw
            self._keep.append(buf)
            nxt = addrs[k + 1] if k + 1 < len(segs) else 0
            C.c_uint64.from_address(addrs[k]).value = nxt                   # m_next
            C.c_uint64.from_address(addrs[k] + 16).value = buf.ctypes.data + start  # m_data
            C.c_int32.from_address(addrs[k] + 24).value = raw.size           # m_len
        self.ptr = addrs[0]
        self.total = sum(len(bytes(d)) for d, _ in segs)


def in_cksum_skip(m: MbufChain, length: int, skip: int) -> int:
    return int(load().in_cksum_skip(C.c_void_p(m.ptr), length, skip))


def in_cksum(m: MbufChain, length: int) -> int:
    return in_cksum_skip(m, length, 0)


def in_cksum_pseudo_header(m: MbufChain, plen: int, off0: int, src: int, dst: int, protonum: int) -> int:
    return int(load().in_cksum_pseudo_header(C.c_void_p(m.ptr), plen, off0, src & 0xFFFFFFFF,
                                             dst & 0xFFFFFFFF, protonum & 0xFF))


def in_cksum_hdr(ip, addr_mod: int = 0) -> int:
    """``ip``: 20 header bytes, placed at an address == addr_mod (mod 64)."""
    raw = np.frombuffer(bytes(ip), np.uint8)
    buf = np.zeros(256, np.uint8)
    start = 64 + ((addr_mod - (buf.ctypes.data + 64)) % 64)
    buf[start:start + raw.size] = raw
    return int(load().in_cksum_hdr(C.c_void_p(buf.ctypes.data + start)))


def in_pseudo(a: int, b: int, c: int) -> int:
    return int(load().in_pseudo(a & 0xFFFFFFFF, b & 0xFFFFFFFF, c & 0xFFFFFFFF))


def in_addword(a: int, b: int) -> int:
    return int(load().in_addword(a & 0xFFFF, b & 0xFFFF))


# ------------------------------------------------------------------ batch (b2)
def _torch():
    import torch  # deferred: the scalar layer needs no torch
    return torch


def _stream(stream) -> int:
    torch = _torch()
    if stream is None:
        return torch.cuda.current_stream().cuda_stream
    return getattr(stream, "cuda_stream", stream)


class PktBatch:
    """n packets in a device uint8 tensor ``buf``.

    Packet i starts at ``offs[i]`` (device int64 tensor) or
    ``first_off + i*stride`` and is ``lens[i]`` (device int32 tensor) or
    ``fixed_len`` bytes long.  ``packed``: offsets ascend and datagrams sit back
    to back (MI_BATCH_PACKED hint; correct either way).  ``demux``: verify /
    finalize take each datagram's L4 sum the way ip_input's protocol switch
    hands it on -- TCP / UDP / ICMP / IGMP / CARP, fragments none
    (MI_BATCH_DEMUX, include/mi_cksum.h).  ``offs32``: pass the offsets as
    u32 (MI_BATCH_OFFS32, 4 descriptor bytes per packet instead of 8).
    """

    def __init__(self, buf, n: int, *, offs=None, stride: int = 0, first_off: int = 0, lens=None,
                 fixed_len: int = 0, max_len: int = 0, packed: bool = False, demux: bool = False,
                 offs32: bool = False):
        torch = _torch()
        if buf.dtype != torch.uint8 or not buf.is_contiguous():
            raise ValueError("buf must be a contiguous uint8 tensor")
        if buf.numel() > MI_BATCH_MAX_BYTES:
            raise ValueError(f"batch buffer of {buf.numel()} B > MI_BATCH_MAX_BYTES ({MI_BATCH_MAX_BYTES})")
        self.buf, self.n = buf, int(n)
        offs32 = bool(offs32 and offs is not None)
        if offs32 and offs.numel() and int(offs.max().item()) >= 1 << 32:
            # u32 would wrap such an offset onto valid bytes; u64 reports it MALFORMED
            raise ValueError("offs32: an offset does not fit in 32 bits")
        # u32 offsets travel as int32 bit patterns (buffers are < 4 GiB)
        self.offs = None if offs is None else (
            offs.to(torch.int64).to(torch.int32) if offs32 else offs.to(torch.int64)).contiguous()
        self.lens = None if lens is None else lens.to(torch.int32).contiguous()
        self.stride, self.first_off, self.fixed_len = int(stride), int(first_off), int(fixed_len)
        self.max_len = int(max_len)
        if self.lens is not None and not self.max_len:
            self.max_len = int(self.lens.max().item()) if self.n else 0
        self._c = PktBatchC(buf.data_ptr(), buf.numel(),
                            self.offs.data_ptr() if self.offs is not None else None,
                            self.stride, self.first_off,
                            self.lens.data_ptr() if self.lens is not None else None,
                            self.fixed_len, self.n, self.max_len,
                            (MI_BATCH_PACKED if packed else 0) | (MI_BATCH_DEMUX if demux else 0)
                            | (MI_BATCH_OFFS32 if offs32 else 0))

    @property
    def c(self) -> PktBatchC:
        return self._c


def _ptr(t):
    return None if t is None else t.data_ptr()


def ipv4_verify(b: PktBatch, *, ip: bool = True, l4: bool = True, status: bool = True,
                bad_count: bool = False, out=None, stream=None) -> dict:
    """RX verify (ip_input.c:459-471 + tcp_input.c:697-720).  Returns a dict of
    device tensors: ip / l4 (uint16), status (uint8), bad (int32[1], a u32 count)."""
    torch = _torch()
    dev = b.buf.device
    res = dict(out or {})
    if ip and "ip" not in res:
        res["ip"] = torch.empty(b.n, dtype=torch.uint16, device=dev)
    if l4 and "l4" not in res:
        res["l4"] = torch.empty(b.n, dtype=torch.uint16, device=dev)
    if status and "status" not in res:
        res["status"] = torch.empty(b.n, dtype=torch.uint8, device=dev)
    if bad_count:
        res["bad"] = res.get("bad", torch.zeros(1, dtype=torch.int32, device=dev))
        res["bad"].zero_()
    check("mi_cksum_ipv4_verify",
          load().mi_cksum_ipv4_verify(C.byref(b.c), _ptr(res.get("ip")), _ptr(res.get("l4")),
                                      _ptr(res.get("status")), _ptr(res.get("bad")),
                                      C.c_void_p(_stream(stream))))
    return res


def ipv4_verify_multi(batches, outs, *, bad=None, stream=None) -> None:
    """RX verify of several batches in one launch (mi_cksum_ipv4_verify_multi):
    outs[k] = dict(ip, l4, status) device tensors for batches[k]; ``bad``: an
    int32[1] device counter for all of them (or None)."""
    nb = len(batches)
    arr = (PktBatchC * nb)(*[b.c for b in batches])
    VP = C.c_void_p * nb
    ptrs = {k: VP(*[_ptr(o.get(k)) for o in outs]) for k in ("ip", "l4", "status")}
    check("mi_cksum_ipv4_verify_multi",
          load().mi_cksum_ipv4_verify_multi(arr, nb, ptrs["ip"], ptrs["l4"], ptrs["status"], _ptr(bad),
                                            C.c_void_p(_stream(stream))))


def verify_plan(b: PktBatch) -> str:
    """Name of the verify kernel ``ipv4_verify`` launches for ``b`` (diagnostics)."""
    return load().mi_cksum_verify_plan(C.byref(b.c)).decode()


def rx_offload(b: PktBatch, *, data: bool = True, bad_count: bool = False, out=None, stream=None) -> dict:
    """RX offload flags for a received burst (mi_cksum_rx_offload): per datagram
    the m_pkthdr.csum_flags (uint32 -> "flags") and csum_data ("data") that
    make ip_input / tcp_input / udp_input take their offload branches with
    unchanged decisions.  Returns a dict of device int32 tensors (u32 values)."""
    torch = _torch()
    dev = b.buf.device
    res = dict(out or {})
    res.setdefault("flags", torch.empty(b.n, dtype=torch.int32, device=dev))
    if data:
        res.setdefault("data", torch.empty(b.n, dtype=torch.int32, device=dev))
    if bad_count:
        res["bad"] = res.get("bad", torch.zeros(1, dtype=torch.int32, device=dev))
        res["bad"].zero_()
    check("mi_cksum_rx_offload",
          load().mi_cksum_rx_offload(C.byref(b.c), _ptr(res["flags"]), _ptr(res.get("data")), _ptr(res.get("bad")),
                                     C.c_void_p(_stream(stream))))
    return res


def ipv4_finalize(b: PktBatch, stream=None) -> None:
    """TX finalize in place (in_delayed_cksum ip_output.c:958-983 + ip_sum :667-672)."""
    check("mi_cksum_ipv4_finalize", load().mi_cksum_ipv4_finalize(C.byref(b.c), C.c_void_p(_stream(stream))))


def span_batch(b: PktBatch, lanes: int = MI_SPAN_STREAM, *, seeds=None, src=None, dst=None, proto=None,
               plens=None, out=None, stream=None):
    """Per-span ~fold(seed + S(span)) -- in_cksum_skip / in_cksum_pseudo_header /
    in_cksum_hdr (lanes=MI_SPAN_ABS) over one-mbuf spans."""
    torch = _torch()
    out = torch.empty(b.n, dtype=torch.uint16, device=b.buf.device) if out is None else out
    keep = [None if x is None else x.contiguous() for x in (seeds, src, dst, proto, plens)]
    s = SpanSeedsC(*[_ptr(x) for x in keep])
    check("mi_cksum_span_batch",
          load().mi_cksum_span_batch(C.byref(b.c), lanes, C.byref(s), out.data_ptr(), C.c_void_p(_stream(stream))))
    return out


class ChainBatch:
    """n mbuf chains gathered into one device buffer (mi_chain_batch).

    ``chains[i]`` is a list of segments, each ``bytes`` or ``(bytes, addr_mod)``
    as for ``MbufChain``; segment data is laid out back to back in a device
    uint8 tensor at offsets == addr_mod (mod 64) from the 64-aligned base, so
    the address parity the reference's swap reacts to is kept.
    """

    def __init__(self, chains, device="cuda"):
        torch = _torch()
        offs, lens, pkt_seg, pos = [], [], [0], 0
        blobs = []
        for ch in chains:
            for seg in ch:
                data, mod = (seg, 0) if isinstance(seg, (bytes, bytearray, memoryview, np.ndarray)) else seg
                raw = np.frombuffer(bytes(data), np.uint8)
                pos += (mod - pos) % 64
                offs.append(pos)
                lens.append(raw.size)
                blobs.append((pos, raw))
                pos += raw.size
            pkt_seg.append(len(offs))
        host = np.zeros(max(pos, 1) + 16, np.uint8)
        for p, raw in blobs:
            host[p:p + raw.size] = raw
        self.n = len(pkt_seg) - 1
        self.buf = torch.from_numpy(host).to(device)
        self.seg_off = torch.tensor(offs or [0], dtype=torch.int64, device=device)
        self.seg_len = torch.tensor(lens or [0], dtype=torch.int32, device=device)
        self.pkt_seg = torch.tensor(pkt_seg, dtype=torch.int32, device=device)
        self.max_seg = max(lens) if lens else 0


def chain_batch(cb: ChainBatch, length, skip, *, src=None, dst=None, proto=None, out=None, stream=None):
    """in_cksum_skip(chain_i, length[i], skip[i]) for every chain, or with
    ``src``/``dst``/``proto`` in_cksum_pseudo_header(chain_i, length[i] (plen),
    skip[i] (off0), src[i], dst[i], proto[i]) -- in_cksum.c:193-276, batched.
    Per-packet arguments are device tensors (int32 / uint32 / uint8)."""
    torch = _torch()
    dev = cb.buf.device
    out = torch.empty(cb.n, dtype=torch.uint16, device=dev) if out is None else out
    pseudo = src is not None
    keep = [torch.as_tensor(length, device=dev).to(torch.int32).contiguous(),
            torch.as_tensor(skip, device=dev).to(torch.int32).contiguous()]
    if pseudo:
        keep += [torch.as_tensor(src, device=dev).to(torch.int64).to(torch.int32).contiguous(),
                 torch.as_tensor(dst, device=dev).to(torch.int64).to(torch.int32).contiguous(),
                 torch.as_tensor(proto, device=dev).to(torch.uint8).contiguous()]
    c = ChainBatchC(cb.buf.data_ptr(), cb.buf.numel(), cb.seg_off.data_ptr(), cb.seg_len.data_ptr(),
                    cb.pkt_seg.data_ptr(), cb.n, MI_CHAIN_PSEUDO if pseudo else MI_CHAIN_SKIP,
                    keep[0].data_ptr(), keep[1].data_ptr(),
                    *([keep[2].data_ptr(), keep[3].data_ptr(), keep[4].data_ptr()] if pseudo else [None] * 3),
                    cb.max_seg, cb.seg_len.numel())
    check("mi_cksum_chain_batch", load().mi_cksum_chain_batch(C.byref(c), out.data_ptr(), C.c_void_p(_stream(stream))))
    return out


def _to_dev(a, dtype: str, dev):
    """numpy / list / tensor -> contiguous device tensor of ``dtype`` (u32
    values wrap into int32, as the C side reads them back as uint32_t)."""
    if a is None:
        return None
    torch = _torch()
    t = a if torch.is_tensor(a) else torch.from_numpy(np.ascontiguousarray(np.asarray(a).astype(np.int64)))
    return t.to(dev).to(getattr(torch, dtype)).contiguous()


class TxBatch:
    """n outgoing frames, each an mbuf chain inside the device uint8 tensor
    ``src`` (segments ``seg_off`` / ``seg_len`` = m_data / m_len, frame i =
    segments [pkt_seg[i], pkt_seg[i+1]), ``pkt_len[i]`` = m_pkthdr.len bytes),
    to be copied into the rte_mbuf data rooms of ``dst`` at
    ``dst_first + i*dst_stride`` (``room`` = buf_len) -- mi_tx_batch.
    ``csum_flags`` / ``csum_data``: m_pkthdr fields (None: by ip_p)."""

    def __init__(self, src, seg_off, seg_len, pkt_seg, pkt_len, dst, *, dst_stride: int, dst_first: int = 0,
                 room: int | None = None, l3_off: int = 14, csum_flags=None, csum_data=None, max_len: int = 0):
        dev = src.device
        self.src, self.dst = src, dst
        self.seg_off = _to_dev(seg_off, "int64", dev)
        self.seg_len = _to_dev(seg_len, "int32", dev)
        self.pkt_seg = _to_dev(pkt_seg, "int32", dev)
        self.pkt_len = _to_dev(pkt_len, "int32", dev)
        self.csum_flags = _to_dev(csum_flags, "int32", dev)
        self.csum_data = _to_dev(csum_data, "int32", dev)
        self.n = int(self.pkt_len.numel())
        room = int(dst_stride) if room is None else int(room)
        self._c = TxBatchC(src.data_ptr(), src.numel(), self.seg_off.data_ptr(), self.seg_len.data_ptr(),
                           self.pkt_seg.data_ptr(), self.pkt_len.data_ptr(), _ptr(self.csum_flags),
                           _ptr(self.csum_data), dst.data_ptr(), dst.numel(), int(dst_stride), int(dst_first),
                           room, int(l3_off), self.n, int(max_len))

    @property
    def c(self) -> TxBatchC:
        return self._c


def tx_copy(tb: TxBatch, *, status=None, stream=None):
    """TX checksum offload fused with the driver's copy (mi_cksum_tx_copy):
    every frame's chain is copied into its slot with ip_sum / the L4 sum
    filled in as in_delayed_cksum + ip_output would.  Returns the per-frame
    status (device uint8: MI_TX_* bits)."""
    torch = _torch()
    status = torch.empty(tb.n, dtype=torch.uint8, device=tb.src.device) if status is None else status
    check("mi_cksum_tx_copy", load().mi_cksum_tx_copy(C.byref(tb.c), status.data_ptr(), C.c_void_p(_stream(stream))))
    return status


def tx_copy_host(src: np.ndarray, seg_off, seg_len, pkt_seg, pkt_len, dst: np.ndarray, *, dst_stride: int,
                 dst_first: int = 0, room: int | None = None, l3_off: int = 14, csum_flags=None, csum_data=None,
                 max_len: int = 0, staged: bool = False) -> np.ndarray:
    """TX copy + sums for frames in host memory (mi_cksum_tx_copy_host): the
    chains in the numpy blob ``src`` are copied into the slots of the numpy
    buffer ``dst`` in place.  Zero-copy when both are registered with
    ``host_register`` (and not ``staged``).  Returns the per-frame status."""
    arr = {k: np.ascontiguousarray(v, dt) if v is not None else None
           for k, v, dt in (("so", seg_off, np.uint64), ("sl", seg_len, np.int32), ("ps", pkt_seg, np.uint32),
                            ("pl", pkt_len, np.uint32), ("cf", csum_flags, np.uint32), ("cd", csum_data, np.uint32))}
    n = int(arr["pl"].size)
    room = int(dst_stride) if room is None else int(room)
    st = np.zeros(max(n, 1), np.uint8)
    c = TxBatchC(src.ctypes.data, src.nbytes, arr["so"].ctypes.data, arr["sl"].ctypes.data, arr["ps"].ctypes.data,
                 arr["pl"].ctypes.data, None if arr["cf"] is None else arr["cf"].ctypes.data,
                 None if arr["cd"] is None else arr["cd"].ctypes.data, dst.ctypes.data, dst.nbytes, int(dst_stride),
                 int(dst_first), room, int(l3_off), n, int(max_len))
    check("mi_cksum_tx_copy_host", load().mi_cksum_tx_copy_host(C.byref(c), st.ctypes.data, 1 if staged else 0))
    return st[:n]


def ipv4_verify_repeat(batches, outs, steps: int, nstreams: int = 1, timing: str = "region",
                       graph: bool = False):
    """Launch ``steps`` verify passes back to back from native code: pass k over
    batches[k % nb] into outs[k % nb] = dict(ip, l4, status), on the library's
    k % nstreams-th non-blocking stream.  Synchronous.

    timing="none" -> None; "region" -> GPU span of all passes in us (one
    hipEvent pair around the region per stream); "pass" -> (per-pass durations
    in us, span in us), events around every pass.  ``graph``: submit the passes
    as one cached hipGraph (MI_REPEAT_GRAPH; "none" / "region" only)."""
    mode = {"none": MI_TIME_NONE, "region": MI_TIME_REGION, "pass": MI_TIME_PER_PASS}[timing]
    if graph:
        mode |= MI_REPEAT_GRAPH
    nb = len(batches)
    arr = (PktBatchC * nb)(*[b.c for b in batches])
    VP = C.c_void_p * nb
    ptrs = {k: VP(*[_ptr(o.get(k)) for o in outs]) for k in ("ip", "l4", "status")}
    us = (C.c_float * steps)() if mode == MI_TIME_PER_PASS else None
    span = C.c_float(0.0)
    check("mi_cksum_ipv4_verify_repeat",
          load().mi_cksum_ipv4_verify_repeat(arr, nb, ptrs["ip"], ptrs["l4"], ptrs["status"], steps, nstreams,
                                             mode, us, C.byref(span)))
    mode &= ~MI_REPEAT_GRAPH
    if mode == MI_TIME_NONE:
        return None
    if mode == MI_TIME_REGION:
        return float(span.value)
    return np.frombuffer(us, dtype=np.float32).copy(), float(span.value)


class VerifyRepeat:
    """A prepared back-to-back verify submission (mi_cksum_repeat_*): pass k
    over batches[k % nb] into outs[k % nb], on the k % nstreams-th of the
    handle's own non-blocking streams.  Everything is marshalled once here, so
    ``run`` costs one ctypes call plus the launches and the wait.

    ``engine="aql"`` (mi_cksum_repeat_set_engine, MI_REPEAT_ENGINE_AQL): the
    passes go out as prebuilt AQL packets in the handle's own HSA queue(s)
    instead of HIP launches (verify only; the batches' producers must have
    completed -- ``after_default`` waits for the legacy stream on the host)."""

    def __init__(self, batches, outs=None, nstreams: int = 2, op: str = "verify", engine: str = "hip"):
        nb = len(batches)
        self._keep = (batches, outs)
        arr = (PktBatchC * nb)(*[b.c for b in batches])
        VP = C.c_void_p * nb
        outs = outs or [{} for _ in batches]
        ptrs = {k: VP(*[_ptr(o.get(k)) for o in outs]) for k in ("ip", "l4", "status")}
        h = C.c_void_p()
        lib = load()
        check("mi_cksum_repeat_create",
              lib.mi_cksum_repeat_create(arr, nb, ptrs["ip"], ptrs["l4"], ptrs["status"], nstreams, C.byref(h)))
        self._h = h
        if op != "verify":
            check("mi_cksum_repeat_set_op",
                  lib.mi_cksum_repeat_set_op(h, {"finalize": 1}[op]))
        self.engine = engine
        if engine != "hip":
            check("mi_cksum_repeat_set_engine", lib.mi_cksum_repeat_set_engine(h, {"aql": 1}[engine]))
        self._run = lib.mi_cksum_repeat_run
        self._span = C.c_float(0.0)
        self._span_ref = C.byref(self._span)

    def run(self, steps: int, *, timed: bool = False, after_default: bool = False, wait: bool = True) -> None:
        """Submit ``steps`` passes (and wait for them unless ``wait=False``).
        ``timed``: hipEvents bracket the passes; read the GPU span with
        ``span()`` afterwards (outside a caller's timed region)."""
        flags = ((MI_TIME_REGION if timed else 0) | (MI_REPEAT_AFTER_DEFAULT if after_default else 0)
                 | (0 if wait else MI_REPEAT_ASYNC))
        rc = self._run(self._h, steps, flags, None)
        if rc:
            check("mi_cksum_repeat_run", rc)

    def span(self) -> float:
        """Wait for the last timed run and return its GPU span in us."""
        check("mi_cksum_repeat_span", load().mi_cksum_repeat_span(self._h, self._span_ref))
        return float(self._span.value)

    def close(self) -> None:
        if self._h:
            load().mi_cksum_repeat_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class TxRepeat(VerifyRepeat):
    """A prepared back-to-back fused-TX submission (mi_cksum_tx_repeat_create):
    pass k copies batches[k % nb] (TxBatch) with its sums into its slots and
    its per-frame status into statuses[k % nb] (device uint8, n each), on the
    handle's streams.  ``engine="aql"``: prebuilt AQL packets of the default
    TX kernel instead of HIP launches.  ``run`` / ``span`` / ``close`` as for
    VerifyRepeat."""

    def __init__(self, batches, statuses, nstreams: int = 2, engine: str = "hip"):
        nb = len(batches)
        if len(statuses) != nb:
            raise ValueError("one status array per batch")
        self._keep = (batches, statuses)
        arr = (TxBatchC * nb)(*[b.c for b in batches])
        VP = C.c_void_p * nb
        st = VP(*[_ptr(s) for s in statuses])
        h = C.c_void_p()
        lib = load()
        check("mi_cksum_tx_repeat_create", lib.mi_cksum_tx_repeat_create(arr, nb, st, nstreams, C.byref(h)))
        self._h = h
        self.engine = engine
        if engine != "hip":
            check("mi_cksum_repeat_set_engine", lib.mi_cksum_repeat_set_engine(h, {"aql": 1}[engine]))
        self._run = lib.mi_cksum_repeat_run
        self._span = C.c_float(0.0)
        self._span_ref = C.byref(self._span)


def synth_ipv4(b: PktBatch, seed: int = 0x5EED5EED, stream=None) -> None:
    """Device-side workload generator (not part of the reference API)."""
    check("mi_cksum_synth_ipv4", load().mi_cksum_synth_ipv4(C.byref(b.c), seed, C.c_void_p(_stream(stream))))


def _host_batch(buf: np.ndarray, n: int, offs, stride, first_off, lens, fixed_len, staged, demux, offs32):
    if offs is not None and offs32:
        o = np.asarray(offs)
        if o.size and int(o.max()) >= 1 << 32:
            raise ValueError("offs32: an offset does not fit in 32 bits")
        offs = np.ascontiguousarray(o, np.uint32)
    elif offs is not None:
        offs = np.ascontiguousarray(offs, np.uint64)
    lens = None if lens is None else np.ascontiguousarray(lens, np.uint32)
    hb = PktBatchC(buf.ctypes.data, buf.nbytes, None if offs is None else offs.ctypes.data, stride, first_off,
                   None if lens is None else lens.ctypes.data, fixed_len, n,
                   int(lens.max()) if lens is not None and n else fixed_len,
                   (MI_BATCH_HOST_STAGED if staged else 0) | (MI_BATCH_DEMUX if demux else 0)
                   | (MI_BATCH_OFFS32 if offs is not None and offs32 else 0))
    return hb, (offs, lens)


def ipv4_verify_host(buf: np.ndarray, n: int, *, offs=None, stride: int = 0, first_off: int = 0, lens=None,
                     fixed_len: int = 0, staged: bool = False, demux: bool = False, offs32: bool = False):
    """Host-resident batch (mi_cksum_ipv4_verify_host).  Returns numpy
    (ip, l4, status, bad_count).  A ``buf`` registered with host_register is
    read in place by the kernel over PCIe (zero-copy) unless ``staged``;
    otherwise chunked H2D -> verify -> D2H.  ``offs32``: pass the offsets as
    u32 (MI_BATCH_OFFS32)."""
    hb, keep = _host_batch(buf, n, offs, stride, first_off, lens, fixed_len, staged, demux, offs32)
    ip = np.zeros(n, np.uint16); l4 = np.zeros(n, np.uint16); st = np.zeros(n, np.uint8)
    bad = C.c_uint32(0)
    check("mi_cksum_ipv4_verify_host",
          load().mi_cksum_ipv4_verify_host(C.byref(hb), ip.ctypes.data, l4.ctypes.data, st.ctypes.data,
                                           C.addressof(bad)))
    del keep
    return ip, l4, st, int(bad.value)


def rx_offload_host(buf: np.ndarray, n: int, *, offs=None, stride: int = 0, first_off: int = 0, lens=None,
                    fixed_len: int = 0, staged: bool = False, demux: bool = False, offs32: bool = False):
    """RX offload flags for a host-resident burst (mi_cksum_rx_offload_host):
    numpy (csum_flags u32, csum_data u32, bad_count)."""
    hb, keep = _host_batch(buf, n, offs, stride, first_off, lens, fixed_len, staged, demux, offs32)
    fl = np.zeros(n, np.uint32); cd = np.zeros(n, np.uint32)
    bad = C.c_uint32(0)
    check("mi_cksum_rx_offload_host",
          load().mi_cksum_rx_offload_host(C.byref(hb), fl.ctypes.data, cd.ctypes.data, C.addressof(bad)))
    del keep
    return fl, cd, int(bad.value)


def host_register(buf: np.ndarray) -> None:
    """mi_cksum_host_register.  Register memory owned page by page (e.g.
    ``page_buffer``), never a view into a malloc heap block that Python may
    free and reuse while the pages are locked."""
    check("mi_cksum_host_register", load().mi_cksum_host_register(buf.ctypes.data, buf.nbytes))


def page_buffer(nbytes: int) -> np.ndarray:
    """A uint8 array of ``nbytes`` on pages of its own: an anonymous mmap,
    page-aligned, that no other object shares and that malloc never hands
    out again -- what host_register should be given (the role DPDK's
    hugepage memory plays for the reference's mbufs)."""
    import mmap
    m = mmap.mmap(-1, max(1, (nbytes + 4095) & ~4095))
    return np.frombuffer(m, np.uint8, count=nbytes)


def set_dropin_mode(mode: str) -> str:
    """Serve the (b1) drop-ins on the CPU ("host", the default) or through the
    device's drop-in service ("gpu"); returns the previous mode."""
    from ._lib import MI_DROPIN_GPU, MI_DROPIN_HOST
    names = {MI_DROPIN_HOST: "host", MI_DROPIN_GPU: "gpu"}
    was = load().mi_cksum_set_dropin_mode({"host": MI_DROPIN_HOST, "gpu": MI_DROPIN_GPU}[mode])
    check("mi_cksum_set_dropin_mode", min(was, 0))
    return names[was]


def dropin_degraded() -> int:
    """GPU-mode drop-in calls that an error sent to the host fold."""
    return int(load().mi_cksum_dropin_degraded())


def host_unregister(buf: np.ndarray) -> None:
    check("mi_cksum_host_unregister", load().mi_cksum_host_unregister(buf.ctypes.data))


def set_busy_wait(on: bool = True) -> None:
    """Busy-poll completion waits on the current device (mi_cksum_set_busy_wait)."""
    check("mi_cksum_set_busy_wait", load().mi_cksum_set_busy_wait(1 if on else 0))


def set_shape(group: int = 0, chunks: int = 0, max_blocks: int = 0) -> None:
    """Force the kernels' lane-group shape / grid cap (0 = automatic); speed only."""
    check("mi_cksum_set_shape", load().mi_cksum_set_shape(group, chunks, max_blocks))


def set_run_kernel(chunks: int = 0, slots: int = 0) -> None:
    """Flat-run kernel for packed batches: 0 = register streaming (default),
    else the LDS-DMA kernel with `chunks` x `slots` (mi_cksum_set_run_kernel)."""
    check("mi_cksum_set_run_kernel", load().mi_cksum_set_run_kernel(chunks, slots))


def init(device: int = 0) -> None:
    check("mi_cksum_init", load().mi_cksum_init(device))


def device_count() -> int:
    return int(load().mi_cksum_device_count())


def version() -> str:
    return load().mi_cksum_version().decode()


__all__ = [
    "MbufChain", "in_cksum_skip", "in_cksum", "in_cksum_pseudo_header", "in_cksum_hdr", "in_pseudo",
    "in_addword", "PktBatch", "ipv4_verify", "ipv4_finalize", "span_batch", "synth_ipv4",
    "ipv4_verify_host", "ipv4_verify_multi", "rx_offload_host", "ipv4_verify_repeat", "VerifyRepeat", "host_register", "host_unregister", "set_shape", "set_run_kernel", "set_busy_wait", "init", "device_count", "version",
    "MI_SPAN_STREAM", "MI_SPAN_ABS", "TxBatch", "tx_copy", "tx_copy_host",
]
