"""Synthetic IPv4 packet batches (host side, numpy).

Lays out batches the way the reference's RX path sees them:
each IPv4 datagram sits in a slot after a 128 B rte_mbuf headroom and a 14 B
Ethernet header, so the IP header is at an address == 2 (mod 4)
(uinet_if_dpdk.c:859-863 + if_ethersubr.c:1059).  Slot strides: 2176 B for
1500 B frames (rte_mbuf data room 2048 + headroom 128, rte_mbuf.h:753-754),
9216 B for 9000 B frames, 64 B for minimum frames (IP at +14 in a 64 B slot).

Headers carry TX-style seeds, as tcp_output.c:1063-1085 / udp_usrreq.c:1233-1241
leave them before in_delayed_cksum (ip_output.c:958-983): ip_sum = 0 and the
L4 checksum field = in_pseudo(src, dst, htons(l4_len + proto)).  Running the
TX finalize (GPU ``ipv4_finalize`` or the oracle) then yields packets whose RX
verify is 0/0.

Nothing here computes a checksum over packet bytes.
"""
from __future__ import annotations

import numpy as np

ETH_HLEN = 14
HEADROOM = 128
IP_OFF = HEADROOM + ETH_HLEN  # 142: IP header offset inside a slot
IPPROTO_TCP = 6
IPPROTO_UDP = 17

# SURVEY.md 8(d) geometry
STRIDE_1500 = 2176
STRIDE_9000 = 9216
STRIDE_64 = 64
MIN_FRAME_IP_LEN = 46  # 64 B frame - 14 B Ethernet - 4 B FCS


def _fold(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64)
    for _ in range(4):
        x = (x & 0xFFFF) + (x >> 16)
    return x


def _swap16(x):
    x = np.asarray(x, dtype=np.uint64) & 0xFFFF
    return ((x & 0xFF) << 8) | (x >> 8)


def in_pseudo_seed(src_le: np.ndarray, dst_le: np.ndarray, l4_len: np.ndarray, proto: np.ndarray) -> np.ndarray:
    """in_pseudo(src, dst, htons(l4_len + proto)) (in_cksum.c:181-191): the
    non-complemented seed tcp_output/udp_output store in the L4 sum field."""
    c = _swap16(np.asarray(l4_len, np.uint64) + np.asarray(proto, np.uint64))
    return _fold(src_le.astype(np.uint64) + dst_le.astype(np.uint64) + c).astype(np.uint16)


def _be16(buf, pos, val):
    buf[pos] = (val >> 8) & 0xFF
    buf[pos + 1] = val & 0xFF


def build_ipv4_batch(n: int, frame_len, *, stride: int | None = None, first_off: int = IP_OFF,
                     offs=None, proto=IPPROTO_TCP, hl=20, seed: int = 0x5EED5EED,
                     buf_size: int | None = None, payload: str = "random") -> dict:
    """Build ``n`` IPv4 datagrams with TX seeds (not yet checksummed).

    frame_len: int or array -- datagram length L (ip_len) per packet.
    Placement: fixed slots (``stride``, ``first_off``) or explicit ``offs``.
    proto / hl: scalars or per-packet arrays (hl in bytes, multiple of 4, 20..60).
    Returns dict(buf, n, offs, stride, first_off, flen) where ``flen`` is the
    per-packet available length (= L here).
    """
    rng = np.random.default_rng(seed)
    L = np.broadcast_to(np.asarray(frame_len, np.int64), (n,)).copy()
    P = np.broadcast_to(np.asarray(proto, np.int64), (n,)).copy()
    H = np.broadcast_to(np.asarray(hl, np.int64), (n,)).copy()
    if offs is None:
        assert stride is not None
        o = first_off + np.arange(n, dtype=np.int64) * stride
    else:
        o = np.asarray(offs, np.int64)
    end = int((o + L).max()) if n else 0
    size = buf_size or (end + 64)
    size = (size + 63) & ~63
    buf = np.zeros(size, np.uint8)
    if payload == "random":
        # fill only the datagram bytes (gaps stay zero, as fresh mbufs would not)
        for i in range(n):
            buf[o[i]:o[i] + L[i]] = rng.integers(0, 256, int(L[i]), dtype=np.uint8)
    elif payload == "pattern":
        for i in range(n):
            buf[o[i]:o[i] + L[i]] = (np.arange(L[i]) + i) & 0xFF
    src = np.zeros(n, np.uint32)
    dst = np.zeros(n, np.uint32)
    for i in range(n):
        p = int(o[i]); hlen = int(H[i]); ln = int(L[i])
        if ln < 20:
            continue
        buf[p] = 0x40 | (hlen // 4)
        buf[p + 1] = 0
        _be16(buf, p + 2, ln)
        _be16(buf, p + 4, i & 0xFFFF)
        _be16(buf, p + 6, 0x4000)
        buf[p + 8] = 64
        buf[p + 9] = int(P[i]) & 0xFF
        buf[p + 10] = buf[p + 11] = 0
        s = bytes([10, 0, (i >> 8) & 0xFF, i & 0xFF])
        d = bytes([10, 1, (i >> 8) & 0xFF, i & 0xFF])
        buf[p + 12:p + 16] = np.frombuffer(s, np.uint8)
        buf[p + 16:p + 20] = np.frombuffer(d, np.uint8)
        src[i] = int.from_bytes(s, "little")
        dst[i] = int.from_bytes(d, "little")
        l4 = p + hlen
        l4len = ln - hlen
        if P[i] == IPPROTO_TCP and l4len >= 20 and hlen <= ln:
            _be16(buf, l4 + 0, 40000 + (i % 1000)); _be16(buf, l4 + 2, 5201)
            buf[l4 + 12] = 5 << 4; buf[l4 + 13] = 0x10
            _be16(buf, l4 + 14, 65535)
            seed16 = int(in_pseudo_seed(np.array([src[i]]), np.array([dst[i]]), np.array([l4len]),
                                        np.array([IPPROTO_TCP]))[0])
            buf[l4 + 16] = seed16 & 0xFF; buf[l4 + 17] = seed16 >> 8  # stored as a host-order u16
            buf[l4 + 18] = buf[l4 + 19] = 0
        elif P[i] == IPPROTO_UDP and l4len >= 8 and hlen <= ln:
            _be16(buf, l4 + 0, 40000 + (i % 1000)); _be16(buf, l4 + 2, 5201)
            _be16(buf, l4 + 4, l4len)
            seed16 = int(in_pseudo_seed(np.array([src[i]]), np.array([dst[i]]), np.array([l4len]),
                                        np.array([IPPROTO_UDP]))[0])
            buf[l4 + 6] = seed16 & 0xFF; buf[l4 + 7] = seed16 >> 8
    return dict(buf=buf, n=n, offs=o.astype(np.uint64), stride=stride or 0, first_off=first_off,
                flen=L.astype(np.uint32), src=src, dst=dst)


def pareto_lengths(n: int, seed: int = 0x9A7E70, lo: int = 64, hi: int = 9000, alpha: float = 1.16) -> np.ndarray:
    """SURVEY.md 8(d) mixed config: L = min(hi, floor(lo * U^(-1/alpha)))."""
    rng = np.random.default_rng(seed)
    u = 1.0 - rng.random(n)  # (0, 1]
    return np.minimum(hi, np.floor(lo * u ** (-1.0 / alpha))).astype(np.int64)


def packed_offsets(lengths: np.ndarray, first_off: int = 0, align: int = 8) -> np.ndarray:
    """Back-to-back placement at ``align``-aligned offsets (Pareto config)."""
    sz = (np.asarray(lengths, np.int64) + align - 1) // align * align
    o = np.zeros(len(sz), np.int64)
    if len(sz):
        o[1:] = np.cumsum(sz)[:-1]
    return (o + first_off).astype(np.uint64)


# ------------------------------------------------------------- TX mbuf chains
MSIZE = 256           # param.h:159
MHLEN_OFF = 56        # m_pktdat inside a packet-header mbuf (MSIZE - MHLEN, mbuf.h)
MCLBYTES = 2048       # param.h


def build_tx_chains(n: int, ip_len, *, layout: str = "socket", proto=IPPROTO_TCP, hl=20,
                    seed: int = 0x7E57, l3_off: int = ETH_HLEN) -> dict:
    """``n`` outgoing Ethernet frames as mbuf chains in one source blob, with
    the sums still to be done (ip_sum = 0, L4 field = in_pseudo seed), as
    ip_output hands them to the driver under if_hwassist (ip_output.c:649-672).

    layout:
      "socket" -- what tcp_output builds (tcp_output.c:848-900): a header mbuf
                  (256 B, data near its end after M_PREPEND of the link header)
                  holding Ethernet + IP + TCP headers, then the payload as
                  references into 2 KiB socket-buffer clusters at a running
                  offset (1 or 2 pieces per frame);
      "single" -- the whole frame in one cluster (m_data 16-aligned + 2);
      "random" -- random cut points (zero-length mbufs, 1-byte mbufs, the IP
                  header split across mbufs) at random addresses mod 64.
    Returns dict(src, seg_off, seg_len, pkt_seg, pkt_len, frames) -- ``frames``
    are the contiguous frame bytes (what m_copydata yields).
    """
    rng = np.random.default_rng(seed)
    L = np.broadcast_to(np.asarray(ip_len, np.int64), (n,)).copy()
    dg = build_ipv4_batch(n, L, stride=int(L.max()) + 64, first_off=0, proto=proto, hl=hl, seed=seed)
    frames = []
    for i in range(n):
        o = int(dg["offs"][i])
        eth = bytes([0x02, 0, 0, 0, 0, 1, 0x02, 0, 0, 0, 0, 2, 0x08, 0x00])[:l3_off].ljust(l3_off, b"\0")
        frames.append(eth + dg["buf"][o:o + int(L[i])].tobytes())
    blob = bytearray()
    seg_off, seg_len, pkt_seg = [], [], [0]

    def put(data: bytes, addr_mod: int, align: int = 64):
        pad = (addr_mod - len(blob)) % align
        blob.extend(b"\0" * pad)
        seg_off.append(len(blob))
        seg_len.append(len(data))
        blob.extend(data)

    sb_off = 0  # running offset in the socket buffer's clusters
    for i, fr in enumerate(frames):
        hdr_len = l3_off + (int(np.broadcast_to(hl, (n,))[i])) + (20 if int(np.broadcast_to(proto, (n,))[i]) == IPPROTO_TCP else 8)
        if layout == "socket":
            hdr_len = min(hdr_len, len(fr))
            put(fr[:hdr_len], (MSIZE - 16 - hdr_len) % 64)  # header mbuf: data ends near m_dat's end
            pay = fr[hdr_len:]
            while pay:
                room = MCLBYTES - sb_off % MCLBYTES
                take = min(room, len(pay))
                put(pay[:take], sb_off % MCLBYTES % 64)
                pay = pay[take:]
                sb_off += take
        elif layout == "single":
            put(fr, 2)
        elif layout == "random":
            cuts = sorted(set(int(c) for c in rng.integers(0, len(fr) + 1, int(rng.integers(0, 6)))))
            if rng.random() < 0.3:  # split the IP header
                cuts.append(l3_off + int(rng.integers(1, 20)))
            cuts = sorted(c for c in set(cuts) if 0 <= c <= len(fr))
            prev = 0
            for c in cuts + [len(fr)]:
                put(fr[prev:c], int(rng.integers(0, 64)))
                if rng.random() < 0.1:
                    put(b"", int(rng.integers(0, 64)))  # zero-length mbuf
                prev = c
        else:
            raise ValueError(layout)
        pkt_seg.append(len(seg_off))
    blob.extend(b"\0" * (64 + (-len(blob)) % 64))
    return dict(src=np.frombuffer(bytes(blob), np.uint8).copy(), seg_off=np.array(seg_off, np.uint64),
                seg_len=np.array(seg_len, np.int32), pkt_seg=np.array(pkt_seg, np.uint32),
                pkt_len=np.array([len(f) for f in frames], np.uint32), frames=frames)
