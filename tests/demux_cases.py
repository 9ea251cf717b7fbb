"""Mixed-protocol batches for the MI_BATCH_DEMUX path (SURVEY.md 8(f) rank 4:
the small-header callers ICMP / IGMP / CARP, fragments, and the TCP / UDP
length rules of their input routines).  Test data, not product code.

Every twist the protocol input routines react to is present (include/mi_cksum.h
lists them with their reference lines): fragments (IP_MF / offsets), TCP with
fewer than 20 L4 bytes, UDP with uh_ulen shorter than, longer than or below the
header, UDP without a checksum (uh_sum = 0), ICMP below hl + ICMP_ADVLENMIN,
IGMP below IGMP_MINLEN, CARP shorter than / exactly / longer than its 36-byte
header, protocols without an L4 checksum (ESP 50, OSPF 89), IP options,
Ethernet padding past ip_len, odd and even datagram starts.
"""
from __future__ import annotations

import numpy as np

from libunsod_amd.synth import build_ipv4_batch

PROTOS = np.array([6, 17, 1, 2, 112, 50, 89])


def _be16(buf, p, v):
    buf[p] = (v >> 8) & 0xFF
    buf[p + 1] = v & 0xFF


def build_demux_batch(n: int = 720, seed: int = 0xDE3A, max_len: int = 2200) -> dict:
    """``n`` datagrams (TX state: sums not yet computed) packed at odd / even
    offsets; returns dict(buf, offs, flen, proto)."""
    rng = np.random.default_rng(seed)
    proto = rng.choice(PROTOS, n, p=[0.25, 0.3, 0.15, 0.1, 0.1, 0.05, 0.05])
    hl = rng.choice([20, 20, 20, 24, 60], n)
    plen = rng.integers(0, max_len, n)
    short = rng.random(n) < 0.25  # lengths around each protocol's threshold
    thr = np.select([proto == 6, proto == 17, proto == 1, proto == 2, proto == 112],
                    [20, 8, 36, 8, 36], 8)
    plen = np.where(short, np.maximum(thr + rng.integers(-6, 7, n), 0), plen)
    carp_exact = (proto == 112) & (rng.random(n) < 0.4)
    plen = np.where(carp_exact, 36, plen)
    L = hl + plen
    pad = rng.integers(0, 8, n) * (rng.random(n) < 0.3)  # Ethernet padding past ip_len
    sz = L + pad + 1 + rng.integers(0, 9, n)
    offs = np.concatenate([[0], np.cumsum(sz)[:-1]]) + 5
    b = build_ipv4_batch(n, L, offs=offs, proto=proto, hl=hl, seed=seed + 1,
                         buf_size=int(offs[-1] + sz[-1] + 64))
    buf = b["buf"]
    flen = (L + pad).astype(np.uint32)
    for i in range(n):
        p = int(offs[i])
        if pad[i]:
            buf[p + L[i]:p + L[i] + pad[i]] = rng.integers(0, 256, int(pad[i]), dtype=np.uint8)
        r = rng.random()
        if r < 0.06:  # a fragment: MF, an offset, or both
            v = [0x2000, int(rng.integers(1, 0x2000)), 0x2000 | int(rng.integers(1, 0x2000))][i % 3]
            _be16(buf, p + 6, v)
        elif r < 0.08:  # DF plus reserved bit: not a fragment
            _be16(buf, p + 6, 0xC000)
        if proto[i] == 17 and plen[i] >= 8 and rng.random() < 0.3:
            pl = int(plen[i])
            u = int(rng.choice([max(8, pl - int(rng.integers(1, 40))), pl + int(rng.integers(1, 9)),
                                int(rng.integers(0, 8))]))
            _be16(buf, p + int(hl[i]) + 4, u & 0xFFFF)
    return dict(buf=buf, offs=offs.astype(np.uint64), flen=flen, proto=proto, hl=hl, plen=plen)


def to_rx(buf: np.ndarray, d: dict, seed: int = 0xDE3B) -> np.ndarray:
    """A received copy of a finalized batch: some UDP sums zeroed (no
    checksum) and ~8 % of the datagrams with one flipped bit."""
    rng = np.random.default_rng(seed)
    out = buf.copy()
    n = len(d["offs"])
    for i in range(n):
        p, hl, pl = int(d["offs"][i]), int(d["hl"][i]), int(d["plen"][i])
        if d["proto"][i] == 17 and pl >= 8 and rng.random() < 0.15:
            out[p + hl + 6] = out[p + hl + 7] = 0
        if rng.random() < 0.08:
            j = p + int(rng.integers(0, int(d["flen"][i]) or 1))
            out[j] ^= np.uint8(1 << int(rng.integers(8)))
    return out
