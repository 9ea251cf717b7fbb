"""TX copy + checksum offload test batches, shared by
the CPU oracle tests and the GPU parity tests.

A case is a host-side description: the chains' source blob and descriptors,
the destination geometry, optional m_pkthdr csum_flags / csum_data, and the
destination's initial bytes (random, so bytes a frame must not touch are
checked too).
"""
from __future__ import annotations

import numpy as np

from libunsod_amd import synth

CSUM_IP, CSUM_TCP, CSUM_UDP = 0x1, 0x2, 0x4


def onesadd(a: int, b: int) -> int:
    s = a + b
    return (s & 0xFFFF) + (s >> 16)


def make_case(n, ip_len, *, layout="socket", seed=1, proto=6, hl=20, l3=14, dst_first=128, stride=2176,
              room=None, flags=None, data=None) -> dict:
    d = synth.build_tx_chains(n, ip_len, layout=layout, proto=proto, hl=hl, seed=seed, l3_off=l3)
    rng = np.random.default_rng(seed + 99)
    room = stride - dst_first if room is None else room
    dst = rng.integers(0, 256, dst_first + n * stride + 64, dtype=np.uint8)
    return dict(src=d["src"], seg_off=d["seg_off"], seg_len=d["seg_len"], pkt_seg=d["pkt_seg"],
                pkt_len=d["pkt_len"].copy(), dst=dst, dst_first=dst_first, stride=stride, room=room, l3=l3,
                flags=flags, data=data, frames=d["frames"])


def run_oracle(orc, c: dict):
    """(dst bytes, status) the software stack would produce."""
    dst = c["dst"].copy()
    st = orc.tx_copy_batch(c["src"], c["seg_off"], c["seg_len"], c["pkt_seg"], c["pkt_len"], dst,
                           dst_stride=c["stride"], dst_first=c["dst_first"], room=c["room"], l3_off=c["l3"],
                           csum_flags=c["flags"], csum_data=c["data"])
    return dst, st


def zero_udp_sum_case(orc, seed=5) -> dict:
    """UDP frames whose computed L4 sum is 0, so in_delayed_cksum stores 0xffff
    (ip_output.c:967-968): a payload word is adjusted by the would-be sum."""
    c = make_case(4, [200, 333, 1500, 64], layout="single", proto=17, seed=seed)
    for i in range(4):
        _, st = run_oracle(orc, c)
        dst, _ = run_oracle(orc, c)
        fr = dst[c["dst_first"] + i * c["stride"]:][:int(c["pkt_len"][i])]
        ip = c["l3"]
        cur = int(fr[ip + 20 + 6]) | int(fr[ip + 20 + 7]) << 8  # the sum the stack stored
        k = int(c["seg_off"][c["pkt_seg"][i]]) + ip + 20 + 8   # first payload word (even offset)
        w = int(c["src"][k]) | int(c["src"][k + 1]) << 8
        w2 = onesadd(w, cur)
        c["src"][k], c["src"][k + 1] = w2 & 0xFF, w2 >> 8
    return c


def edge_cases(orc) -> list[tuple[str, dict]]:
    out = []
    rng = np.random.default_rng(7)
    out.append(("socket-1514", make_case(64, 1500, layout="socket", seed=11)))
    out.append(("single-1514-odd-dst", make_case(32, 1500, layout="single", seed=12, dst_first=131)))
    out.append(("single-9014", make_case(8, 9000, layout="single", seed=13, stride=9216 + 128, dst_first=128)))
    out.append(("socket-9014", make_case(8, 9000, layout="socket", seed=14, stride=9216 + 128)))
    lens = rng.integers(20, 1500, 96)
    out.append(("random-mixed", make_case(96, lens, layout="random", seed=15, dst_first=2)))
    out.append(("random-udp-opts", make_case(64, rng.integers(60, 1500, 64), layout="random", seed=16, proto=17,
                                             hl=rng.choice([20, 24, 40, 60], 64), dst_first=5)))
    out.append(("icmp-default-flags", make_case(16, 300, layout="socket", proto=1, seed=17)))
    out.append(("raw-ip-l3-0", make_case(16, 700, layout="random", seed=18, l3=0, dst_first=1)))
    out.append(("vlan-l3-18", make_case(16, 700, layout="socket", seed=19, l3=18)))
    c = make_case(32, 1500, layout="socket", seed=20)
    c["flags"] = rng.choice([0, CSUM_IP, CSUM_TCP, CSUM_IP | CSUM_TCP, CSUM_IP | CSUM_UDP], 32).astype(np.uint32)
    c["data"] = rng.choice([16, 16, 16, 6, 0, 34, 1000, 3000], 32).astype(np.uint32)
    out.append(("flags-and-data", c))
    c = make_case(16, 1500, layout="socket", seed=21)
    c["pkt_len"][3] += 10          # chain too short
    c["pkt_len"][5] = c["room"] + 1  # does not fit the slot
    c["pkt_len"][7] = 30           # shorter than the IP datagram: malformed
    c["pkt_len"][9] = 10           # not even a link header + IP header
    out.append(("short-nobufs-malformed", c))
    # > 16 segments per frame (the generic path)
    d = make_case(8, 1500, layout="socket", seed=22)
    out.append(("many-segments", _resegment(d, 40)))
    out.append(("zero-udp-sum", zero_udp_sum_case(orc)))
    # Ethernet padding after the datagram (short frames padded to 60 B, and
    # a few full-size ones): the L4 sum must stop at ip_len
    out.append(("eth-padding", _pad_frames(make_case(40, rng.integers(28, 47, 40), layout="single", proto=17,
                                                     seed=23), rng.integers(0, 20, 40))))
    out.append(("eth-padding-socket", _pad_frames(make_case(24, 1400, layout="socket", seed=24),
                                                  rng.integers(1, 40, 24))))
    # IP header and TCP sum far into the slot: l3 = 64, 60-byte IP header,
    # 15 bytes into the first 16-byte chunk
    out.append(("l3-64-hl-60", make_case(24, 900, layout="socket", seed=25, l3=64, hl=60, dst_first=15)))
    # more frames than one wave's group, ragged count, mixed layouts' lengths
    out.append(("ragged-count-mixed", make_case(203, rng.integers(20, 1500, 203), layout="socket", seed=26,
                                                dst_first=7)))
    return out


def _pad_frames(c: dict, pad) -> dict:
    """Extend every frame's last mbuf by pad[i] bytes (whatever follows it in
    the blob): pkt_len grows, the IP datagram does not."""
    c = dict(c)
    sl, pl = c["seg_len"].copy(), c["pkt_len"].copy()
    for i in range(len(pl)):
        sl[int(c["pkt_seg"][i + 1]) - 1] += int(pad[i])
        pl[i] += int(pad[i])
    c.update(seg_len=sl, pkt_len=pl)
    return c


def _resegment(c: dict, nseg: int) -> dict:
    """Cut every frame into nseg pieces (some empty) at odd addresses."""
    rng = np.random.default_rng(nseg)
    blob, so, sl, ps = bytearray(), [], [], [0]
    for fr in c["frames"]:
        cuts = np.sort(rng.integers(0, len(fr) + 1, nseg - 1))
        prev = 0
        for x in list(cuts) + [len(fr)]:
            blob.extend(b"\0" * int(rng.integers(1, 8)))
            so.append(len(blob))
            sl.append(int(x) - prev)
            blob.extend(fr[prev:int(x)])
            prev = int(x)
        ps.append(len(so))
    blob.extend(b"\0" * (64 + (-len(blob)) % 64))
    c = dict(c)
    c.update(src=np.frombuffer(bytes(blob), np.uint8).copy(), seg_off=np.array(so, np.uint64),
             seg_len=np.array(sl, np.int32), pkt_seg=np.array(ps, np.uint32))
    return c
