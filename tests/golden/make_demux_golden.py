#!/usr/bin/env python3
"""Golden vectors for the MI_BATCH_DEMUX path (small-header callers), from
the REFERENCE's own in_cksum.c (oracle/_ref/libref.so, see make_golden.py),
driven the way ip_input's protocol input routines call it
(oracle/batch_driver.c demux_l4 / the demux finalize).

    python tests/golden/make_demux_golden.py   # writes tests/golden/demux_golden.npz
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from oracle.pyoracle import Oracle  # noqa: E402
from demux_cases import build_demux_batch, to_rx  # noqa: E402

OUT = os.path.join(HERE, "demux_golden.npz")


def aligned_copy(a):
    """A 64-aligned copy, so address parity == offset parity."""
    raw = np.zeros(a.size + 128, np.uint8)
    s = (-raw.ctypes.data) % 64
    v = raw[s:s + a.size]
    v[:] = a
    return raw, v


def main():
    o = Oracle("reference")
    d = build_demux_batch()
    n = len(d["offs"])
    kw = dict(offs=d["offs"], flen=d["flen"], demux=True)
    keep1, fin = aligned_copy(d["buf"])
    o.ipv4_finalize_batch(fin, n, **kw)
    fin_out = fin.copy()
    ver_in = to_rx(fin_out, d)
    keep2, ver = aligned_copy(ver_in)
    ip, l4, st = o.ipv4_verify_batch(ver, n, **kw)
    # every rule is exercised
    for bit in (0, 1, 2, 4, 8):
        assert ((st == 0) if bit == 0 else (st & bit) != 0).any(), bit
    for p in (6, 17, 1, 2, 112):
        assert ((d["proto"] == p) & (st == 0)).any(), p
    np.savez_compressed(OUT, fin_in=d["buf"], fin_out=fin_out, ver_in=ver_in, offs=d["offs"],
                        flen=d["flen"], ip=ip, l4=l4, st=st)
    print(f"wrote {OUT}: {n} datagrams, status counts",
          {b: int(((st & b) != 0).sum()) for b in (1, 2, 4, 8)}, "valid", int((st == 0).sum()))


if __name__ == "__main__":
    main()
