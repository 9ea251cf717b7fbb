#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (CSV) for the checksum kernels.

    python tools/prof_summary.py gpurun_out/prof/run_kernel_trace.csv [--kernel NAME]
        [--pmc-fetch DIR/run_counter_collection.csv] [--pmc-write ...]

Per kernel: dispatches, mean / median duration.  For the verify kernel (by
default the k_ipv4_verify* kernel with the most dispatches: k_ipv4_verify for
1500 / 9000 B, k_ipv4_verify_slot64 for 64 B slots, k_ipv4_verify_packed or
k_ipv4_verify_run_dma for Pareto) also the
GPU time per launch = union of its dispatch intervals / dispatches -- when
launches on several streams overlap, per-dispatch durations double-count the
shared time and the union is what bench.py's hipEvent span measures.  With PMC
files: HBM bytes per dispatch, FETCH_SIZE doubled (gfx950 reports half of a
wide streaming read, MI355X_MICROARCH.md section HBM) + WRITE_SIZE, in bytes.
"""
from __future__ import annotations

import argparse
import csv
import json
import re
import statistics
from collections import defaultdict


def short(name: str, templ: bool = False) -> str:
    m = re.search(r"(k_[a-z0-9_]+)(<[^>]*>)?", name)
    if not m:
        return name[:40]
    return m.group(1) + ((m.group(2) or "") if templ else "")


def union_len(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot


def pmc(path):
    out = defaultdict(list)
    for r in csv.DictReader(open(path)):
        out[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: statistics.mean(v) for k, v in out.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default=None, help="kernel whose bursts to report (default: see above)")
    ap.add_argument("--pmc-fetch")
    ap.add_argument("--pmc-write")
    ap.add_argument("--skip-first", type=int, default=0, help="ignore the first N dispatches of the kernel")
    ap.add_argument("--templates", action="store_true", help="keep template arguments in kernel names")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    per = defaultdict(list)
    for r in rows:
        per[short(r["Kernel_Name"], a.templates)].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    res = {}
    for k, iv in per.items():
        d = [e - s for s, e in iv]
        res[k] = dict(dispatches=len(iv), mean_us=round(statistics.mean(d) / 1e3, 3),
                      median_us=round(statistics.median(d) / 1e3, 3))
    if a.kernel is None:
        cand = [k for k in per if k.startswith("k_ipv4_verify")]
        a.kernel = max(cand, key=lambda k: len(per[k])) if cand else ""
    iv = sorted(per.get(a.kernel, []))[a.skip_first:]
    if iv:
        # split into bursts separated by > 1 ms idle (warmup / timed / isolated phases)
        bursts, cur = [], [iv[0]]
        for x in iv[1:]:
            if x[0] - max(e for _, e in cur) > 1_000_000:
                bursts.append(cur)
                cur = [x]
            else:
                cur.append(x)
        bursts.append(cur)
        res[a.kernel]["bursts"] = [dict(dispatches=len(b), gpu_us_per_launch=round(union_len(b) / len(b) / 1e3, 3),
                                        mean_dispatch_us=round(statistics.mean(e - s for s, e in b) / 1e3, 3))
                                   for b in bursts]
    if a.pmc_fetch or a.pmc_write:
        f = pmc(a.pmc_fetch) if a.pmc_fetch else {}
        w = pmc(a.pmc_write) if a.pmc_write else {}
        for k in res:
            fs = f.get((k, "FETCH_SIZE"))
            ws = w.get((k, "WRITE_SIZE"))
            if fs is not None or ws is not None:
                res[k]["fetch_bytes"] = None if fs is None else int(fs * 2 * 1024)
                res[k]["write_bytes"] = None if ws is None else int(ws * 1024)
                res[k]["hbm_bytes"] = int((fs or 0) * 2 * 1024 + (ws or 0) * 1024)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
