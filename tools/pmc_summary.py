#!/usr/bin/env python3
"""Per-kernel mean of every PMC counter in rocprofv3 result databases
(rocpd SQLite, the `counters_collection` view), one JSON line per kernel.

    python tools/pmc_summary.py gpurun_out/pmc_tx_*/pmc_results.db [--match tx_]
    python tools/pmc_summary.py --trace gpurun_out/txprof/trace/tx_results.db --match k_tx_copy
"""
from __future__ import annotations

import argparse
import collections
import json
import re
import sqlite3


def summarize(db: str, match: str = ""):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(counters_collection)")]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in c.execute("select * from counters_collection"):
        d = dict(zip(cols, r))
        name = d.get("kernel_name") or ""
        if match and match not in name:
            continue
        agg[name][d["counter_name"]].append(float(d["value"]))
    for name, m in agg.items():
        short = re.search(r"::(\w+(<[^>]*>)?)\(", name)
        yield dict(db=db, kernel=short.group(1) if short else name, dispatches=max(len(v) for v in m.values()),
                   **{k: round(sum(v) / len(v), 1) for k, v in sorted(m.items())})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dbs", nargs="+")
    ap.add_argument("--match", default="")
    ap.add_argument("--trace", action="store_true", help="the dbs are --kernel-trace databases: dispatch stats")
    a = ap.parse_args()
    for db in a.dbs:
        if a.trace:
            print(json.dumps(trace_union(db, a.match)))
            continue
        for row in summarize(db, a.match):
            print(json.dumps(row))



def trace_union(db: str, match: str):
    """Per-kernel dispatch statistics from a rocprofv3 --kernel-trace database:
    count, mean / min / max duration, and the union of the dispatch intervals
    per dispatch (the GPU time per launch when launches overlap on 2 streams)."""
    c = sqlite3.connect(db)
    iv = sorted((s, e) for n, s, e in c.execute("select name, start, end from kernels") if match in n)
    if not iv:
        return None
    union, cs, ce = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > ce:
            union += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    union += ce - cs
    d = [e - s for s, e in iv]
    return dict(db=db, kernel=match, dispatches=len(iv), mean_us=round(sum(d) / len(d) / 1e3, 3),
                min_us=round(min(d) / 1e3, 3), max_us=round(max(d) / 1e3, 3),
                union_us_per_dispatch=round(union / len(iv) / 1e3, 3))


if __name__ == "__main__":
    main()
