#!/usr/bin/env python3
"""Per-kernel mean of every PMC counter in rocprofv3 result databases
(rocpd SQLite, the `counters_collection` view), one JSON line per kernel.

    python tools/pmc_summary.py gpurun_out/pmc_tx_*/pmc_results.db [--match tx_]
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
    a = ap.parse_args()
    for db in a.dbs:
        for row in summarize(db, a.match):
            print(json.dumps(row))


if __name__ == "__main__":
    main()
