#!/usr/bin/env python3
"""HBM bytes per dispatch from the L2's memory-side request counters split by
request size (rocprofv3 --pmc CSV, one pass for reads, one for writes):

    reads  = 32 B x RDREQ_32B + 64 B x RDREQ_64B + 128 B x RDREQ_128B
    writes = 64 B x WRREQ_64B + 32 B x (WRREQ - WRREQ_64B)

(RDREQ counts 32-byte and 64-byte requests, a 128-byte request once, which is
why FETCH_SIZE = 64 B x RDREQ reads half of a wide streaming read on gfx950.)
One JSON line per (CSV, kernel): median over its dispatches.

    python tools/pmc_reqsize.py gpurun_out/TAG/pmc_*/run_counter_collection.csv [--match verify]
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import re
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csvs", nargs="+")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    for path in a.csvs:
        per = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"]
            if "rocclr" in name or (a.match and a.match not in name):
                continue
            short = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", "").replace("void ", "")) or "(AQL dispatch)"
            per[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, m in per.items():
            med = {c: statistics.median(v) for c, v in m.items()}
            out = dict(csv=path, kernel=k, dispatches=max(len(v) for v in m.values()), **{c: round(x) for c, x in med.items()})
            if "TCC_EA0_RDREQ_32B_sum" in med:
                out["read_bytes"] = round(32 * med["TCC_EA0_RDREQ_32B_sum"] + 64 * med.get("TCC_EA0_RDREQ_64B_sum", 0)
                                          + 128 * med.get("TCC_EA0_RDREQ_128B_sum", 0))
                out["fetch_size_bytes"] = round(64 * med.get("TCC_EA0_RDREQ_sum", 0))
            if "TCC_EA0_WRREQ_sum" in med:
                w64 = med.get("TCC_EA0_WRREQ_64B_sum", 0)
                out["write_bytes"] = round(64 * w64 + 32 * (med["TCC_EA0_WRREQ_sum"] - w64))
            print(json.dumps(out))


if __name__ == "__main__":
    main()
