#!/usr/bin/env python3
"""Per-config HBM traffic record for bench.py's roofline `traffic` field, from
one round's rocprofv3 --pmc passes (tools/gpu.sh pmc:CFG:..., a read pass with
TCC_EA0_RDREQ_{32B,64B,128B}_sum and a write pass with TCC_EA0_WRREQ{,_64B}_sum):
reads = 32 B x RDREQ_32B + 64 B x RDREQ_64B + 128 B x RDREQ_128B, writes =
64 B x WRREQ_64B + 32 B x the rest (tools/pmc_reqsize.py), median over the
config's verify dispatches.

    python tools/pmc_traffic_json.py gpurun_out/TAG --round r05 > profiles/r05/pmc_traffic_r05.json
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
import statistics

# config -> (record key, kernel-name prefix of its verify kernel, algorithmic bytes per launch)
CONFIGS = {
    "1500": ("1500", "k_ipv4_verify<16, 6>", 65536 * 1500 + 5 * 65536),
    "9000": ("9000", "k_ipv4_verify<8, 12>", 65536 * 9000 + 5 * 65536),
    "64": ("64", "k_ipv4_verify_slot64", (1 << 20) * 46 + 5 * (1 << 20)),
    "pareto": ("pareto_u32", "k_ipv4_verify_packed<8, 0, 2, false>", None),
    # bench.py config_tx: 65536 frames of 1514 B read + written + 1 B status
    "tx": ("tx", "k_tx_lds<2, 2>", 65536 * (2 * 1514 + 1)),
}


def medians(path: str, prefix: str) -> tuple[dict, int]:
    per: dict[str, list] = {}
    for r in csv.DictReader(open(path)):
        name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", ""))
        if name.startswith(prefix):
            per.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {c: statistics.median(v) for c, v in per.items()}, max((len(v) for v in per.values()), default=0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--round", default="r06")
    ap.add_argument("--pareto-alg", type=int, default=1205618850,
                    help="Pareto algorithmic bytes per launch (bench.py's alg_bytes_per_launch)")
    a = ap.parse_args()
    out = {}
    for cfg, (key, prefix, alg) in CONFIGS.items():
        reads = writes = None
        nd = 0
        for path in glob.glob(os.path.join(a.dir, f"pmc_{cfg}_*", "**", "*counter_collection.csv"), recursive=True):
            m, n = medians(path, prefix)
            if "TCC_EA0_RDREQ_32B_sum" in m:
                reads = 32 * m["TCC_EA0_RDREQ_32B_sum"] + 64 * m.get("TCC_EA0_RDREQ_64B_sum", 0) + \
                    128 * m.get("TCC_EA0_RDREQ_128B_sum", 0)
                nd = max(nd, n)
            if "TCC_EA0_WRREQ_sum" in m:
                w64 = m.get("TCC_EA0_WRREQ_64B_sum", 0)
                writes = 64 * w64 + 32 * (m["TCC_EA0_WRREQ_sum"] - w64)
        if reads is None or writes is None:
            continue
        alg = alg if alg is not None else a.pareto_alg
        out[key] = dict(kernel=prefix, bytes_per_launch=round(reads + writes), read_bytes=round(reads),
                        write_bytes=round(writes), alg_bytes_per_launch=alg,
                        traffic_over_alg=round((reads + writes) / alg, 4), dispatches=nd,
                        method=f"rocprofv3 --pmc, two passes over bench.py --submit launch ({a.round} code, "
                               "tools/gpu.sh pmc): reads = 32 B x TCC_EA0_RDREQ_32B + 64 B x _64B + 128 B x _128B, "
                               "writes = 64 B x TCC_EA0_WRREQ_64B + 32 B x the rest; median over the verify "
                               "dispatches (tools/pmc_traffic_json.py)")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
