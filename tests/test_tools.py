"""CPU checks of the round-5 measurement tools' own arithmetic: the range
tables tools/pareto_ranges.py hands the byte-balanced kernel (every datagram
in exactly one range of 1-64), and the request-size traffic formula
tools/pmc_traffic_json.py turns rocprofv3 counters into (the bench's roofline
`traffic`)."""
import csv
import importlib.util
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tool(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "tools", name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_range_tables_cover_every_datagram_once():
    pr = _tool("pareto_ranges")
    from libunsod_amd import synth
    lens = synth.pareto_lengths(1 << 14)
    mean64 = float(lens.sum()) / (len(lens) / 64)
    for fn in (pr.greedy, pr.bucket):
        for f in (0.75, 1.0, 1.5):
            st = fn(lens, mean64 * f).astype(np.int64)
            d = np.diff(st)
            assert st[0] == 0 and st[-1] == len(lens)
            assert d.min() >= 1 and d.max() <= 64, (fn.__name__, f)
    # greedy closes a range at T bytes: no range holds T plus more than one datagram
    T = mean64
    st = pr.greedy(lens, T).astype(np.int64)
    rb = np.add.reduceat(lens.astype(np.int64), st[:-1])
    assert rb.max() < T + lens.max()


def test_traffic_from_request_size_counters(tmp_path):
    rows = []
    for disp in range(3):
        for c, v in (("TCC_EA0_RDREQ_32B_sum", 10), ("TCC_EA0_RDREQ_64B_sum", 20), ("TCC_EA0_RDREQ_128B_sum", 1000),
                     ("TCC_EA0_RDREQ_sum", 1030)):
            rows.append(("pmc_1500_rd", "k_ipv4_verify<16, 6>(Desc, unsigned short*)", c, v + disp))
        for c, v in (("TCC_EA0_WRREQ_sum", 50), ("TCC_EA0_WRREQ_64B_sum", 40)):
            rows.append(("pmc_1500_wr", "k_ipv4_verify<16, 6>(Desc, unsigned short*)", c, v))
        rows.append(("pmc_1500_wr", "k_fill(unsigned char*)", "TCC_EA0_WRREQ_sum", 99999))
    for d in ("pmc_1500_rd", "pmc_1500_wr"):
        os.makedirs(tmp_path / d)
        with open(tmp_path / d / "run_counter_collection.csv", "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Kernel_Name", "Counter_Name", "Counter_Value"])
            for dd, k, c, v in rows:
                if dd == d:
                    w.writerow([k, c, v])
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic_json.py"), str(tmp_path)],
                         check=True, capture_output=True, text=True).stdout
    r = json.loads(out)["1500"]
    reads = 32 * 11 + 64 * 21 + 128 * 1001  # medians over the three dispatches
    writes = 64 * 40 + 32 * (50 - 40)
    assert r["read_bytes"] == reads and r["write_bytes"] == writes
    assert r["bytes_per_launch"] == reads + writes and r["alg_bytes_per_launch"] == 65536 * 1505
