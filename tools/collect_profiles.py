#!/usr/bin/env python3
"""Copy the judged evidence of tools/gpu_profile_all.sh into profiles/.

    python tools/collect_profiles.py [--src gpurun_out/prof_all] [--round r01]

Per config: the bench line, rocprofv3's kernel stats CSV, a summary of the
kernel trace (per-kernel mean dispatch and the verify kernel's GPU time per
launch = union of its overlapping dispatch intervals / dispatches, which is
what bench.py's avg_launch_us measures), and HBM bytes per verify dispatch from
the separate FETCH_SIZE / WRITE_SIZE passes (FETCH_SIZE x2: gfx950 half-count
correction, MI355X_MICROARCH.md) -> profiles/pmc_traffic.json.
"""
import argparse
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out", "prof_all"))
    ap.add_argument("--round", default="r01")
    ap.add_argument("--configs", default="1500 9000 64 pareto")
    a = ap.parse_args()
    prof = os.path.join(ROOT, "profiles")
    tfile = os.path.join(prof, "pmc_traffic.json")
    traffic = json.load(open(tfile)) if os.path.exists(tfile) else {}
    lines = []
    for c in a.configs.split():
        bench = json.load(open(os.path.join(a.src, f"bench_{c}.json")))
        lines.append(bench)
        kt = os.path.join(a.src, f"kt_{c}")
        # the verify kernel that dominates the trace (the bench line names it too)
        stats = open(os.path.join(kt, "run_kernel_stats.csv")).read().splitlines()[1:]
        kern = max((l for l in stats if "k_ipv4_verify" in l), key=lambda l: int(l.rsplit('",', 1)[1].split(",")[1]))
        kern = kern.split('"')[1].split("((anonymous")[0]
        kern = kern.replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::", "")
        short = kern.split("<")[0]
        shutil.copy(os.path.join(kt, "run_kernel_stats.csv"),
                    os.path.join(prof, f"rocprof_kernel_stats_{c}_{a.round}.csv"))
        out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "prof_summary.py"),
                              os.path.join(kt, "run_kernel_trace.csv"), "--kernel", short,
                              "--pmc-fetch", os.path.join(a.src, f"fetch_{c}", "run_counter_collection.csv"),
                              "--pmc-write", os.path.join(a.src, f"write_{c}", "run_counter_collection.csv")],
                             check=True, capture_output=True, text=True).stdout
        shutil.copy(os.path.join(a.src, f"kt_bench_{c}.json"),
                    os.path.join(prof, f"bench_under_rocprof_{c}_{a.round}.json"))
        summ = json.loads(out)
        summ["_bench_kernel"] = kern
        json.dump(summ, open(os.path.join(prof, f"rocprof_summary_{c}_{a.round}.json"), "w"), indent=1)
        k = summ[short]
        alg = bench["roofline"]["alg_bytes_per_launch"]
        traffic[c] = dict(kernel=kern, bytes_per_launch=k["hbm_bytes"], fetch_bytes=k["fetch_bytes"],
                          write_bytes=k["write_bytes"], alg_bytes=alg, traffic_over_alg=round(k["hbm_bytes"] / alg, 4),
                          note=f"rocprofv3 --pmc FETCH_SIZE (x2, gfx950) and --pmc WRITE_SIZE in separate passes, "
                               f"mean over {k['dispatches']} {short} dispatches, round {a.round}")
        print(c, kern, "traffic/alg", traffic[c]["traffic_over_alg"], "gpu us/launch",
              [b["gpu_us_per_launch"] for b in k.get("bursts", [])][-1:], "bench", bench["roofline"]["avg_launch_us"])
    json.dump(traffic, open(tfile, "w"), indent=1)
    if lines and lines[0]["config"]["workload"].startswith("65536 x 1500"):
        json.dump(lines[0], open(os.path.join(prof, f"bench_{a.round}.json"), "w"), indent=1)
    with open(os.path.join(prof, f"bench_all_{a.round}.jsonl"), "w") as f:
        for l in lines:
            f.write(json.dumps(l) + "\n")


if __name__ == "__main__":
    main()
