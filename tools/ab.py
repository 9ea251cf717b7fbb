#!/usr/bin/env python3
"""Interleaved A/B of library builds / environment knobs through bench.py.

    python tools/ab.py --config pareto --rounds 2 \
        old:tools/ab/libmicksum_old.so new: new_u4::MI_CKSUM_PACKED_U=4

Each spec is NAME:LIB[:ENV=V,ENV=V]; an empty LIB is the in-tree build.  Every
(round, spec) runs `bench.py --steps S --config C` (no side legs) in its own
child process under a time limit, so the builds never share a process; one
JSON line per run: name, value, avg launch us, fraction of 8 TB/s.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("specs", nargs="+")
    ap.add_argument("--config", default="pareto")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--submit", default="aql")
    ap.add_argument("--timeout", type=int, default=240)
    a = ap.parse_args()
    for rnd in range(a.rounds):
        for spec in a.specs:
            name, lib, *rest = spec.split(":") + [""]
            env = dict(os.environ)
            if lib:
                env["MI_CKSUM_LIB"] = os.path.join(ROOT, lib)
            for kv in filter(None, (rest[0] if rest else "").split(",")):
                k, v = kv.split("=", 1)
                env[k] = v
            cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--steps", str(a.steps), "--warmup", "5",
                   "--config", a.config, "--also", "none", "--sustain-seconds", "0", "--cpu-seconds", "0",
                   "--no-host-path", "--no-dropin", "--submit", a.submit]
            p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=a.timeout)
            if p.returncode != 0:
                print(json.dumps(dict(round=rnd, name=name, rc=p.returncode, err=p.stderr[-800:])), flush=True)
                sys.exit(p.returncode)
            line = json.loads(p.stdout.strip().splitlines()[-1])
            rf = line["roofline"]
            print(json.dumps(dict(round=rnd, name=name, spec=spec, value=line["value"], us=rf["avg_launch_us"],
                                  frac=rf["frac"], kernel=rf.get("kernel"), wall_frac=rf.get("wall_frac"))),
                  flush=True)


if __name__ == "__main__":
    main()
