#!/bin/bash
# Pareto flat run: grid cap of the flat-run kernel (MI_CKSUM_MAX_BLOCKS; default
# 16384 = one 64-datagram run per wave for 2^22 datagrams).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/runcap
mkdir -p $O
rm -f $O/cap.jsonl
for round in 1 2; do
  for cap in 0 1024 2048 4096 8192; do
    e=""; [ $cap -gt 0 ] && e="MI_CKSUM_MAX_BLOCKS=$cap"
    line=$(env $e timeout -k 10 150 python -u bench.py --config pareto --steps 20 --warmup 5 --no-dropin --no-host-path --cpu-seconds 0 2>> $O/cap.err) || exit 1
    python - "$cap" "$line" >> $O/cap.jsonl <<'PY'
import json, sys
d = json.loads(sys.argv[2]); r = d["roofline"]
print(json.dumps(dict(cap=int(sys.argv[1]), value=d["value"], avg_launch_us=r["avg_launch_us"], frac=r["frac"], wall_frac=r["wall_frac"])))
PY
    tail -1 $O/cap.jsonl
  done
done
