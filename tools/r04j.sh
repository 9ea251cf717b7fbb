#!/bin/bash
# round-4 GPU step: TX grid cap (frames per lane group) and Pareto flat-run grid
# cap (ranges per wave) A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04j; mkdir -p $O
for r in 0 1; do
  for cap in 2048 1024 1536 4096; do
    for lay in socket single; do
      MI_CKSUM_GRID_CAP=$cap timeout -k 10 120 python -u tools/bench_tx.py --layout $lay --steps 200 --cpu-seconds 0 \
        | sed "s/^{/{\"cap\": $cap, \"round\": $r, /" >> $O/tx_cap.jsonl || exit 1
    done
  done
done
python3 -c "
import json
for l in open('$O/tx_cap.jsonl'):
    d=json.loads(l); print(d['cap'], d['round'], d['layout'], d['us_per_launch'], round(d['roofline']['frac'],3))
"
timeout -k 10 600 python -u tools/ab.py --config pareto --rounds 2 --steps 200 c16384: c8192::MI_CKSUM_RUN_BLOCKS=8192 c4096::MI_CKSUM_RUN_BLOCKS=4096 c32768::MI_CKSUM_RUN_BLOCKS=32768 > $O/ab_pareto_cap.jsonl 2> $O/ab.err || { tail $O/ab.err; exit 1; }
cut -c1-140 $O/ab_pareto_cap.jsonl
echo done
