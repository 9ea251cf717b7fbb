#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
rm -f gpurun_out/b6_*.jsonl
for i in 1 2; do
for w in stream event spin; do
  MI_CKSUM_REPEAT_WAIT=$w MI_CKSUM_REPEAT_TRACE=1 timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-host-path --no-dropin --warm-regions 8 >> gpurun_out/b6_$w.jsonl 2>/dev/null
done
done
echo done
