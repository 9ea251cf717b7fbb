#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
rm -f gpurun_out/b5_*.jsonl
for e in 1 0 1 0; do
  MI_CKSUM_REPEAT_EXT=$e MI_CKSUM_REPEAT_TRACE=1 timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-host-path --no-dropin --warm-regions 6 >> gpurun_out/b5_$e.jsonl 2> gpurun_out/b5_$e.err
  echo "bench $e done"
done
