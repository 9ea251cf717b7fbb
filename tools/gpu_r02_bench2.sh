#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-host-path --no-dropin --probe-regions 8 > gpurun_out/b2_$i.json 2> gpurun_out/b2_$i.err
  echo "bench $i done"
done
for w in spin event; do
  MI_CKSUM_REPEAT_WAIT=$w timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-host-path --no-dropin --probe-regions 8 > gpurun_out/b2_$w.json 2> gpurun_out/b2_$w.err
done
echo done
