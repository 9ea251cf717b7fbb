#!/bin/bash
# Round-2: GPU tests, then the driver's bench command a few times (+ 9000 B).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  tail -3 gpurun_out/gpu_tests.log
fi
for i in 1 2 3; do
  timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench20_$i.json 2> gpurun_out/bench20_$i.err
  echo "bench $i done"
done
timeout -k 10 180 python -u bench.py --config 9000 --steps 20 --warmup 5 --cpu-seconds 2 > gpurun_out/bench20_9000.json 2> gpurun_out/bench20_9000.err
echo "9000 done"
