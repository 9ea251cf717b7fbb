#!/bin/bash
# TX copy shape sweep (one JSON line per shape) on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/tx_sweep.jsonl
for sh in ${SHAPES:-8x2 8x4 8x8 16x2 16x4 16x6 16x8}; do
  timeout -k 10 120 python tools/bench_tx.py --shape $sh --cpu-seconds 0 --steps 100 ${TX_ARGS:-} >> gpurun_out/tx_sweep.jsonl 2>> gpurun_out/tx_sweep.err || exit $?
done
echo "exit 0"
