#!/bin/bash
# Flat-run kernel grid cap (MI_CKSUM_RUN_BLOCKS) on the Pareto and 64 B configs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/run_blocks.jsonl
for cfg in pareto 64; do
  for b in ${BLOCKS:-1024 2048 4096 8192 16384}; do
    MI_CKSUM_RUN_BLOCKS=$b timeout -k 10 120 python bench.py --config $cfg --cpu-seconds 0 --no-host-path | sed "s/^{/{\"run_blocks\": $b, /" >> gpurun_out/run_blocks.jsonl 2>> gpurun_out/run_blocks.err || exit $?
  done
done
echo "exit 0"
