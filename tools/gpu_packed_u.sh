#!/bin/bash
# Flat-run kernel chunk depth (MI_CKSUM_PACKED_U) on the Pareto and 64 B configs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/packed_u.jsonl
for cfg in pareto 64; do
  for u in 4 8 16; do
    MI_CKSUM_PACKED_U=$u timeout -k 10 120 python bench.py --config $cfg --streams ${NS:-2} --cpu-seconds 0 --no-host-path | sed "s/^{/{\"packed_u\": $u, /" >> gpurun_out/packed_u.jsonl 2>> gpurun_out/packed_u.err || exit $?
  done
done
echo "exit 0"
