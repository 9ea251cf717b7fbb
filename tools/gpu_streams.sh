#!/bin/bash
# bench.py per stream count (1500 / 9000 / pareto / 64), one JSON line each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/streams.jsonl
for cfg in ${CFGS:-1500 9000}; do
  for ns in ${NS:-1 2 3 4}; do
    timeout -k 10 120 python bench.py --config $cfg --streams $ns --cpu-seconds 0 --no-host-path >> gpurun_out/streams.jsonl 2>> gpurun_out/streams.err || exit $?
  done
done
echo "exit 0"
