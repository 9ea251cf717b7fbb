#!/bin/bash
# bench.py with host launches vs one hipGraph per timed region, every config.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/submit.jsonl
for cfg in ${CFGS:-1500 9000 64 pareto}; do
  for sub in launch graph; do
    timeout -k 10 120 python bench.py --config $cfg --submit $sub --cpu-seconds 0 --no-host-path >> gpurun_out/submit.jsonl 2>> gpurun_out/submit.err || exit $?
  done
done
echo "exit 0"
