#!/bin/bash
# bench.py over every BASELINE config on one GPU (one JSON line each).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/bench_all.jsonl
for cfg in 1500 9000 64 pareto; do
  timeout -k 10 300 python bench.py --config $cfg --cpu-seconds ${CPU_SECONDS:-5} >> gpurun_out/bench_all.jsonl 2> gpurun_out/bench_$cfg.err || exit $?
done
echo "exit 0"
