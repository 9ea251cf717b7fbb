#!/bin/bash
# TX fused copy: every chain layout, plus a rocprofv3 kernel-trace of the socket-layout bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/tx_layouts.jsonl
for lay in socket single random; do
  timeout -k 10 180 python tools/bench_tx.py --layout $lay --check --cpu-seconds ${CPU_SECONDS:-3} >> gpurun_out/tx_layouts.jsonl 2>> gpurun_out/tx_layouts.err || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_tx -o run --output-format csv -- python3 tools/bench_tx.py --cpu-seconds 0 > gpurun_out/kt_tx.json 2> gpurun_out/kt_tx.err
rc=$?
echo "exit $rc"
exit $rc
