#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
rm -f gpurun_out/defer_ab.jsonl
L=$PWD/libunsod_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_tx_finalize_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tx_tests.log 2>&1
tail -1 gpurun_out/tx_tests.log
for i in 1 2; do
  for lib in libmicksum.so libmicksum_nodefer.so; do
    MI_CKSUM_LIB=$L/$lib timeout -k 10 300 python -u tools/bench_finalize.py --configs 1500,9000,pareto,64 --ops verify,finalize --rounds 1 >> gpurun_out/defer_ab.jsonl
  done
done
echo done
