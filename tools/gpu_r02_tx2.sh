#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_tx_finalize_gpu.py tests/test_gpu_parity.py tests/test_host_gpu.py tests/test_demux_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tx_tests.log 2>&1
tail -2 gpurun_out/tx_tests.log
rm -f gpurun_out/fin5.jsonl
timeout -k 10 300 python -u tools/bench_finalize.py --configs 1500,9000,pareto,64 >> gpurun_out/fin5.jsonl
MI_CKSUM_TX_BLOCKS=0 timeout -k 10 300 python -u tools/bench_finalize.py --configs 1500,9000 --rounds 1 >> gpurun_out/fin5.jsonl
echo done
