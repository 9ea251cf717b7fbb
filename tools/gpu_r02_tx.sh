#!/bin/bash
# Round-2: TX finalize (whole-block stores) parity + timing, A/B against byte stores.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_tx_finalize_gpu.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tx_tests.log 2>&1
tail -2 gpurun_out/tx_tests.log
timeout -k 10 300 python -u tools/bench_finalize.py > gpurun_out/fin_blocks.jsonl
MI_CKSUM_TX_BLOCKS=0 timeout -k 10 300 python -u tools/bench_finalize.py --configs 1500,9000 > gpurun_out/fin_bytes.jsonl
echo done
