#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "multi" --timeout 120 --timeout-method thread > gpurun_out/multi_tests.log 2>&1
MI_CKSUM_MULTI_INTERLEAVE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "multi" --timeout 120 --timeout-method thread >> gpurun_out/multi_tests.log 2>&1
tail -1 gpurun_out/multi_tests.log
timeout -k 10 200 python -u tools/bench_multi.py --config 1500 > gpurun_out/multi2.jsonl
MI_CKSUM_MULTI_INTERLEAVE=1 timeout -k 10 200 python -u tools/bench_multi.py --config 1500 | sed 's/}$/, "interleave": 1}/' >> gpurun_out/multi2.jsonl
echo done
