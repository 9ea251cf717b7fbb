#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_link_gpu.py tests/test_host_gpu.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/misc_tests.log 2>&1
tail -2 gpurun_out/misc_tests.log
timeout -k 10 60 oracle/_ref/linktest > gpurun_out/linktest.json
timeout -k 10 300 python -u tools/bench_burst.py > gpurun_out/burst.jsonl
echo done
