#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/grid_iso.py --config 1500 > gpurun_out/grid_iso.jsonl
timeout -k 10 200 python -u tools/grid_iso.py --config 9000 --caps 512,1024,1280,2048,4096 >> gpurun_out/grid_iso.jsonl
echo done
