#!/bin/bash
# Round-2 probe: wall-clock overhead of short timed regions and the read
# ceiling of the bench's pattern (tools/overhead_probe.py, tools/ceiling.py).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for w in spin event stream; do
  MI_CKSUM_REPEAT_WAIT=$w timeout -k 10 300 python -u tools/overhead_probe.py --tag "$w" > "gpurun_out/overhead_$w.jsonl"
  echo "overhead $w done"
done
timeout -k 10 300 python -u tools/ceiling.py > gpurun_out/ceiling.jsonl
echo "ceiling done"
