#!/bin/bash
# round-4 GPU step: service bursts with 8 lanes per datagram (64 per round)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04o; mkdir -p $O
MI_CKSUM_LIB=tools/ab/libmicksum_g8.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "host_bursts or service_runs" > $O/gpu_tests_g8.log 2>&1 || { tail -30 $O/gpu_tests_g8.log; exit 1; }
tail -n 1 $O/gpu_tests_g8.log
for r in 0 1; do
  MI_CKSUM_BURST_SERVICE_MAX=128 timeout -k 10 300 python -u tools/bench_burst.py --sizes 1,8,32,64,128 | sed "s/^{/{\"lib\": \"g16\", \"round\": $r, /" >> $O/burst_g.jsonl || exit 1
  MI_CKSUM_LIB=tools/ab/libmicksum_g8.so MI_CKSUM_BURST_SERVICE_MAX=128 timeout -k 10 300 python -u tools/bench_burst.py --sizes 1,8,32,64,128 | sed "s/^{/{\"lib\": \"g8\", \"round\": $r, /" >> $O/burst_g.jsonl || exit 1
done
python3 -c "
import json
for l in open('$O/burst_g.jsonl'):
    d=json.loads(l); print(d['lib'], d['round'], d['burst'], d['gpu_zero_copy'], d['cpu_reference_1thread'])
"
echo done
