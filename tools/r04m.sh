#!/bin/bash
# round-4 GPU step: host bursts through the drop-in service (parity, latency)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04m; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -k "dropin or service or host or link or threads or demux" > $O/gpu_tests.log 2>&1 || { grep -v amdgpu.ids $O/gpu_tests.log | tail -40; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u tools/bench_burst.py --sizes 1,8,32,64,128,256,512,4096 > $O/burst.jsonl 2> $O/burst.err || { tail $O/burst.err; exit 1; }
cut -c1-300 $O/burst.jsonl
MI_CKSUM_BURST_SERVICE_MAX=0 timeout -k 10 300 python -u tools/bench_burst.py --sizes 1,8,32,64,128 > $O/burst_dispatch.jsonl 2>> $O/burst.err || { tail $O/burst.err; exit 1; }
cut -c1-300 $O/burst_dispatch.jsonl
echo done
