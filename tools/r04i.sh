#!/bin/bash
# round-4 GPU step: drop-in service after the one-load mailbox read
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04i; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "dropin or service or threads or link" -s > $O/gpu_tests_dropin.log 2>&1 || { tail -40 $O/gpu_tests_dropin.log; exit 1; }
tail -1 $O/gpu_tests_dropin.log
timeout -k 10 180 python -u tools/dropin_breakdown.py --calls 400 > $O/dropin_breakdown.jsonl 2> $O/dropin.err || { tail $O/dropin.err; exit 1; }
MI_CKSUM_DROPIN_MAILBOX=device timeout -k 10 180 python -u tools/dropin_breakdown.py --calls 400 > $O/dropin_breakdown_devbox.jsonl 2>> $O/dropin.err || { tail $O/dropin.err; exit 1; }
cut -c1-330 $O/dropin_breakdown.jsonl $O/dropin_breakdown_devbox.jsonl
./tools/pool_probe > $O/pool_probe.jsonl 2>&1 || true
cat $O/pool_probe.jsonl
echo done
