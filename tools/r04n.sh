#!/bin/bash
# round-4 GPU step: the multi-batch next-unit offset prefetch (commit 90aebba,
# opt-in MI_MULTI_DESC_PF) measured once, parity first
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04n; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "verify_multi" > $O/gpu_tests_multi.log 2>&1 || { tail -30 $O/gpu_tests_multi.log; exit 1; }
MI_CKSUM_LIB=tools/ab/libmicksum_pf.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "verify_multi" > $O/gpu_tests_multi_pf.log 2>&1 || { tail -30 $O/gpu_tests_multi_pf.log; exit 1; }
tail -1 $O/gpu_tests_multi.log $O/gpu_tests_multi_pf.log
for r in 0 1; do
  for v in base pf; do
    lib=""; [ $v = pf ] && lib=tools/ab/libmicksum_pf.so
    MI_CKSUM_LIB=$lib timeout -k 10 200 python -u tools/bench_multi.py --offs --ms 4,16 --shapes auto | sed "s/^{/{\"lib\": \"$v\", \"round\": $r, /" >> $O/multi_pf.jsonl || exit 1
  done
done
cut -c1-220 $O/multi_pf.jsonl
echo done
