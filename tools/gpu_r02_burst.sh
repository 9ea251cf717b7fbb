#!/bin/bash
# Host-memory burst path with the one-shot AQL dispatch vs HIP launch +
# stream synchronize: the host-path parity tests, then per-burst latency.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/burst
mkdir -p $O
echo "== tests"
timeout -k 10 300 python -u -m pytest tests/test_host_gpu.py tests/test_gpu_parity.py -k "host" -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -12 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for aql in 1 0; do
  echo "== burst aql=$aql"
  MI_CKSUM_HOST_AQL=$aql timeout -k 10 240 python -u tools/bench_burst.py --sizes ${BURST_SIZES:-32,128,512,4096} > $O/burst_aql$aql.jsonl 2> $O/burst.err || exit 1
  cat $O/burst_aql$aql.jsonl | cut -c1-240
done
