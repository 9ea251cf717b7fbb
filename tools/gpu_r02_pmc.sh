#!/bin/bash
# PMC traffic per config (FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/pmc2
mkdir -p $O
rc=0
for c in 9000 64 pareto; do
  A="--config $c --steps 30 --warmup 5 --settle 0 --cpu-seconds 0 --no-host-path --no-dropin --warm-regions 0"
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$c -o run --output-format csv -- python3 bench.py $A > /dev/null 2>> $O/err && \
  timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d $O/write_$c -o run --output-format csv -- python3 bench.py $A > /dev/null 2>> $O/err || { rc=1; break; }
  echo "pmc $c done"
done
exit $rc
