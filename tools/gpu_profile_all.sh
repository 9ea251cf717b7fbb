#!/bin/bash
# Round-end evidence for every bench config on one GPU: the bench line, a
# kernel-trace + stats profile of the same command, then FETCH_SIZE and
# WRITE_SIZE each in their own rocprofv3 pass (counters + kernel names only, as
# MI355X_MICROARCH.md prescribes).  Every GPU step has its own time limit and
# the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/prof_all
mkdir -p $O
CFGS=${CFGS:-1500 9000 64 pareto}
for c in $CFGS; do
  A="--config $c --cpu-seconds 0 --no-host-path"
  timeout -k 10 300 python bench.py --config $c --cpu-seconds ${CPU_SECONDS:-10} > $O/bench_$c.json 2> $O/bench_$c.err && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$c -o run --output-format csv -- \
      python3 bench.py $A > $O/kt_bench_$c.json 2> $O/kt_$c.err && \
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$c -o run --output-format csv -- \
      python3 bench.py $A --steps 50 --warmup 5 --settle 0 > /dev/null 2> $O/fetch_$c.err && \
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/write_$c -o run --output-format csv -- \
      python3 bench.py $A --steps 50 --warmup 5 --settle 0 > /dev/null 2> $O/write_$c.err || { echo "failed at $c"; exit 1; }
  echo "$c done: $(cat $O/bench_$c.json)"
done
echo "exit 0"
