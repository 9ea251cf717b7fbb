#!/bin/bash
# One GPU round-trip: parity tests, smoke, bench, kernel-trace profile of the
# same bench command.  Every GPU step has its own time limit; the chain stops
# at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out
BENCH_ARGS=${BENCH_ARGS:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py $BENCH_ARGS > $OUT/bench.json 2> $OUT/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/prof -o run --output-format csv -- \
    python3 bench.py $BENCH_ARGS --cpu-seconds 0 --no-host-path > $OUT/prof_bench.json 2> $OUT/prof.err && \
python tools/prof_summary.py $OUT/prof/run_kernel_trace.csv > $OUT/prof_summary.json && \
if [ -n "$SWEEP" ]; then timeout -k 10 900 python tools/sweep.py $SWEEP > $OUT/sweep.jsonl 2> $OUT/sweep.err; fi
rc=$?
echo "exit $rc"
tail -3 $OUT/pytest_gpu.log; tail -2 $OUT/smoke.log 2>/dev/null; cat $OUT/bench.json 2>/dev/null
exit $rc
