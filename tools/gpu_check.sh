#!/bin/bash
# One GPU round-trip: parity tests, smoke, bench, kernel-trace profile.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out
rocm-smi --showproductname > $OUT/smi.txt 2>&1 || true
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/prof -o run --output-format csv -- \
    python3 bench.py --steps 200 --cpu-seconds 0 --no-host-path > $OUT/prof_bench.json 2> $OUT/prof.err
rc=$?
echo "exit $rc"
tail -3 $OUT/pytest_gpu.log; cat $OUT/smoke.log 2>/dev/null | tail -2; cat $OUT/bench.json 2>/dev/null
exit $rc
