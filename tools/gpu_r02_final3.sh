#!/bin/bash
# Round-2 closing evidence: full GPU suite, the driver's bench line, 400 steps,
# the other configs, and a rocprofv3 kernel trace (HIP-launch submission: the
# profiler serializes the AQL engine's queues).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/final3
mkdir -p $O
step() { echo "== $*"; }
step tests && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 && tail -1 $O/gpu_tests.log && \
step bench && timeout -k 10 240 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_1500.json 2> $O/bench_1500.err && \
step bench400 && timeout -k 10 240 python -u bench.py --gpus 1 --steps 400 --warmup 5 --cpu-seconds 0 --no-host-path --no-dropin > $O/bench_1500_k400.json 2>> $O/bench.err && \
for c in 9000 64 pareto; do
  step bench $c && timeout -k 10 240 python -u bench.py --gpus 1 --steps 20 --warmup 5 --config $c --cpu-seconds 3 --no-dropin > $O/bench_$c.json 2>> $O/bench.err || exit 1
done && \
step rocprof && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_1500 -o run --output-format csv -- python3 bench.py --steps 400 --warmup 5 --submit launch --cpu-seconds 0 --no-host-path --no-dropin > $O/trace_1500.json 2> $O/trace_1500.err
rc=$?
echo "exit $rc"
exit $rc
