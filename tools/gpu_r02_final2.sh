#!/bin/bash
# Round-2 measurement pass: GPU tests, the driver's bench line, the other
# configs, rocprofv3 kernel trace of the headline command, PMC traffic passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/final2
O=gpurun_out/final2
step() { echo "== $*"; }
step tests && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 && tail -1 $O/gpu_tests.log && \
step bench && timeout -k 10 240 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_1500.json 2> $O/bench_1500.err && \
step bench400 && timeout -k 10 240 python -u bench.py --gpus 1 --steps 400 --warmup 5 --cpu-seconds 0 --no-host-path --no-dropin > $O/bench_1500_k400.json 2>> $O/bench.err && \
for c in 9000 64 pareto; do
  step bench $c && timeout -k 10 240 python -u bench.py --gpus 1 --steps 20 --warmup 5 --config $c --cpu-seconds 3 > $O/bench_$c.json 2>> $O/bench.err || exit 1
done && \
step rocprof && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_1500 -o run --output-format csv -- python3 bench.py --steps 400 --warmup 5 --cpu-seconds 0 --no-host-path --no-dropin > $O/trace_1500.json 2> $O/trace_1500.err && \
step rocprof9000 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_9000 -o run --output-format csv -- python3 bench.py --config 9000 --steps 200 --warmup 5 --cpu-seconds 0 --no-host-path --no-dropin > $O/trace_9000.json 2> $O/trace_9000.err && \
step pmc && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_1500 -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --settle 0 --cpu-seconds 0 --no-host-path --no-dropin > /dev/null 2> $O/pmc.err && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_1500 -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --settle 0 --cpu-seconds 0 --no-host-path --no-dropin > /dev/null 2>> $O/pmc.err
rc=$?
echo "exit $rc"
exit $rc
