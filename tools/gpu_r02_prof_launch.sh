#!/bin/bash
# rocprofv3 kernel trace of the 400-step 1500 B bench with HIP launches
# (--submit launch): rocprofv3 intercepts the AQL engine's own queues and
# serializes their dispatches, so the overlapped per-launch time is traced on
# the HIP path, which runs the same kernel body; the in-process spans of both
# engines come from the same box right before.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/prof_launch
mkdir -p $O
timeout -k 10 240 python -u bench.py --steps 400 --warmup 5 --cpu-seconds 0 --no-host-path --no-dropin > $O/bench_aql_k400.json 2> $O/bench.err && \
timeout -k 10 240 python -u bench.py --steps 400 --warmup 5 --submit launch --cpu-seconds 0 --no-host-path --no-dropin > $O/bench_launch_k400.json 2>> $O/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 400 --warmup 5 --submit launch --cpu-seconds 0 --no-host-path --no-dropin > $O/trace_launch.json 2> $O/trace.err
rc=$?
echo "exit $rc"
exit $rc
