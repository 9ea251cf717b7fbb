#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/hbm_probe > gpurun_out/hbm_probe.json 2> gpurun_out/hbm_probe.err && \
timeout -k 10 900 python tools/sweep.py "$@" > gpurun_out/sweep.jsonl 2> gpurun_out/sweep.err
rc=$?
echo "exit $rc"; tail -3 gpurun_out/sweep.err
exit $rc
