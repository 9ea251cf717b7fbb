#!/bin/bash
# HBM probe + PMC traffic passes (FETCH_SIZE and WRITE_SIZE in separate runs,
# kernel-trace only besides the counters, as MI355X_MICROARCH.md prescribes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
CFG=${CFG:-1500}
timeout -k 10 180 ./tools/hbm_probe > gpurun_out/hbm_probe.json 2> gpurun_out/hbm_probe.err && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- \
    python3 bench.py --config $CFG --steps 50 --warmup 5 --cpu-seconds 0 --no-host-path > gpurun_out/pmc_fetch.json 2> gpurun_out/pmc_fetch.err && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- \
    python3 bench.py --config $CFG --steps 50 --warmup 5 --cpu-seconds 0 --no-host-path > gpurun_out/pmc_write.json 2> gpurun_out/pmc_write.err
rc=$?
echo "exit $rc"
exit $rc
