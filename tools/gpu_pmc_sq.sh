#!/bin/bash
# SQ (instruction / wait) counters for one bench config, then FETCH_SIZE and
# WRITE_SIZE -- each in its own rocprofv3 pass (counters + kernel names only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
CFG=${CFG:-1500}
ARGS="--config $CFG --steps 50 --warmup 5 --settle 0 --cpu-seconds 0 --no-host-path --no-dropin --submit launch"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT \
    -d gpurun_out/pmc_sq_$CFG -o run --output-format csv -- python3 bench.py $ARGS > /dev/null 2> gpurun_out/pmc_sq_$CFG.err && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$CFG -o run --output-format csv -- \
    python3 bench.py $ARGS > /dev/null 2> gpurun_out/pmc_fetch_$CFG.err && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$CFG -o run --output-format csv -- \
    python3 bench.py $ARGS > /dev/null 2> gpurun_out/pmc_write_$CFG.err
rc=$?
echo "exit $rc"
exit $rc
