#!/bin/bash
# SQ counters for the TX copy bench (one rocprofv3 pass, counters only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
    -d gpurun_out/pmc_tx -o run --output-format csv -- python3 tools/bench_tx.py --steps 40 --warmup 5 --cpu-seconds 0 ${TX_ARGS:-} > gpurun_out/pmc_tx.json 2> gpurun_out/pmc_tx.err
rc=$?
echo "exit $rc"
exit $rc
