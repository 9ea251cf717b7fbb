#!/bin/bash
# PMC of TX finalize vs RX verify on the same 1500 B batches (one pass per counter group).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS="tools/bench_finalize.py --configs ${CFGS:-1500} --rounds 1 --steps 100"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/fin_trace -o run --output-format csv -- python3 $ARGS > gpurun_out/fin_trace.jsonl 2> gpurun_out/fin_trace.err && \
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES \
    -d gpurun_out/fin_pmc_sq -o run --output-format csv -- python3 $ARGS > /dev/null 2> gpurun_out/fin_pmc_sq.err && \
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/fin_pmc_fetch -o run --output-format csv -- python3 $ARGS > /dev/null 2> gpurun_out/fin_pmc_fetch.err && \
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/fin_pmc_write -o run --output-format csv -- python3 $ARGS > /dev/null 2> gpurun_out/fin_pmc_write.err
rc=$?
echo "exit $rc"
exit $rc
