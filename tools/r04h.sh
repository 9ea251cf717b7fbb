#!/bin/bash
# round-4 GPU step: rocprofv3 kernel trace + request-size PMC of the TX fused
# copy (in-tree build), socket and single-segment layouts
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04h; mkdir -p $O
for lay in socket single; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$lay -o tx -- python3 tools/bench_tx.py --layout $lay --steps 200 --cpu-seconds 0 > $O/bench_tx_$lay.json 2> $O/trace_$lay.err || { tail $O/trace_$lay.err; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d $O/pmc_rd_$lay -o rd -- python3 tools/bench_tx.py --layout $lay --steps 10 --cpu-seconds 0 > /dev/null 2> $O/pmc_rd_$lay.err || { tail $O/pmc_rd_$lay.err; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $O/pmc_wr_$lay -o wr -- python3 tools/bench_tx.py --layout $lay --steps 10 --cpu-seconds 0 > /dev/null 2> $O/pmc_wr_$lay.err || { tail $O/pmc_wr_$lay.err; exit 1; }
done
find $O -name "*.csv" | head -20
for f in $(find $O -name "*counter_collection.csv"); do python3 tools/pmc_reqsize.py $f --match tx_copy; done > $O/pmc_reqsize_tx.jsonl
cut -c1-400 $O/pmc_reqsize_tx.jsonl
for f in $(find $O -name "*kernel_stats.csv"); do echo $f; head -5 $f | cut -c1-200; done
echo done
