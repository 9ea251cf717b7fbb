# TX fused copy at the socket layout: rocprofv3 kernel trace + stats, then the
# HBM traffic counters in their own passes (FETCH_SIZE, WRITE_SIZE), as the
# microarch guide prescribes.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/txprof
rm -rf $OUT && mkdir -p $OUT
timeout -k 10 180 python tools/bench_tx.py --cpu-seconds 0 --steps 200 > $OUT/bench_plain.json || exit 1
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $OUT/trace -o tx -- python3 tools/bench_tx.py --cpu-seconds 0 --steps 200 > $OUT/bench_under_rocprof.json 2> $OUT/trace.log || { tail -n 20 $OUT/trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o pmc -- python3 tools/bench_tx.py --cpu-seconds 0 --steps 20 --warmup 5 > $OUT/pmc_fetch.log 2>&1 || { tail -n 20 $OUT/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o pmc -- python3 tools/bench_tx.py --cpu-seconds 0 --steps 20 --warmup 5 > $OUT/pmc_write.log 2>&1 || { tail -n 20 $OUT/pmc_write.log; exit 1; }
find $OUT -name "*stats*" | head
python tools/pmc_summary.py $OUT/pmc_fetch/pmc_results.db $OUT/pmc_write/pmc_results.db --match k_tx_copy
