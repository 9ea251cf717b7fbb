# TX copy shapes: bench lines + one SQ counter pass per shape (tools/pmc_summary.py)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/tx_flat.jsonl gpurun_out/pmc_tx_*
SHAPES=${SHAPES:-"8x2 f16x2 f16x4 8x4 16x2"}
for s in $SHAPES; do MI_CKSUM_TX_SHAPE=$s timeout -k 10 120 python tools/bench_tx.py --cpu-seconds 0 >> gpurun_out/tx_flat.jsonl || exit 1; done
python -c "
import json
for l in open('gpurun_out/tx_flat.jsonl'):
    d=json.loads(l); print(d['shape'], d['us_per_launch'], d['isolated_us'], d['roofline']['frac'])"
PMC_SHAPES=${PMC_SHAPES:-"8x2 f16x2"}
for s in $PMC_SHAPES; do
MI_CKSUM_TX_SHAPE=$s timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU -d gpurun_out/pmc_tx_$s -o pmc -- python3 tools/bench_tx.py --cpu-seconds 0 --steps 20 --warmup 5 > gpurun_out/pmc_tx_$s.log 2>&1 || { tail -n 20 gpurun_out/pmc_tx_$s.log; exit 1; }
done
python tools/pmc_summary.py gpurun_out/pmc_tx_*/pmc_results.db --match tx_
