#!/bin/bash
# round-4 GPU step: TX kernels (parity + A/B), Pareto waves A/B, grid sweep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04d; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -k "tx or verify_multi" > $O/gpu_tests_tx.log 2>&1 || { tail -30 $O/gpu_tests_tx.log; exit 1; }
tail -1 $O/gpu_tests_tx.log
for r in 0 1; do
  for k in pair wave; do
    for lay in socket single; do
      MI_CKSUM_TX_KERNEL=$k timeout -k 10 120 python -u tools/bench_tx.py --layout $lay --steps 200 --cpu-seconds 0 $([ $r = 0 ] && echo --check) \
        | sed "s/^{/{\"kernel\": \"$k\", \"round\": $r, /" >> $O/tx_ab.jsonl || exit 1
    done
  done
done
cut -c1-200 $O/tx_ab.jsonl
timeout -k 10 500 python -u tools/ab.py --config pareto --rounds 3 --steps 200 w4: w1::MI_CKSUM_RUN_WAVES=1 w2::MI_CKSUM_RUN_WAVES=2 > $O/ab_pareto_waves.jsonl 2> $O/ab.err || exit 1
cut -c1-160 $O/ab_pareto_waves.jsonl
timeout -k 10 300 python -u tools/grid_iso.py --config 1500 --caps 1024,1280,2048,2560 > $O/grid_iso.jsonl 2> $O/grid_iso.err || exit 1
cut -c1-250 $O/grid_iso.jsonl
timeout -k 10 120 python -u tools/dropin_breakdown.py --calls 400 > $O/dropin_breakdown.jsonl 2> $O/dropin.err || exit 1
cut -c1-300 $O/dropin_breakdown.jsonl
for r in 0 1; do for d in 0 1; do
  MI_CKSUM_MULTI_DYN=$d timeout -k 10 200 python -u tools/bench_multi.py --ms 4,16 --shapes auto,16x6 | sed "s/^{/{\"dyn\": $d, \"round\": $r, /" >> $O/multi_dyn.jsonl || exit 1
done; done
cut -c1-220 $O/multi_dyn.jsonl
echo done
