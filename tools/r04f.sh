#!/bin/bash
# round-4 GPU step: drop-in service (parity, lifetimes, breakdown); TX copy
# register diet A/B (in-tree vs LDS-parked at 4 / 5 waves per SIMD)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04f; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "dropin or service or threads or link or tx or aql" > $O/gpu_tests_dropin.log 2>&1 || { tail -40 $O/gpu_tests_dropin.log; exit 1; }
tail -1 $O/gpu_tests_dropin.log
timeout -k 10 180 python -u tools/dropin_breakdown.py --calls 400 > $O/dropin_breakdown.jsonl 2> $O/dropin.err || { tail $O/dropin.err; exit 1; }
cut -c1-420 $O/dropin_breakdown.jsonl
for r in 0 1; do
  for v in base tx4 tx5 tx5b; do
    for lay in socket single; do
      MI_CKSUM_LIB=tools/ab/libmicksum_$v.so timeout -k 10 120 python -u tools/bench_tx.py --layout $lay --steps 200 --cpu-seconds 0 $([ $r = 0 ] && echo --check) \
        | sed "s/^{/{\"lib\": \"$v\", \"round\": $r, /" >> $O/tx_lds_ab.jsonl || exit 1
    done
  done
done
python3 -c "
import json
for l in open('$O/tx_lds_ab.jsonl'):
    d=json.loads(l); print(d['lib'], d['round'], d['layout'], d['us_per_launch'], round(d['roofline']['frac'],3), d.get('check'))
"
echo done
