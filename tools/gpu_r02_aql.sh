#!/bin/bash
# AQL engine: parity tests first, then the driver-equivalent bench line
# (20 steps, 1500 B) with HIP launches vs AQL packets, interleaved, with the
# repeat handle's host trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/aql
mkdir -p $O
echo "== tests"
timeout -k 10 240 python -u -m pytest tests/test_aql_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -15 $O/tests.log
[ $rc -eq 0 ] || exit $rc
rm -f $O/bench.jsonl
for round in 1 2 3; do
  for sub in ${AQL_SUBMITS:-launch aql}; do
    echo "== $round $sub"
    line=$(MI_CKSUM_REPEAT_TRACE=1 timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --submit $sub \
           --no-dropin --no-host-path --cpu-seconds 0 $BENCH_ARGS 2>> $O/bench.err) || exit 1
    python - "$sub" "$line" >> $O/bench.jsonl <<'PY'
import json, sys
d = json.loads(sys.argv[2])
r = d["roofline"]
print(json.dumps(dict(submit=sys.argv[1], value=d["value"], ms_per_step=d["ms_per_step"],
                      avg_launch_us=r["avg_launch_us"], frac=r["frac"], wall_frac=r["wall_frac"],
                      trace=d.get("host_trace_us"), warm=d.get("warm_region_walls_us"))))
PY
    tail -1 $O/bench.jsonl
  done
done
