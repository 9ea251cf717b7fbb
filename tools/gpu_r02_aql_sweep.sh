#!/bin/bash
# AQL engine variants on the driver-equivalent bench line (20 steps, 1500 B):
# one or two HSA queues, release fence at system or agent scope; HIP launches
# as the reference point.  Interleaved rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/aql${SWEEP_TAG:-}
mkdir -p $O
mv -f $O/sweep.jsonl $O/sweep_prev.jsonl 2>/dev/null
# (first pass, barrier bit 0: one queue 17.9 us per pass, two 15.0-15.2, HIP
# 14.7-15.0; agent vs system release no difference)
VARIANTS=(${AQL_VARIANTS:-"launch:2:system:1" "aql:2:system:1" "aql:2:system:0" "aql:3:system:1" "aql:4:system:1"})
for round in $(seq 1 ${ROUNDS:-3}); do
  for v in "${VARIANTS[@]}"; do
    IFS=: read sub ns rel bar <<< "$v"
    echo "== $round $v"
    line=$(MI_CKSUM_AQL_BARRIER=${bar:-1} MI_CKSUM_AQL_RELEASE=$rel MI_CKSUM_REPEAT_TRACE=1 timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 \
           --submit $sub --streams $ns --no-dropin --no-host-path --cpu-seconds 0 $BENCH_ARGS 2>> $O/sweep.err) || exit 1
    python - "$v" "$line" >> $O/sweep.jsonl <<'PY'
import json, sys
d = json.loads(sys.argv[2])
r = d["roofline"]
print(json.dumps(dict(variant=sys.argv[1], value=d["value"], ms_per_step=d["ms_per_step"],
                      avg_launch_us=r["avg_launch_us"], frac=r["frac"], wall_frac=r["wall_frac"],
                      trace=d.get("host_trace_us"), warm=d.get("warm_region_walls_us"))))
PY
    tail -1 $O/sweep.jsonl
  done
done
