#!/bin/bash
# Driver-equivalent bench line (20 steps, 1500 B) under HIP runtime settings
# that govern the timed region's fixed costs: how the host waits for the last
# kernel (active spin vs. interrupt), signal scope, kernel-argument placement.
# Two interleaved rounds; one JSON line per run with the setting as "env".
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/envsweep.jsonl
rm -f $O
# (round-2 first pass: ROC_ACTIVE_WAIT_TIMEOUT=100000 no change, 5405 vs 5449
# GiB/s; ROC_SYSTEM_SCOPE_SIGNAL=0 made the bench fail -- dropped)
SETTINGS=(${ENVSWEEP_SETTINGS:-"BASE=1" "HIP_FORCE_DEV_KERNARG=0" "DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0"})
for round in 1 2; do
  for s in "${SETTINGS[@]}"; do
    echo "== $round $s"
    line=$(env $s MI_CKSUM_REPEAT_TRACE=1 timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 \
           --no-dropin --no-host-path --cpu-seconds 0 2>> gpurun_out/envsweep.err) || exit 1
    python - "$s" "$line" >> $O <<'PY'
import json, sys
d = json.loads(sys.argv[2])
r = d["roofline"]
print(json.dumps(dict(env=sys.argv[1], value=d["value"], ms_per_step=d["ms_per_step"], avg_launch_us=r["avg_launch_us"],
                      isolated_us=r["isolated_launch_us"], trace=d.get("host_trace_us"),
                      warm=d.get("warm_region_walls_us"))))
PY
    tail -1 $O
  done
done
