#!/bin/bash
# Grid cap / lane-group shape of the 1500 B verify under the AQL engine
# (driver-equivalent 20-step line and 400 steps), interleaved rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/aqlgrid
mkdir -p $O
rm -f $O/g.jsonl
for round in 1 2; do
  for v in "BASE=1" "MI_CKSUM_MAX_BLOCKS=1280" "MI_CKSUM_MAX_BLOCKS=4096" "MI_CKSUM_SHAPE=8x12" "MI_CKSUM_SHAPE=8x4"; do
    for k in 20 400; do
      line=$(env $v timeout -k 10 150 python -u bench.py --steps $k --warmup 5 --no-dropin --no-host-path --cpu-seconds 0 2>> $O/g.err) || exit 1
      python - "$v" "$k" "$line" >> $O/g.jsonl <<'PY'
import json, sys
d = json.loads(sys.argv[3]); r = d["roofline"]
print(json.dumps(dict(variant=sys.argv[1], steps=int(sys.argv[2]), value=d["value"], avg_launch_us=r["avg_launch_us"], frac=r["frac"], wall_frac=r["wall_frac"], kernel=r["kernel"])))
PY
      tail -1 $O/g.jsonl
    done
  done
done
