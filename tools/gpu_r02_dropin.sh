#!/bin/bash
# (b1) drop-ins through the AQL one-shot dispatch (default) vs a HIP launch
# (MI_CKSUM_HOST_AQL=0): drop-in / C-caller / link-time tests, then the
# bench's per-call latency leg under both.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/dropin
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_c_example.py tests/test_link_gpu.py tests/test_host_gpu.py -k "dropin or c_example or link or host" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
fi
rm -f $O/lat.jsonl
for round in 1 2; do
  for aql in ${DROPIN_VARIANTS:-1 0}; do
    e="MI_CKSUM_HOST_AQL=1"; [ "$aql" = 0 ] && e="MI_CKSUM_HOST_AQL=0"; [ "$aql" = sys ] && e="MI_CKSUM_SCALAR_SYS=1"
    env $e timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-host-path > $O/b.json 2>> $O/b.err || exit 1
    python - "$aql" $O/b.json >> $O/lat.jsonl <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read())
print(json.dumps(dict(host_aql=sys.argv[1], value=d["value"], dropin=d.get("dropin_latency"))))
PY
    tail -1 $O/lat.jsonl | cut -c1-400
  done
done
