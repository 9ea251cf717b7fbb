#!/bin/bash
# 64 B slots: next-range prefetch (libmicksum.so) vs none (libmicksum_nopf.so)
# at several grid caps; slot-kernel parity tests first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/slot64pf
mkdir -p $O
rm -f $O/pf.jsonl
L=$PWD/libunsod_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_aql_gpu.py -k "slot64 or full_size or every_plan" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for lib in libmicksum.so libmicksum_nopf.so; do
    for cap in 512 1024 2048; do
      line=$(MI_CKSUM_LIB=$L/$lib MI_CKSUM_MAX_BLOCKS=$cap timeout -k 10 150 python -u bench.py --config 64 --steps 20 --warmup 5 --no-dropin --no-host-path --cpu-seconds 0 2>> $O/pf.err) || exit 1
      python - "$lib" "$cap" "$line" >> $O/pf.jsonl <<'PY'
import json, sys
d = json.loads(sys.argv[3]); r = d["roofline"]
print(json.dumps(dict(lib=sys.argv[1], cap=int(sys.argv[2]), value=d["value"], avg_launch_us=r["avg_launch_us"], frac=r["frac"], wall_frac=r["wall_frac"])))
PY
      tail -1 $O/pf.jsonl
    done
  done
done
