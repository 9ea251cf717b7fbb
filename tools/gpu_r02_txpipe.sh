#!/bin/bash
# TX copy: pass-pipelined kernel (MI_TX_PIPE=1, libmicksum.so) vs one pass at
# a time (libmicksum_txnopipe.so): TX parity tests on the new build, then
# bench_tx on both layouts, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/txpipe
mkdir -p $O
rm -f $O/tx.jsonl
L=$PWD/libunsod_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_tx_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for lib in libmicksum.so libmicksum_txnopipe.so; do
    for lay in socket single; do
      MI_CKSUM_LIB=$L/$lib timeout -k 10 200 python -u tools/bench_tx.py --layout $lay --cpu-seconds 0 --check 2>> $O/tx.err | sed "s/}$/, \"lib\": \"$lib\"}/" >> $O/tx.jsonl || exit 1
      tail -1 $O/tx.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['lib'], d['layout'], d['us_per_launch'], d['roofline']['frac'], d.get('check'))"
    done
  done
done
