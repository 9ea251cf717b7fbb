#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
rm -f gpurun_out/txc.jsonl
L=$PWD/libunsod_amd/lib
for i in 1 2; do
for lib in libmicksum_txhead.so libmicksum.so libmicksum_txlb4.so; do
  for lay in socket single; do
    MI_CKSUM_LIB=$L/$lib timeout -k 10 200 python -u tools/bench_tx.py --layout $lay --cpu-seconds 0 --check | sed "s/}$/, \"lib\": \"$lib\"}/" >> gpurun_out/txc.jsonl
  done
done
done
echo done
