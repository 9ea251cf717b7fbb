#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
rm -f gpurun_out/db6.jsonl
L=$PWD/libunsod_amd/lib
for i in 1 2; do
for lib in libmicksum.so libmicksum_db6.so; do
  MI_CKSUM_LIB=$L/$lib timeout -k 10 200 python -u tools/grid_iso.py --config 1500 --caps 2048 | sed "s/}$/, \"lib\": \"$lib\"}/" >> gpurun_out/db6.jsonl
  MI_CKSUM_LIB=$L/$lib timeout -k 10 200 python -u tools/bench_multi.py --config 1500 --ms 1,4 | sed "s/}$/, \"lib\": \"$lib\"}/" >> gpurun_out/db6.jsonl
done
done
echo done
