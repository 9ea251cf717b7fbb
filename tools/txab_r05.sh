set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05txab; mkdir -p $O
for r in 0 1; do
 for lay in socket single; do
  timeout -k 10 200 python -u tools/bench_tx.py --layout $lay --check --cpu-seconds 0 > $O/early_${lay}_$r.json 2>>$O/err.log || exit 11
  MI_CKSUM_LIB=tools/ab/libmicksum_txlate.so timeout -k 10 200 python -u tools/bench_tx.py --layout $lay --check --cpu-seconds 0 > $O/late_${lay}_$r.json 2>>$O/err.log || exit 12
 done
done
echo done
