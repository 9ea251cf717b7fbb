#!/bin/bash
# Rehearse bench.py's N>1 path on a one-GPU box: 2 ranks on device 0, gloo for
# the barrier / max-over-ranks (RCCL refuses two ranks on one GPU).  The
# driver's real multi-GPU runs use LOCAL_RANK devices and RCCL.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for np in ${NPROCS:-2}; do
for cfg in ${CONFIGS:-1500 pareto}; do
  MI_BENCH_DEVICE=0 MI_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $np --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $np --config $cfg \
    --steps ${STEPS:-200} --warmup 20 > gpurun_out/dist${np}_$cfg.json 2> gpurun_out/dist${np}_$cfg.err || exit $?
  cut -c1-400 gpurun_out/dist${np}_$cfg.json
done
done
echo "exit 0"
