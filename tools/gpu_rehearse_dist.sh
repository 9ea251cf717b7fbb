#!/bin/bash
# Rehearse bench.py's N>1 path on a one-GPU box: 2 ranks on device 0, gloo for
# the barrier / max-over-ranks (RCCL refuses two ranks on one GPU).  The
# driver's real multi-GPU runs use LOCAL_RANK devices and RCCL.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in 1500 pareto; do
  MI_BENCH_DEVICE=0 MI_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --config $cfg \
    --steps 200 --warmup 20 > gpurun_out/dist2_$cfg.json 2> gpurun_out/dist2_$cfg.err || exit $?
done
echo "exit 0"
