#!/bin/bash
# round-4 GPU step: N=2 bench rehearsal (gloo, one device); Pareto flat-run
# LDS capture off / 5 waves per SIMD A/B (HIP launches)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04l; mkdir -p $O
MI_BENCH_DEVICE=0 MI_BENCH_BACKEND=gloo timeout -k 10 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_n2_rehearsal.json 2> $O/bench_n2.err || { tail -20 $O/bench_n2.err; exit 1; }
grep '^{"metric' $O/bench_n2_rehearsal.json | cut -c1-300
timeout -k 10 600 python -u tools/ab.py --config pareto --rounds 2 --steps 200 --submit launch base: cap0:tools/ab/libmicksum_cap0.so cap0w5:tools/ab/libmicksum_cap0w5.so > $O/ab_pareto_capture.jsonl 2> $O/ab.err || { tail $O/ab.err; exit 1; }
cut -c1-140 $O/ab_pareto_capture.jsonl
echo done
