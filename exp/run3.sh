cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for u in 4 8 16; do
  MI_CKSUM_PACKED_U=$u timeout -k 10 200 python tools/pareto_grid.py > gpurun_out/v4_u$u.jsonl 2>gpurun_out/v4_u$u.err || exit 1
  grep '"round": 1' gpurun_out/v4_u$u.jsonl
done
