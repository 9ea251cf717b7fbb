cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
CPU_SECONDS=2 bash tools/gpu_bench_all.sh || exit 1
python - <<'PY'
import json
for l in open("gpurun_out/bench_all.jsonl"):
    d=json.loads(l); print(d["config"]["workload"][:50], d["value"], d["roofline"]["frac"], d["ms_per_step"])
PY
