# Three driver-equivalent bench runs with the repeat handle's host trace.
cd $GRAFT_REPO_ROOT
rm -f gpurun_out/bench_trace.jsonl
for k in 1 2 3; do
  MI_CKSUM_REPEAT_TRACE=1 timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-dropin --no-host-path --cpu-seconds 0 $BENCH_ARGS >> gpurun_out/bench_trace.jsonl || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/bench_trace.jsonl"):
    d = json.loads(l)
    print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_us"], d.get("host_trace_us"), d["warm_region_walls_us"])
PY
