cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "pareto or packed or full_size or rx_offload" > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for v in base LB6 LB8; do
  if [ $v = base ]; then L=""; else L=$PWD/exp/lib_$v.so; fi
  MI_CKSUM_LIB=$L timeout -k 10 200 python tools/pareto_grid.py > gpurun_out/exp_$v.jsonl 2>gpurun_out/exp_$v.err || exit 1
  echo $v; grep '"round": 1' gpurun_out/exp_$v.jsonl | head -3
  for c in 64 pareto; do
    MI_CKSUM_LIB=$L timeout -k 10 200 python bench.py --config $c --cpu-seconds 0 --no-host-path > gpurun_out/exp_${v}_$c.json 2>>gpurun_out/exp_$v.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/exp_${v}_$c.json'));print('$c',d['value'],d['roofline']['frac'])"
  done
done
