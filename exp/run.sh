cd $GRAFT_REPO_ROOT
for v in base NOCREDIT NOBOUND; do
  if [ $v = base ]; then L=""; else L=$PWD/exp/lib_$v.so; fi
  MI_CKSUM_LIB=$L timeout -k 10 200 python tools/pareto_grid.py > gpurun_out/exp_$v.jsonl 2>gpurun_out/exp_$v.err || exit 1
done
echo done
