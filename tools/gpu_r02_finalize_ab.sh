# In-place finalize vs the in-place write probe, same box, same process order;
# default byte stores vs nontemporal ones (MI_TX_STORE_EXP=2 build in tools/ab/).
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/ceiling_writes.py > gpurun_out/ceiling_writes_nt.jsonl || exit 1
timeout -k 10 300 python tools/bench_finalize.py --configs 1500,pareto --rounds 1 --steps 200 > gpurun_out/fin_default.jsonl || exit 1
MI_CKSUM_LIB=$PWD/tools/ab/libmicksum_nt.so timeout -k 10 300 python tools/bench_finalize.py --configs 1500,pareto --rounds 1 --steps 200 > gpurun_out/fin_nt.jsonl || exit 1
cut -c1-200 gpurun_out/ceiling_writes_nt.jsonl gpurun_out/fin_default.jsonl gpurun_out/fin_nt.jsonl
