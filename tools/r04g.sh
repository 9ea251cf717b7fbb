#!/bin/bash
# round-4 GPU step: Pareto flat-run U x waves; single-launch shapes; TX 5-wave
# spill-free variant
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 600 python -u tools/ab.py --config pareto --rounds 2 --steps 200 w2u8: w2u4::MI_CKSUM_PACKED_U=4 w1u4::MI_CKSUM_PACKED_U=4,MI_CKSUM_RUN_WAVES=1 w4u4::MI_CKSUM_PACKED_U=4,MI_CKSUM_RUN_WAVES=4 > $O/ab_pareto_u.jsonl 2> $O/ab.err || { tail $O/ab.err; exit 1; }
cut -c1-160 $O/ab_pareto_u.jsonl
for sh in 32x3 64x2 16x6; do
  timeout -k 10 240 python -u tools/grid_iso.py --config 1500 --shape $sh --caps 1280,2560,5120 >> $O/grid_iso_shapes.jsonl 2>> $O/grid_iso.err || { tail $O/grid_iso.err; exit 1; }
done
cut -c1-250 $O/grid_iso_shapes.jsonl
echo done
