#!/bin/bash
# fused first conv (numerics + timing), the GEMM engine tiles at the config-5 learner shapes, syn200 bench with /
# without the large-A tile overrides
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
VARIANTS="1:1" bash $R/scripts/gpurun/gnn200_ab.sh || exit $?
timeout -k 10 600 python $R/scripts/gemm_tune.py syn200 25600 > $OUT/gemm_tune_syn200.txt 2>&1 || exit $?
: > $OUT/tiles_ab.txt
for v in 1 0; do
  GSC_LARGE_A_TILES=$v timeout -k 10 400 python $R/bench.py --preset syn200 --steps 30 --warmup 5 > $OUT/bench_syn200_t$v.json 2> $OUT/bench_syn200_t$v.err || exit $?
  echo "tiles=$v: $(cut -c1-250 $OUT/bench_syn200_t$v.json)" >> $OUT/tiles_ab.txt
done
