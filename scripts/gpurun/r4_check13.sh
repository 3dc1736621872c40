#!/bin/bash
# whole-embedding fused forward (numerics + timing + syn200 bench), then the GNN input staging A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
VARIANTS="1:1" bash $R/scripts/gpurun/gnn200_ab.sh || exit $?
timeout -k 10 400 python $R/bench.py --preset syn200 --steps 30 --warmup 5 > $OUT/bench_syn200.json 2> $OUT/bench_syn200.err || exit $?
echo "syn200: $(grep -o '"value": [0-9.]*' $OUT/bench_syn200.json)" >> $OUT/gnn200_ab.txt
GSC_LW_EMBED=0 timeout -k 10 400 python $R/bench.py --preset syn200 --steps 30 --warmup 5 > $OUT/bench_syn200_0.json 2> $OUT/bench_syn200_0.err || exit $?
echo "syn200 GSC_LW_EMBED=0: $(grep -o '"value": [0-9.]*' $OUT/bench_syn200_0.json)" >> $OUT/gnn200_ab.txt
bash $R/scripts/gpurun/stage_ab.sh
