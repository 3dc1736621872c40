#!/bin/bash
# layer-wise GNN numerics + timing (fused pool backward, fused first conv with stores), learner tests, syn200 bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
VARIANTS="1:1" bash $R/scripts/gpurun/gnn200_ab.sh || exit $?
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_learner.py -x -v --timeout 120 --timeout-method thread > $OUT/learner.log 2>&1 || exit $?
echo "learner: $(tail -1 $OUT/learner.log)" >> $OUT/gnn200_ab.txt
timeout -k 10 400 python $R/bench.py --preset syn200 --steps 30 --warmup 5 > $OUT/bench_syn200.json 2> $OUT/bench_syn200.err || exit $?
echo "syn200: $(cut -c1-250 $OUT/bench_syn200.json)" >> $OUT/gnn200_ab.txt
