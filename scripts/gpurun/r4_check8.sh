#!/bin/bash
# layer-wise GNN numerics + A/B, op / learner tests (actor_proj), actor_proj microbench vs the eaa3635 build,
# syn200 + abilene benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
VARIANTS="1:1 1:0" bash $R/scripts/gpurun/gnn200_ab.sh || exit $?
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_ops.py $R/tests/test_gpu_learner.py $R/tests/test_gpu_mlp.py -x -v --timeout 120 --timeout-method thread > $OUT/ops.log 2>&1 || exit $?
echo "ops: $(tail -1 $OUT/ops.log)" >> $OUT/gnn200_ab.txt
bash $R/scripts/gpurun/aproj_ab.sh || exit $?
cat $OUT/aproj_ab.txt >> $OUT/gnn200_ab.txt
for p in syn200 abilene; do
  timeout -k 10 400 python $R/bench.py --preset $p --steps 30 --warmup 5 > $OUT/bench_$p.json 2> $OUT/bench_$p.err || exit $?
  echo "$p: $(cut -c1-250 $OUT/bench_$p.json)" >> $OUT/gnn200_ab.txt
done
