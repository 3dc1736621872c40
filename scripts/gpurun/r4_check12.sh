#!/bin/bash
# batched GNN input staging (gnn_mf / gnn_mt): GNN op tests, then abilene x2 and syn50 benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/r4c12.txt
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_ops.py $R/tests/test_gpu_learner.py -x -v --timeout 120 --timeout-method thread > $OUT/ops.log 2>&1 || exit $?
echo "tests: $(tail -1 $OUT/ops.log)" >> $OUT/r4c12.txt
for p in abilene syn50 abilene; do
  timeout -k 10 400 python $R/bench.py --preset $p --steps 40 --warmup 5 > $OUT/bench_$p.json 2> $OUT/bench_$p.err || exit $?
  echo "$p: $(grep -o '"value": [0-9.]*' $OUT/bench_$p.json)" >> $OUT/r4c12.txt
done
timeout -k 10 300 python $R/scripts/gnn_bench.py --iters 10 > $OUT/gnn_abilene.txt 2>&1 || exit $?
grep -v amdgpu.ids $OUT/gnn_abilene.txt | head -3 >> $OUT/r4c12.txt
