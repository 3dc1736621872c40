#!/bin/bash
# layer-wise GNN numerics + A/B (streamed conv grads, skipped stores), GEMM / actor_proj / GNN op tests,
# then the syn200 and syn50 preset benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
bash $R/scripts/gpurun/gnn200_ab.sh || exit $?
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_ops.py $R/tests/test_gpu_mlp.py -x -v --timeout 120 --timeout-method thread > $OUT/ops.log 2>&1 || exit $?
echo "ops: $(tail -1 $OUT/ops.log)" >> $OUT/gnn200_ab.txt
for p in syn200 syn50; do
  timeout -k 10 400 python $R/bench.py --preset $p --steps ${STEPS:-30} --warmup 5 > $OUT/bench_$p.json 2> $OUT/bench_$p.err || exit $?
  echo "$p: $(cut -c1-300 $OUT/bench_$p.json)" >> $OUT/gnn200_ab.txt
done
