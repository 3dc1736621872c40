#!/bin/bash
# packed large-graph GATv2 kernels for 33..64-node graphs: numerics, micro-benchmark and syn50 bench, pack vs mt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pack6
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_gnn_lg.py tests/test_gpu_ops.py -x -v --timeout 200 --timeout-method thread -k "gnn or lg" > $OUT/tests.log 2>&1 || exit $?
for p in 1 0; do
  GSC_GNN_LG_PACK=$p timeout -k 10 200 python scripts/gnn_bench.py --network configs/networks/synthetic/syn50-in8-cap1-3.graphml --n-pad 50 --batch 25600 --iters 5 > $OUT/gb_$p.txt 2>&1 || exit $?
done
[ -n "$BENCH" ] || exit 0
for p in 1 0; do
  GSC_GNN_LG_PACK=$p timeout -k 10 400 python bench.py --preset syn50 --steps 20 --warmup 5 > $OUT/syn50_$p.json 2> $OUT/syn50_$p.err || exit $?
done
