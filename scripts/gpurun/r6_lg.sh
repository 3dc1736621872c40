#!/bin/bash
# large-graph fused GATv2 (gnn_lg.hip): numerics vs fp32, micro-benchmark vs the layer-wise kernels, config-5 bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/lg.txt
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_gnn_lg.py -x -v --timeout 120 --timeout-method thread > $OUT/lg_tests.log 2>&1 || { echo "lg tests failed" >> $OUT/lg.txt; exit 1; }
echo "lg tests: $(tail -1 $OUT/lg_tests.log)" >> $OUT/lg.txt
for lg in 1 0; do
  GSC_GNN_LG=$lg timeout -k 10 200 python $R/scripts/gnn_bench.py --network configs/networks/synthetic/syn200-in16-cap1-3-s0.graphml --n-pad 200 --batch 25600 --iters 5 > $OUT/gb.txt 2>&1 || exit $?
  echo "GSC_GNN_LG=$lg $(tail -1 $OUT/gb.txt)" >> $OUT/lg.txt
done
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_learner.py -k "200_nodes" $R/tests/test_gpu_gnn_lw.py -x -v --timeout 200 --timeout-method thread > $OUT/lg_tests2.log 2>&1 || { echo "learner/lw tests failed" >> $OUT/lg.txt; exit 1; }
echo "learner/lw tests: $(tail -1 $OUT/lg_tests2.log)" >> $OUT/lg.txt
timeout -k 10 400 python $R/bench.py --preset syn200 --steps 20 --warmup 5 > $OUT/bench_syn200_lg.json 2> $OUT/bench_syn200_lg.err || exit $?
echo "syn200: $(grep -o '"value": [0-9.]*' $OUT/bench_syn200_lg.json)" >> $OUT/lg.txt
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_handoff.py $R/tests/test_gpu_explore_pmask.py -x -v --timeout 200 --timeout-method thread > $OUT/lg_tests3.log 2>&1 || { echo "handoff/pmask tests failed" >> $OUT/lg.txt; exit 1; }
echo "handoff/pmask tests: $(tail -1 $OUT/lg_tests3.log)" >> $OUT/lg.txt
