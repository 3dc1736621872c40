#!/bin/bash
# GNN kernels: numerics tests vs fp32 (one-tile, two-tile, layer-wise) and the micro-benchmark at
# Abilene (11 nodes, n_pad 24) and syn50 (50 nodes, n_pad 50), B = 25,600
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_ops.py $R/tests/test_gpu_gnn_lw.py -x -v --timeout 120 --timeout-method thread > $OUT/gnn_tests.log 2>&1 &&
timeout -k 10 120 python $R/scripts/gnn_bench.py > $OUT/gnn_bench.txt 2>&1 &&
timeout -k 10 120 python $R/scripts/gnn_bench.py --network configs/networks/synthetic/syn50-in8-cap1-3.graphml --n-pad 50 >> $OUT/gnn_bench.txt 2>&1
