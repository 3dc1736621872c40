#!/bin/bash
# MFMA GNN bring-up: numerics tests, kernel timings per path, then the headline bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_ops.py -x -v --timeout 120 --timeout-method thread > $OUT/mf_tests.log 2>&1 &&
timeout -k 10 120 python $R/scripts/gnn_bench.py --path 11 > $OUT/gnn_cl.txt 2>&1 &&
timeout -k 10 120 python $R/scripts/gnn_bench.py --path 59 --profile > $OUT/gnn_mf.txt 2>&1 &&
timeout -k 10 300 python $R/bench.py --steps 30 --warmup 5 > $OUT/bench.log 2>&1 &&
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
