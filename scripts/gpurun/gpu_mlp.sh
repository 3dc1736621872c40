#!/bin/bash
# MFMA GEMM engine: numerics tests + learner-shape timings
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_mlp.py -x -v --timeout 120 --timeout-method thread > $OUT/mlp_tests.log 2>&1 &&
timeout -k 10 200 python $R/scripts/mlp_bench.py > $OUT/mlp_bench.txt 2>&1
