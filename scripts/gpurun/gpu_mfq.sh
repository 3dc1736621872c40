#!/bin/bash
# quick MFMA GNN check: numerics of the MFMA path + kernel timings (cl vs mf, mf phase profile)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest $R/tests/test_gpu_ops.py -x -v -k "mfma" --timeout 120 --timeout-method thread > $OUT/mf_tests.log 2>&1 &&
timeout -k 10 120 python $R/scripts/gnn_bench.py --path 59 --profile > $OUT/gnn_mf.txt 2>&1
