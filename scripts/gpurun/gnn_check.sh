#!/bin/bash
# GATv2 kernel changes: GPU op tests against fp32, learner tests, the GNN micro-benchmark, syn50 bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_ops.py $R/tests/test_gpu_learner.py -x -v --timeout 120 --timeout-method thread > $OUT/gnn_tests.log 2>&1 &&
timeout -k 10 120 python $R/scripts/gnn_bench.py > $OUT/gb.txt 2>&1 &&
timeout -k 10 300 python $R/bench.py --preset syn50 --steps 10 --warmup 3 > $OUT/bench_syn50.json 2> $OUT/bench_syn50.err
