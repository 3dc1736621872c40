#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_gnn_lw.py -x -v --timeout 200 --timeout-method thread > $OUT/lw_tests.log 2>&1 &&
timeout -k 10 300 python $R/bench.py --preset syn200 --steps 10 --warmup 3 > $OUT/bench_syn200.log 2>&1 &&
timeout -k 10 300 python $R/bench.py --preset syn50 --steps 10 --warmup 3 > $OUT/bench_syn50.log 2>&1
