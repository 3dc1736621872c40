#!/bin/bash
# sparse critic products (delta images + base column): numerics tests, standalone timing, syn200 bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/sparse6
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse_replay.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 120 python scripts/sparse_bench.py --B 25600 --R 1800 --P 200 --iters 10 > $OUT/bench.txt 2>&1 || exit $?
timeout -k 10 400 python bench.py --preset syn200 --steps 20 --warmup 5 > $OUT/syn200.json 2> $OUT/syn200.err || exit $?
