#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/aproj6
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_learner.py -x -v --timeout 200 --timeout-method thread -k "aproj or actor_proj or learner" > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 120 python scripts/aproj_bench.py --slab-mb 256 --iters 10 > $OUT/default.txt 2>&1 || exit $?
timeout -k 10 400 python bench.py --preset syn200 --steps 20 --warmup 5 > $OUT/syn200.json 2> $OUT/syn200.err || exit $?
timeout -k 10 400 python bench.py --preset syn50 --steps 20 --warmup 5 > $OUT/syn50.json 2> $OUT/syn50.err || exit $?
