#!/bin/bash
# fused TD-target projection: GPU tests vs fp32, learner tests, syn50 / headline benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_ops.py $R/tests/test_gpu_learner.py -x -v -k "actor_proj or native_update" --timeout 120 --timeout-method thread > $OUT/aproj_tests.log 2>&1 &&
timeout -k 10 300 python $R/bench.py --preset syn50 --steps 10 --warmup 3 > $OUT/bench_syn50.json 2> $OUT/bench_syn50.err &&
timeout -k 10 300 python $R/bench.py --steps 40 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
