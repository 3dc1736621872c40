#!/bin/bash
# learner kernel changes: GPU tests against fp32 references (ops, GEMMs, learner), then the presets
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_ops.py $R/tests/test_gpu_learner.py $R/tests/test_gpu_mlp.py -x -v --timeout 120 --timeout-method thread > $OUT/learn_tests.log 2>&1 &&
timeout -k 10 400 python $R/bench.py --preset syn200 --steps 25 --warmup 5 > $OUT/bench_syn200.json 2> $OUT/bench_syn200.err &&
timeout -k 10 300 python $R/bench.py --preset syn50 --steps 10 --warmup 3 > $OUT/bench_syn50.json 2> $OUT/bench_syn50.err &&
timeout -k 10 300 python $R/bench.py --steps 40 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
