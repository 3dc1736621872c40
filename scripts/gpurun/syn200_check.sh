#!/bin/bash
# Large-action (syn200, A = 360,000) learner checks: numerics of the native update (composed actor loss
# with per-topology masks, materialised path), the GEMM tile sweep at syn200 shapes, the syn200 bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread $R/tests/test_gpu_learner.py $R/tests/test_gpu_gnn_lw.py $R/tests/test_large_topologies.py \
  > $OUT/syn200_learner_tests.txt 2>&1 &&
timeout -k 10 300 python -u $R/scripts/gemm_tune.py syn200 > $OUT/gemm_tune_syn200.txt 2>&1 &&
timeout -k 10 400 python $R/bench.py --preset syn200 --steps 25 --warmup 5 > $OUT/bench_syn200.json 2> $OUT/bench_syn200.err
