#!/bin/bash
# GPU: GNN/learner tests, then bench.py three times (A/B against the last recorded headline)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_ops.py $R/tests/test_gpu_learner.py $R/tests/test_gpu_replay.py $R/tests/test_gpu_graphs.py $R/tests/test_gpu_sim.py -x -q --timeout 200 --timeout-method thread > $OUT/ab_tests.log 2>&1 &&
: > $OUT/ab.txt &&
timeout -k 10 120 python $R/scripts/gnn_bench.py >> $OUT/ab.txt 2>&1 &&
for i in 1 2 3; do
  timeout -k 10 200 python $R/bench.py --steps 40 --warmup 5 2>/dev/null | grep -o '"value": [0-9.]*' | sed "s/^/bench $i /" >> $OUT/ab.txt || exit 1
done
