#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_ops.py $R/tests/test_gpu_learner.py -x -q --timeout 200 --timeout-method thread > $OUT/pack_tests.log 2>&1 &&
: > $OUT/pack_ab.txt &&
for v in 1 0; do
  GSC_GNN_PACK=$v timeout -k 10 120 python $R/scripts/gnn_bench.py 2>&1 | grep -v amdgpu | sed "s/^/pack=$v /" >> $OUT/pack_ab.txt || exit 1
done
for v in 1 0 1; do
  GSC_GNN_PACK=$v timeout -k 10 200 python $R/bench.py --steps 40 --warmup 5 2>/dev/null | grep -o '"value": [0-9.]*' | sed "s/^/bench pack=$v /" >> $OUT/pack_ab.txt || exit 1
done
