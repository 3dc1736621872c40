#!/bin/bash
# GNN backward register budget A/B (1 vs 2 waves per SIMD) + GPU op tests + bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread > $OUT/gnn_tests.log 2>&1 &&
for w in 1 2; do
  GSC_GNN_BWD_WPE=$w timeout -k 10 120 python $R/scripts/gnn_bench.py 2>&1 | grep -v amdgpu | sed "s/^/wpe=$w /" >> $OUT/gnn_ab.txt || exit 1
done
for w in 1 2; do
  GSC_GNN_BWD_WPE=$w timeout -k 10 120 python $R/bench.py --steps 30 --warmup 5 2>/dev/null | grep -o '"value": [0-9.]*' | sed "s/^/bench wpe=$w /" >> $OUT/gnn_ab.txt || exit 1
done
