#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/lw50.txt
for n in 32 1000; do
  GSC_GNN_LW_MIN_NODES=$n timeout -k 10 300 python $R/bench.py --preset syn50 --steps 10 --warmup 3 2>/dev/null | grep -o '"value": [0-9.]*' | sed "s/^/syn50 lw_min_nodes=$n /" >> $OUT/lw50.txt || exit 1
done
timeout -k 10 200 python -u -m pytest $R/tests/test_gpu_gnn_lw.py $R/tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread > $OUT/lw_tests.log 2>&1
