#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/exp_save.txt
for v in 1 0 1 0; do
  GSC_GNN_SAVE=$v timeout -k 10 200 python $R/bench.py --steps 40 --warmup 5 2>/dev/null | grep -o '"value": [0-9.]*' | sed "s/^/gnn_save=$v /" >> $OUT/exp_save.txt || exit 1
done
