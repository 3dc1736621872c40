#!/bin/bash
# gnn_mt A/B: in-tree (new) vs the ab/wt checkout (old): 50-node GPU tests, then syn50 bench x3 interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R && timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py > $OUT/mt_tests.txt 2>&1 || exit $?
: > $OUT/mt_ab.txt
for k in 1 2 3; do
  for v in new old; do
    D=$R; [ $v = old ] && D=$R/ab/wt
    (cd $D && timeout -k 10 400 python bench.py --preset syn50 --steps 40 --warmup 5 > $OUT/ma.json 2> $OUT/ma.err) || exit $?
    echo "$v $(grep -o '"value": [0-9.]*' $OUT/ma.json)" >> $OUT/mt_ab.txt
  done
done
