#!/bin/bash
# per-graph d bias sums in the staged backward: in-tree (new) vs the ab/wt checkout of the commit before
# (old, its own Python + extension), syn200 bench interleaved x3
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/bias_ab.txt
for k in 1 2 3; do
  for v in new old; do
    D=$R; [ $v = old ] && D=$R/ab/wt
    (cd $D && timeout -k 10 400 python bench.py --preset syn200 --steps 30 --warmup 5 > $OUT/ba.json 2> $OUT/ba.err) || exit $?
    echo "$v $(grep -o '"value": [0-9.]*' $OUT/ba.json)" >> $OUT/bias_ab.txt
  done
done
