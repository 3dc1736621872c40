#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/ab_repeat.txt
for i in 1 2 3; do
  timeout -k 10 300 python $R/bench.py --steps 40 --warmup 5 > $OUT/p.json 2> $OUT/p.err || exit $?
  cat $OUT/p.json >> $OUT/ab_repeat.txt
done
bash $R/scripts/gpurun/syn50_partition.sh
