#!/bin/bash
# headline bench over different timed windows: within one episode (190 steps) vs across the boundary
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/bench_windows.txt
for sw in "190 5" "40 150" "201 5"; do
  set -- $sw
  timeout -k 10 300 python $R/bench.py --steps $1 --warmup $2 > $OUT/p.json 2> $OUT/p.err || exit $?
  echo "steps=$1 warmup=$2 $(cat $OUT/p.json)" >> $OUT/bench_windows.txt
done
