#!/bin/bash
# A/B: bench.py under env settings A and B, interleaved twice (usage: A="X=1" B="Y=1" ab.sh [bench args])
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/ab.txt
for i in 1 2; do
  for v in A B; do
    env ${!v} timeout -k 10 300 python $R/bench.py "$@" 2>/dev/null | grep -o '"value": [0-9.]*' | sed "s/^/$v(${!v}) /" >> $OUT/ab.txt || exit 1
  done
done
