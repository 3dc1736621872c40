#!/bin/bash
# bench A/B over an environment variable: VAR=<name> VALS="<v1> <v2> ..." (each value run twice, interleaved)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/envab.txt
for rep in 1 2; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 200 python $R/bench.py --steps 40 --warmup 5 $EXTRA 2>/dev/null | grep -o '"value": [0-9.]*' | sed "s/^/$VAR=$v /" >> $OUT/envab.txt || exit 1
  done
done
