#!/bin/bash
# A/B of an environment switch on the headline bench: alternating runs, 20 timed steps each
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/ab.txt
for i in 1 2 3; do
  for v in $AB_VALUES; do
    env $AB_VAR=$v timeout -k 10 120 python $R/bench.py --steps 30 --warmup 5 $EXTRA 2>/dev/null | grep -o '"value": [0-9.]*' | sed "s/^/$AB_VAR=$v /" >> $OUT/ab.txt || exit 1
  done
done
