#!/bin/bash
# bench A/B over bench.py argument sets: ARGS="--sim-cus 96|--sim-cus 128" (|-separated, each run twice, interleaved)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/argab.txt
IFS='|' read -ra SETS <<< "$ARGS"
for rep in 1 2; do
  for a in "${SETS[@]}"; do
    timeout -k 10 200 python $R/bench.py --steps 40 --warmup 5 $a 2>/dev/null | grep -o '"value": [0-9.]*' | sed "s/^/[$a] /" >> $OUT/argab.txt || exit 1
  done
done
