#!/bin/bash
# same-box A/B of the syn200 bench: HEAD vs the gnn_lg / gnn.hip of another commit (scripts/lg_variant_ab.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/lgab
mkdir -p $OUT
cd $R
V=$(ls $R/ab/lgvar/${REV}/_native*.so)
: > $OUT/ab.txt
for round in 1 2; do
  timeout -k 10 300 python bench.py --preset syn200 --steps 20 --warmup 5 > $OUT/head_$round.json 2>/dev/null || exit $?
  GSC_NATIVE_SO=$V timeout -k 10 300 python bench.py --preset syn200 --steps 20 --warmup 5 > $OUT/var_$round.json 2>/dev/null || exit $?
  echo "round $round head $(grep -o '"value": [0-9.]*' $OUT/head_$round.json) var $(grep -o '"value": [0-9.]*' $OUT/var_$round.json)" >> $OUT/ab.txt
done
