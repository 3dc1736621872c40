#!/bin/bash
# component timing of the headline step: full / no learner (act + sim chain) / GNN state save off
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/diag.txt
for i in 1 2; do
for v in "X=0" "GSC_DIAG_NO_LEARN=1" "GSC_GNN_SAVE=0"; do
  env $v timeout -k 10 120 python $R/bench.py --steps 30 --warmup 5 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | sed "s/^/$v /" >> $OUT/diag.txt || exit 1
done
done
