#!/bin/bash
# actor_proj split sweep at config-5 shapes (dispatch-round tail), SPLITS="8 16 32 ..."
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/aproj6
mkdir -p $OUT
cd $R
: > $OUT/sweep.txt
for S in ${SPLITS:-8 16 24 32 40}; do
  GSC_APROJ_SPLITS=$S timeout -k 10 120 python scripts/aproj_bench.py --slab-mb 512 --iters 10 >> $OUT/sweep.txt 2>&1 || exit $?
done
