#!/bin/bash
# config 5 (learner-bound): simulator partition size x learner CU mask
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/syn200_partition.txt
for v in "64 1" "64 0" "32 1" "32 0" "96 0"; do
  set -- $v
  GSC_LEARNER_MASK=$2 timeout -k 10 400 python $R/bench.py --preset syn200 --steps 30 --warmup 5 --sim-cus $1 > $OUT/sp.json 2> $OUT/sp.err || exit $?
  echo "sim_cus=$1 learner_mask=$2 $(grep -o '"value": [0-9.]*' $OUT/sp.json)" >> $OUT/syn200_partition.txt
done
