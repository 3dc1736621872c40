#!/bin/bash
# syn50 CU partition sweep (simulator CUs x learner mask): bench JSON lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/syn50_partition.txt
for cfg in "-1 auto" "64 1" "64 0" "96 1" "32 1"; do
  set -- $cfg
  GSC_LEARNER_MASK=$2 timeout -k 10 300 python $R/bench.py --preset syn50 --steps 8 --warmup 3 --sim-cus $1 > $OUT/p.json 2> $OUT/p.err || exit $?
  echo "sim_cus=$1 learner_mask=$2 $(cat $OUT/p.json)" >> $OUT/syn50_partition.txt
done
