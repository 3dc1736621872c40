#!/bin/bash
# sweep: learner CU mask on/off x simulator CU count (headline bench, short runs)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/sweep2.txt
for cfg in ${CFGS:-"0 80" "0 96" "0 112" "0 128" "0 160"}; do
  set -- $cfg
  echo "mask=$1 simcus=$2" >> $OUT/sweep2.txt
  GSC_LEARNER_MASK=$1 timeout -k 10 120 python $R/bench.py --steps 30 --warmup 5 --sim-cus $2 2>/dev/null | grep -o '"value": [0-9.]*' >> $OUT/sweep2.txt || exit 1
done
