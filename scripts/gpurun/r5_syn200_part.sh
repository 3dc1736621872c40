#!/bin/bash
# config-5 simulator / learner CU partition sweep (bench.py --sim-cus)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/part200
mkdir -p $OUT
: > $OUT/sweep.txt
for c in ${CUS:-64 96 128}; do
  timeout -k 10 300 python3 $R/bench.py --preset ${PRESET:-syn200} --steps 25 --warmup 5 --sim-cus $c > $OUT/b_$c.json 2> $OUT/b_$c.err || exit 1
  echo "sim_cus=$c $(grep -o '"value": [0-9.]*' $OUT/b_$c.json) $(grep -o '"ms_per_step": [0-9.]*' $OUT/b_$c.json)" >> $OUT/sweep.txt
done
