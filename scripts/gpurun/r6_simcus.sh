#!/bin/bash
# syn200 simulator CU partition sweep at HEAD (interleaved twice)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/simcus
mkdir -p $OUT
cd $R
: > $OUT/sweep.txt
for i in 1 2; do
  for c in ${CUS:-96 112 128 144}; do
    timeout -k 10 400 python bench.py --preset syn200 --sim-cus $c --steps 25 --warmup 5 > $OUT/b.json 2> $OUT/b.err || exit $?
    echo "$i sim_cus=$c $(grep -o '"value": [0-9.]*' $OUT/b.json)" >> $OUT/sweep.txt
  done
done
cat $OUT/sweep.txt
