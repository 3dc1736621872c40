#!/bin/bash
# headline simulator CU share sweep at HEAD (per-XCD spread mask), interleaved twice
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/simcus_ab
mkdir -p $OUT
cd $R
: > $OUT/sweep.txt
for i in 1 2; do
  for c in ${CUS:-64 72 80 96}; do
    timeout -k 10 300 python bench.py --sim-cus $c --steps 40 --warmup 5 > $OUT/b.json 2> $OUT/b.err || exit $?
    echo "$i sim_cus=$c $(grep -o '"value": [0-9.]*' $OUT/b.json)" >> $OUT/sweep.txt
  done
done
cat $OUT/sweep.txt
