#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/b200.txt
for P in ${PRESETS:-syn200}; do
  timeout -k 10 400 python $R/bench.py --preset $P --steps 20 --warmup 5 > $OUT/bench_$P.json 2> $OUT/bench_$P.err || exit $?
  echo "$P: $(grep -o '"value": [0-9.]*' $OUT/bench_$P.json)" >> $OUT/b200.txt
done
