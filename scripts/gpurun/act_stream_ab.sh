#!/bin/bash
# headline: act path on the simulator's CUs (default) vs an unmasked stream (GSC_ACT_STREAM=1), interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/act_stream_ab.txt
for k in 1 2 3; do
  for v in 0 1; do
    GSC_ACT_STREAM=$v timeout -k 10 300 python $R/bench.py --steps 60 --warmup 5 > $OUT/as.json 2> $OUT/as.err || exit $?
    echo "act_stream=$v $(grep -o '"value": [0-9.]*' $OUT/as.json)" >> $OUT/act_stream_ab.txt
  done
done
