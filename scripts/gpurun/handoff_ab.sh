#!/bin/bash
# act <-> simulator hand-off: sequence words (GSC_STREAM_VALUES=1, default) vs events, the equivalence test, then
# the headline bench interleaved (two rounds each)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/handoff
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_handoff.py -x -v --timeout 240 --timeout-method thread > $OUT/tests.txt 2>&1 || exit $?
: > $OUT/ab.txt
for r in 1 2; do
  for v in 1 0; do
    GSC_STREAM_VALUES=$v timeout -k 10 300 python $R/bench.py --steps 40 --warmup 5 ${BENCH_ARGS:-} > $OUT/b_$v.json 2> $OUT/b_$v.err || exit $?
    echo "values=$v $(grep -o '"value": [0-9.]*' $OUT/b_$v.json) $(grep -o '"ms_per_step": [0-9.]*' $OUT/b_$v.json)" >> $OUT/ab.txt
  done
done
