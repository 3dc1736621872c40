#!/bin/bash
# actor_proj numerics (tests/test_gpu_ops.py -k actor_proj) and the syn200 / abilene benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/aproj.txt
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_ops.py $R/tests/test_gpu_learner.py -x -v --timeout 120 --timeout-method thread > $OUT/aproj_tests.log 2>&1 || exit $?
echo "tests: $(tail -1 $OUT/aproj_tests.log)" >> $OUT/aproj.txt
for p in syn200 abilene; do
  timeout -k 10 400 python $R/bench.py --preset $p --steps 30 --warmup 5 > $OUT/bench_$p.json 2> $OUT/bench_$p.err || exit $?
  echo "$p: $(cut -c1-250 $OUT/bench_$p.json)" >> $OUT/aproj.txt
done
