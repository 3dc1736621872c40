#!/bin/bash
# persistent work-stealing actor_proj: numerics tests, standalone time at config-5 shapes, syn200 + headline benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/apq
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -k "actor_proj or explore" tests/test_gpu_learner.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.txt 2>&1 || exit $?
timeout -k 10 120 python scripts/aproj_bench.py --slab-mb 512 --iters 10 > $OUT/aproj.txt 2>&1 || exit $?
: > $OUT/bench.txt
for i in 1 2; do
  for P in syn200 abilene; do
    timeout -k 10 400 python bench.py --preset $P --steps 20 --warmup 5 > $OUT/b.json 2> $OUT/b.err || exit $?
    echo "$P: $(grep -o '"value": [0-9.]*' $OUT/b.json)" >> $OUT/bench.txt
  done
done
cat $OUT/bench.txt
