#!/bin/bash
# 16-byte-load mask fold: tests, micro-benchmark (pair loop vs vectors, actor 256 rows / critic 64 rows), syn200 A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/rowdot
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "rowdot" -x -v --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1 || exit $?
: > $OUT/ab.txt
for v in 0 1; do
  for n in 256 64; do
    GSC_ROWDOT_VEC=$v timeout -k 10 120 python scripts/rowdot_bench.py --N $n >> $OUT/ab.txt 2>&1 || exit $?
  done
done
for i in ${ROUNDS:-1 2}; do
  for v in 0 1; do
    GSC_ROWDOT_VEC=$v timeout -k 10 400 python bench.py --preset syn200 --steps 30 --warmup 5 > $OUT/b.json 2> $OUT/b.err || exit $?
    echo "$i vec=$v syn200: $(grep -o '"value": [0-9.]*' $OUT/b.json)" >> $OUT/ab.txt
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_learner.py -x -v --timeout 300 --timeout-method thread > $OUT/tests_learner.txt 2>&1 || exit $?
cat $OUT/ab.txt
