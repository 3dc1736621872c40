#!/bin/bash
# in-tree (new) vs the ab/wt checkout (old): GPU tests named by TESTS, then bench.py for each preset in
# PRESETS (default "syn50"), REPS interleaved pairs (default 3); results in gpurun_out/ab.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  cd $R && timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $TESTS > $OUT/ab_tests.txt 2>&1 || exit $?
fi
: > $OUT/ab.txt
for p in ${PRESETS:-syn50}; do
  for k in $(seq ${REPS:-3}); do
    for v in new old; do
      D=$R; [ $v = old ] && D=$R/ab/wt
      (cd $D && timeout -k 10 400 python bench.py --preset $p --steps ${STEPS:-40} --warmup 5 > $OUT/ab.json 2> $OUT/ab.err) || exit $?
      echo "$p $v $(grep -o '"value": [0-9.]*' $OUT/ab.json)" >> $OUT/ab.txt
    done
  done
done
