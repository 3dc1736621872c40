#!/bin/bash
# the same tree with the environment assignment in ENVA (e.g. "GSC_ACT_STREAM=1") vs without, bench.py for each
# preset in PRESETS, REPS interleaved pairs; results in gpurun_out/ab_env.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/ab_env.txt
cd $R
for p in ${PRESETS:-syn50}; do
  for k in $(seq ${REPS:-2}); do
    for v in on off; do
      if [ $v = on ]; then
        env $ENVA timeout -k 10 400 python bench.py --preset $p --steps ${STEPS:-40} --warmup 5 > $OUT/abe.json 2> $OUT/abe.err || exit $?
      else
        timeout -k 10 400 python bench.py --preset $p --steps ${STEPS:-40} --warmup 5 > $OUT/abe.json 2> $OUT/abe.err || exit $?
      fi
      echo "$p $v $(grep -o '"value": [0-9.]*' $OUT/abe.json)" >> $OUT/ab_env.txt
    done
  done
done
