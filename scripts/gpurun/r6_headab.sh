#!/bin/bash
# same-box A/B of the tree against ab/head (the extension + exploration wrapper of the last commit): headline and
# syn200 benches, interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/hab
SO=gsc_amd/_native.cpython-310-x86_64-linux-gnu.so
PY=gsc_amd/ops/explore.py
mkdir -p $OUT
cd $R
cp $SO /tmp/new.so && cp $PY /tmp/new_explore.py || exit 1
: > $OUT/ab.txt
for i in 1 2 3; do
  for v in head new; do
    if [ $v = head ]; then cp ab/head/$SO $SO && cp ab/head/$PY $PY; else cp /tmp/new.so $SO && cp /tmp/new_explore.py $PY; fi || exit 1
    for P in ${PRESETS:-abilene}; do
      timeout -k 10 400 python bench.py --preset $P --steps 30 --warmup 5 > $OUT/b.json 2> $OUT/b.err || exit $?
      echo "$i $v $P: $(grep -o '"value": [0-9.]*' $OUT/b.json)" >> $OUT/ab.txt
    done
  done
done
cp /tmp/new.so $SO && cp /tmp/new_explore.py $PY
cat $OUT/ab.txt
