#!/bin/bash
# ab/head vs this tree: exploration kernel at Abilene shapes (n_pad 24, 1 SFC x 3 SFs) and the headline bench over seeds
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/seed
SO=gsc_amd/_native.cpython-310-x86_64-linux-gnu.so
PY=gsc_amd/ops/explore.py
mkdir -p $OUT
cd $R
cp $SO /tmp/new.so && cp $PY /tmp/new_explore.py || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k explore tests/test_gpu_explore_pmask.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1 || exit $?
: > $OUT/ab.txt
for v in head new; do
  if [ $v = head ]; then cp ab/head/$SO $SO && cp ab/head/$PY $PY; else cp /tmp/new.so $SO && cp /tmp/new_explore.py $PY; fi || exit 1
  timeout -k 10 120 python scripts/explore_bench.py --n-pad 24 --C 1 --F 3 > $OUT/ex_$v.txt 2>&1 || exit $?
  echo "$v $(grep explore $OUT/ex_$v.txt | tr '\n' ' ')" >> $OUT/ab.txt
  for s in 0 1 2; do
    timeout -k 10 300 python bench.py --steps 30 --warmup 5 --seed $s > $OUT/b.json 2> $OUT/b.err || exit $?
    echo "$v seed $s: $(grep -o '"value": [0-9.]*' $OUT/b.json) $(grep -o '"success_ratio": [0-9.]*' $OUT/b.json)" >> $OUT/ab.txt
  done
done
cp /tmp/new.so $SO && cp /tmp/new_explore.py $PY
cat $OUT/ab.txt
