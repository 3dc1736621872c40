#!/bin/bash
# actor_proj Wa row stride 68 (this tree) vs 72 (ab/aphead): numerics tests, standalone time, syn200 bench, interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/apldp
SO=gsc_amd/_native.cpython-310-x86_64-linux-gnu.so
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "actor_proj" -x -v --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1 || exit $?
cp $SO /tmp/new.so || exit 1
: > $OUT/ab.txt
for i in 1 2; do
  for v in head new; do
    if [ $v = head ]; then cp ab/aphead/$SO $SO; else cp /tmp/new.so $SO; fi || exit 1
    echo "$i $v $(timeout -k 10 120 python scripts/aproj_bench.py --slab-mb 512 --iters 10 2>&1 | grep actor_proj)" >> $OUT/ab.txt || exit 1
    timeout -k 10 400 python bench.py --preset syn200 --steps 30 --warmup 5 > $OUT/b.json 2> $OUT/b.err || exit $?
    echo "$i $v syn200: $(grep -o '"value": [0-9.]*' $OUT/b.json)" >> $OUT/ab.txt
  done
done
cp /tmp/new.so $SO
cat $OUT/ab.txt
