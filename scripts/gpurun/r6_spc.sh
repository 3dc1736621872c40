#!/bin/bash
# 16-byte-load sparse compress: record equality + sparse replay tests, then the syn200 A/B (GSC_SP_COMPRESS4=0 vs default)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/spc
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_sparse_replay.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1 || exit $?
: > $OUT/ab.txt
for i in 1 2; do
  for v in 0 1; do
    GSC_SP_COMPRESS4=$v timeout -k 10 400 python bench.py --preset syn200 --steps 30 --warmup 5 > $OUT/b.json 2> $OUT/b.err || exit $?
    echo "$i c4=$v syn200: $(grep -o '"value": [0-9.]*' $OUT/b.json)" >> $OUT/ab.txt
  done
done
cat $OUT/ab.txt
