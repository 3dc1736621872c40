#!/bin/bash
# copy2d row grid: bitwise test, syn200 A/B (GSC_COPY2D_ROWS=0 vs default); then the round evidence (GPU suite, smoke,
# presets, syn200 profile last)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/c2d
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "copy2d" -x -v --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1 || exit $?
: > $OUT/ab.txt
for i in 1 2; do
  for v in 0 1; do
    GSC_COPY2D_ROWS=$v timeout -k 10 400 python bench.py --preset syn200 --steps 30 --warmup 5 > $OUT/b.json 2> $OUT/b.err || exit $?
    echo "$i rows=$v syn200: $(grep -o '"value": [0-9.]*' $OUT/b.json)" >> $OUT/ab.txt
  done
done
bash $R/scripts/gpurun/evidence.sh tests syn200
