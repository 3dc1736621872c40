#!/bin/bash
# split-K block target A/B (GSC_SPLITK_BLOCKS 512 = default vs 1024 / 2048), interleaved, syn200 and the headline
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/splitk
mkdir -p $OUT
cd $R
: > $OUT/ab.txt
for i in 1 2; do
  for b in 512 1024 2048; do
    for P in syn200 abilene; do
      GSC_SPLITK_BLOCKS=$b timeout -k 10 400 python bench.py --preset $P --steps 30 --warmup 5 > $OUT/b.json 2> $OUT/b.err || exit $?
      echo "$i blocks=$b $P: $(grep -o '"value": [0-9.]*' $OUT/b.json)" >> $OUT/ab.txt
    done
  done
done
cat $OUT/ab.txt
