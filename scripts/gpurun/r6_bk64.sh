#!/bin/bash
# split-K weight-gradient GEMMs staged 64 deep (GSC_SPLITK_BK64=1) vs 32, interleaved, syn200 and the headline
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/bk64
mkdir -p $OUT
cd $R
: > $OUT/ab.txt
for i in 1 2; do
  for b in 0 1; do
    for P in syn200 abilene; do
      GSC_SPLITK_BK64=$b timeout -k 10 400 python bench.py --preset $P --steps 30 --warmup 5 > $OUT/b.json 2> $OUT/b.err || exit $?
      echo "$i bk64=$b $P: $(grep -o '"value": [0-9.]*' $OUT/b.json)" >> $OUT/ab.txt
    done
  done
done
cat $OUT/ab.txt
