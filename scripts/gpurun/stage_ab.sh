#!/bin/bash
# batched GNN input staging A/B: in-tree build vs ab/_native_prestage (HEAD before it), interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/stage_ab.txt
for k in 1 2; do
  for v in new prestage; do
    if [ $v = new ]; then unset GSC_NATIVE_SO; else export GSC_NATIVE_SO=$R/ab/_native_prestage.cpython-310-x86_64-linux-gnu.so; fi
    timeout -k 10 300 python $R/scripts/gnn_bench.py --iters 10 > $OUT/sab.txt 2>&1 || exit $?
    echo "$v abilene-gnn $(grep fused $OUT/sab.txt | cut -d: -f2-)" >> $OUT/stage_ab.txt
    timeout -k 10 300 python $R/scripts/gnn_bench.py --iters 10 --network $R/configs/networks/synthetic/syn50-in8-cap1-3.graphml --n-pad 50 > $OUT/sab.txt 2>&1 || exit $?
    echo "$v syn50-gnn $(grep fused $OUT/sab.txt | cut -d: -f2-)" >> $OUT/stage_ab.txt
    timeout -k 10 400 python $R/bench.py --preset syn50 --steps 40 --warmup 5 > $OUT/sab.json 2> $OUT/sab.err || exit $?
    echo "$v syn50 $(grep -o '"value": [0-9.]*' $OUT/sab.json)" >> $OUT/stage_ab.txt
  done
done
