#!/bin/bash
# A/B of builds of the native extension on one box (GSC_NATIVE_SO = an alternative build; "new" = the
# in-tree build): standalone simulator and the headline bench, interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
VARIANTS=${VARIANTS:-"new old"}
: > $OUT/ab.txt
for k in 1 2; do
  for v in $VARIANTS; do
    if [ $v = new ]; then unset GSC_NATIVE_SO; else export GSC_NATIVE_SO=$R/ab/_native_$v.cpython-310-x86_64-linux-gnu.so; fi
    timeout -k 10 120 python $R/scripts/sim_throughput.py --steps 100 > $OUT/ab_sim.txt 2>&1 || exit $?
    echo "$v sim: $(grep cus= $OUT/ab_sim.txt)" >> $OUT/ab.txt
    timeout -k 10 300 python $R/bench.py --steps 40 --warmup 5 > $OUT/ab_bench.json 2> $OUT/ab_bench.err || exit $?
    echo "$v bench: $(cat $OUT/ab_bench.json)" >> $OUT/ab.txt
  done
done
