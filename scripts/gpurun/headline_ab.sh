#!/bin/bash
# headline critical path: full step vs the act + simulator chain alone (GSC_DIAG_NO_LEARN=1, diagnostic), and
# the simulator partition sizes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/headline_ab.txt
for k in 1 2; do
  for v in full nolearn cus96 cus128; do
    case $v in
      full) E=""; A="";;
      nolearn) E="GSC_DIAG_NO_LEARN=1"; A="";;
      cus96) E=""; A="--sim-cus 96";;
      cus128) E=""; A="--sim-cus 128";;
    esac
    env $E timeout -k 10 300 python $R/bench.py --steps 40 --warmup 5 $A > $OUT/hb.json 2> $OUT/hb.err || exit $?
    echo "$v $(grep -o '"value": [0-9.]*' $OUT/hb.json)" >> $OUT/headline_ab.txt
  done
done
