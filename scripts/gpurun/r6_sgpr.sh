#!/bin/bash
# SGPR-spill A/B: the standalone simulator (256 Abilene envs, the bench's 64 XCD-spread CUs) with the default build and
# SGPR-capped variants (scripts/sim_sgpr_ab.py), interleaved, two rounds
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/sgpr
mkdir -p $OUT
cd $R
: > $OUT/ab.txt
for round in 1 2; do
  for v in default 96 88 80 64; do
    if [ $v = default ]; then so=""; else so=$(ls $R/ab/simvar/sgpr$v/_native*.so); fi
    echo "== round $round variant $v" >> $OUT/ab.txt
    GSC_NATIVE_SO=$so timeout -k 10 120 python scripts/sim_throughput.py --cus 64 --cu-per-xcd 8 --steps 200 >> $OUT/ab.txt 2>&1 || exit $?
  done
done
