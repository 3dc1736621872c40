#!/bin/bash
# bench.py at several simulator CU partitions (CUS), then the act/sim chain alone (GSC_DIAG_NO_LEARN) at
# NOLEARN_CUS partitions
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/simcus.txt
for c in ${CUS:-64 80 96 128}; do
  timeout -k 10 120 python $R/bench.py --steps 30 --warmup 5 --sim-cus $c 2>/dev/null | grep -o '"value": [0-9.]*' | sed "s/^/sim_cus=$c /" >> $OUT/simcus.txt || exit 1
done
for c in ${NOLEARN_CUS:--1}; do
  GSC_DIAG_NO_LEARN=1 timeout -k 10 120 python $R/bench.py --steps 30 --warmup 5 --sim-cus $c 2>/dev/null | grep -o '"value": [0-9.]*' | sed "s/^/no_learn sim_cus=$c /" >> $OUT/simcus.txt || exit 1
done
