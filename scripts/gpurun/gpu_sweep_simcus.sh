#!/bin/bash
# bench.py over simulator CU reservations (one GPU process at a time, each under its own limit)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/sweep.txt
for K in ${KS:-0 64 96 128}; do
  timeout -k 10 240 python $R/bench.py --steps 30 --warmup 5 --sim-cus $K > $OUT/bench_k$K.log 2>&1 || exit 1
  echo "sim_cus=$K $(tail -1 $OUT/bench_k$K.log | cut -c1-160)" >> $OUT/sweep.txt
done
