#!/bin/bash
# round-6 baseline at HEAD: GPU suite, the three bench presets, 200-node GATv2 micro-benchmark
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/base.txt
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
echo "gpu tests: $(tail -1 $OUT/gpu_tests.log)" >> $OUT/base.txt
for P in abilene syn50 syn200; do
  timeout -k 10 400 python $R/bench.py --preset $P --steps 20 --warmup 5 > $OUT/bench_$P.json 2> $OUT/bench_$P.err || exit $?
  echo "$P: $(grep -o '"value": [0-9.]*' $OUT/bench_$P.json)" >> $OUT/base.txt
done
timeout -k 10 200 python $R/scripts/gnn_bench.py --network configs/networks/synthetic/syn200-in16-cap1-3-s0.graphml --n-pad 200 --batch 25600 --iters 5 > $OUT/gb.txt 2>&1 || exit $?
echo "gnn200: $(tail -1 $OUT/gb.txt)" >> $OUT/base.txt
