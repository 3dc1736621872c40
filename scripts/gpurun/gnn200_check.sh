#!/bin/bash
# 200-node layer-wise GATv2: MFMA node linears / input gradients (default) vs the VALU epilogues
# (GSC_LW_MFMA=0): fp32-reference tests, micro-benchmark at 2,048 and 25,600 graphs, config-5 bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_gnn_lw.py -x -v --timeout 200 --timeout-method thread > $OUT/gnn200_tests.log 2>&1 &&
: > $OUT/gnn200_bench.txt &&
for B in 2048 25600; do
  for m in 1 0; do
    GSC_LW_MFMA=$m timeout -k 10 200 python $R/scripts/gnn_bench.py --network configs/networks/synthetic/syn200-in16-cap1-3-s0.graphml --n-pad 200 --batch $B --iters 5 > $OUT/gb.txt 2>&1 || exit $?
    echo "GSC_LW_MFMA=$m $(tail -1 $OUT/gb.txt)" >> $OUT/gnn200_bench.txt
  done
done &&
timeout -k 10 600 python $R/bench.py --preset syn200 --envs 256 --batch-size 25600 --steps 4 --warmup 3 > $OUT/bench_syn200_full.json 2> $OUT/bench_syn200_full.err &&
timeout -k 10 400 python $R/bench.py --preset syn200 --steps 25 --warmup 5 > $OUT/bench_syn200.json 2> $OUT/bench_syn200.err
