#!/bin/bash
# kernel changes check: GNN / explore / learner / simulator GPU tests, simulator throughput per preset,
# GNN micro-bench, headline bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_ops.py $R/tests/test_gpu_learner.py $R/tests/test_gpu_sim.py -x -v -s --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 &&
timeout -k 10 120 python $R/scripts/sim_throughput.py --steps 100 > $OUT/sim_tp.txt 2>&1 &&
timeout -k 10 120 python $R/scripts/sim_throughput.py --preset syn50 --steps 20 >> $OUT/sim_tp.txt 2>&1 &&
timeout -k 10 200 python $R/scripts/sim_throughput.py --preset syn200 --steps 10 --envs 64 >> $OUT/sim_tp.txt 2>&1 &&
timeout -k 10 120 python $R/scripts/gnn_bench.py > $OUT/gb.txt 2>&1 &&
timeout -k 10 200 python $R/bench.py --steps 30 --warmup 5 > $OUT/bench.json 2>$OUT/bench.err
