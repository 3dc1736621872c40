#!/bin/bash
# Perf probe: sim-only throughput + bench with and without sim/learner stream overlap.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -m pytest $R/tests/test_gpu_sim.py -x -q > $OUT/gpu_sim_test.log 2>&1 &&
timeout -k 10 200 python $R/scripts/sim_throughput.py --envs 256 --steps 100 > $OUT/sim_tp.log 2>&1 &&
timeout -k 10 200 python $R/scripts/sim_throughput.py --envs 2048 --steps 30 >> $OUT/sim_tp.log 2>&1 &&
timeout -k 10 300 python $R/bench.py --steps 30 --warmup 5 > $OUT/bench_overlap.log 2>&1 &&
timeout -k 10 300 python $R/bench.py --steps 30 --warmup 5 --no-overlap > $OUT/bench_serial.log 2>&1
