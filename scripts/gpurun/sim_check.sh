#!/bin/bash
# simulator kernel: device == host bit-exact tests, standalone throughput per preset (+ the per-event
# cycle profile on Abilene), headline bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_sim.py -x -v --timeout 120 --timeout-method thread > $OUT/sim_tests.log 2>&1 &&
timeout -k 10 120 python $R/scripts/sim_throughput.py --steps 50 --profile > $OUT/sim_tp.txt 2>&1 &&
timeout -k 10 120 python $R/scripts/sim_throughput.py --steps 100 >> $OUT/sim_tp.txt 2>&1 &&
timeout -k 10 120 python $R/scripts/sim_throughput.py --preset syn50 --steps 20 >> $OUT/sim_tp.txt 2>&1 &&
timeout -k 10 200 python $R/scripts/sim_throughput.py --preset syn200 --steps 10 --envs 64 >> $OUT/sim_tp.txt 2>&1 &&
timeout -k 10 200 python $R/bench.py --steps 30 --warmup 5 > $OUT/bench.json 2>$OUT/bench.err
