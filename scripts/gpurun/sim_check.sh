#!/bin/bash
# simulator: device == host tests, standalone throughput, per-(type, state) cycle profile
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_sim.py -x -q --timeout 120 --timeout-method thread > $OUT/sim_tests.log 2>&1 &&
timeout -k 10 120 python $R/scripts/sim_throughput.py --steps 100 > $OUT/simq.txt 2>&1 &&
timeout -k 10 120 python $R/scripts/sim_throughput.py --steps 30 --profile >> $OUT/simq.txt 2>&1
