#!/bin/bash
# simulator A/B: lane-0 handlers vs wave-uniform handlers (device == host tests for both + throughput)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
GSC_SIM_UNIFORM=1 timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_sim.py -x -q --timeout 120 --timeout-method thread > $OUT/sim_tests_uni.log 2>&1 &&
for u in 0 1 0 1; do
  GSC_SIM_UNIFORM=$u timeout -k 10 120 python $R/scripts/sim_throughput.py --steps 100 2>&1 | grep env_steps | sed "s/^/uni=$u /" >> $OUT/simab.txt || exit 1
done
