#!/bin/bash
# simulator: device == host tests, throughput with / without the compile-time dims bucket, profile
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_sim.py -x -q --timeout 120 --timeout-method thread > $OUT/sim_tests.log 2>&1 &&
for b in 1 0 1; do
  GSC_SIM_BUCKET=$b timeout -k 10 120 python $R/scripts/sim_throughput.py --steps 100 2>&1 | grep env_steps | sed "s/^/bucket=$b /" >> $OUT/simab.txt || exit 1
done
timeout -k 10 120 python $R/scripts/sim_throughput.py --steps 30 --profile > $OUT/simprof.txt 2>&1
