#!/bin/bash
# simulator: device == host tests, per-state profile, standalone throughput, headline bench, then PMC passes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_sim.py -x -q --timeout 120 --timeout-method thread > $OUT/sim_tests.log 2>&1 &&
timeout -k 10 120 python $R/scripts/sim_throughput.py --profile --steps 50 > $OUT/simprof.txt 2>&1 &&
timeout -k 10 120 python $R/scripts/sim_throughput.py --steps 100 >> $OUT/simprof.txt 2>&1 &&
for i in 1 2; do timeout -k 10 200 python $R/bench.py --steps 40 --warmup 5 2>/dev/null | grep -o '"value": [0-9.]*' >> $OUT/simprof.txt || exit 1; done &&
if [ -n "$PMC" ]; then bash $R/scripts/gpurun/gpu_simpmc.sh; fi
