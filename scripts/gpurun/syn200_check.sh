#!/bin/bash
# syn200 at 256 envs (one rank's share of a 2,048-env 8-GPU job): device == host test, then the
# standalone simulator with and without the cycle-counting variant (20-step episodes: the timed
# window crosses resets), then the Abilene cycle profile at HEAD
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_sim.py -x -v --timeout 200 --timeout-method thread > $OUT/sim_tests.log 2>&1 &&
timeout -k 10 200 python $R/scripts/sim_throughput.py --preset syn200 --steps 30 > $OUT/sim_tp_syn200.txt 2>&1 &&
timeout -k 10 200 python $R/scripts/sim_throughput.py --preset syn200 --steps 30 --profile > $OUT/sim_prof_syn200.txt 2>&1 &&
timeout -k 10 120 python $R/scripts/sim_throughput.py --steps 100 > $OUT/sim_tp.txt 2>&1 &&
timeout -k 10 120 python $R/scripts/sim_throughput.py --steps 50 --profile > $OUT/sim_prof_abilene.txt 2>&1
