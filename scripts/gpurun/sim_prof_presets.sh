#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 200 python $R/scripts/sim_throughput.py --preset syn200 --steps 6 --envs 128 --profile > $OUT/sim_prof_syn200.txt 2>&1 &&
timeout -k 10 200 python $R/scripts/sim_throughput.py --preset syn50 --steps 10 --profile > $OUT/sim_prof_syn50.txt 2>&1 &&
bash $R/scripts/gpurun/preset_prof.sh syn50 6 2
