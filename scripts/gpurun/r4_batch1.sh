#!/bin/bash
# round-4 batch: A/B of native builds (headline), DP rehearsal + ops tests, the 200-node learner test, and a
# timed-window kernel table of config 5 at equal learner work (256 envs, 25,600 samples per update)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
VARIANTS="new old newsim_oldgemm" bash $R/scripts/gpurun/ab_native.sh &&
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_dp.py $R/tests/test_gpu_ops.py $R/tests/test_gpu_learner.py -x -v -s --timeout 300 --timeout-method thread > $OUT/dp_tests.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && export GSC_PROF_WINDOW=1 && rm -rf $OUT/prof_syn200full &&
timeout -k 10 500 rocprofv3 --kernel-trace --marker-trace --stats -d $OUT/prof_syn200full -o run -- python3 $R/bench.py --preset syn200 --envs 256 --batch-size 25600 --steps 4 --warmup 3 > $OUT/prof_syn200full.log 2>&1
