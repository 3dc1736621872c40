#!/bin/bash
# rocprofv3 kernel tables of the syn50 / syn200 presets (BASELINE configs 4 / 5)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof50 -o run -- python3 $R/bench.py --preset syn50 --steps 6 --warmup 2 > $OUT/prof50.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof200 -o run -- python3 $R/bench.py --preset syn200 --steps 6 --warmup 2 > $OUT/prof200.log 2>&1
ls $OUT/prof50 $OUT/prof200
