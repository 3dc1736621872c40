#!/bin/bash
# timed-window kernel table of one bench preset (PRESET, default syn200); the profiled process can segfault
# in the tool's finalizer after the database is written, so this is the last GPU step of its call
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
P=${PRESET:-syn200}
cd /tmp && export TMPDIR=/tmp && export GSC_PROF_WINDOW=1 && rm -rf $OUT/prof_$P &&
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats -d $OUT/prof_$P -o run -- python3 $R/bench.py --preset $P --steps ${STEPS:-20} --warmup 3 > $OUT/prof_$P.log 2>&1
