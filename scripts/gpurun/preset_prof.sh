#!/bin/bash
# One preset's bench JSON and its rocprofv3 kernel table over the timed steps only.
# Usage: preset_prof.sh <preset> <steps> <warmup>   (the profiled process may crash in the tool's
# finalizer after the database is written: keep this the last GPU step of a call)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
P=${1:-abilene}; S=${2:-20}; W=${3:-5}
mkdir -p $OUT
rm -rf $OUT/prof_$P
timeout -k 10 400 python $R/bench.py --preset $P --steps $S --warmup $W > $OUT/bench_$P.json 2> $OUT/bench_$P.err &&
cd /tmp && export TMPDIR=/tmp && export GSC_PROF_WINDOW=1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --stats -d $OUT/prof_$P -o run -- python3 $R/bench.py --preset $P --steps $S --warmup $W > $OUT/prof_$P.log 2>&1
