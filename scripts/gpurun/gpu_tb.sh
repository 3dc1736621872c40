#!/bin/bash
# GPU tests + bench + kernel-trace profile (timeline)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
rm -rf $OUT/prof
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 &&
timeout -k 10 300 python $R/bench.py --steps 30 --warmup 5 $EXTRA > $OUT/bench.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python $R/bench.py --steps 10 --warmup 3 $EXTRA > $OUT/prof.log 2>&1
test -f $OUT/prof/run_results.db
