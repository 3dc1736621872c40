#!/bin/bash
# One GPU call: numerics tests, smoke, bench, rocprofv3 kernel stats. Each GPU step has its own
# time limit and steps are chained so that a failure ends the call.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
STEPS=${STEPS:-30}
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 400 python $R/bench.py --steps $STEPS --warmup 5 > $OUT/bench.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python $R/bench.py --steps 10 --warmup 3 > $OUT/prof.log 2>&1
