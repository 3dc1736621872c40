#!/bin/bash
# exploration tests, then per-kernel mean times of the headline bench for this tree (last: the profiled process can
# crash in the tool's finalizer after the database is written)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/abp
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k explore tests/test_gpu_explore_pmask.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/new -o run -- python3 $R/bench.py --steps 40 --warmup 5 > $OUT/new.log 2>&1
