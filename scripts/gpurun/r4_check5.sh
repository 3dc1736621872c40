#!/bin/bash
# full GPU suite (GEMM row-image swizzle, gnn_mt NVS, staged 200-node GNN kernels), smoke, then the
# config-5 (256 envs, 25,600 samples) timed-window kernel table last (the profiled process can segfault
# in the tool's finalizer after the database is written)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && export GSC_PROF_WINDOW=1 && rm -rf $OUT/prof_${PRESET:-syn200}full &&
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats -d $OUT/prof_${PRESET:-syn200}full -o run -- python3 $R/bench.py --preset ${PRESET:-syn200} ${BENCH_ARGS:---envs 256 --batch-size 25600} --steps 4 --warmup 3 > $OUT/prof_${PRESET:-syn200}full.log 2>&1
