#!/bin/bash
# sparse product timing, sparse/explore/pmask device tests, config-5/4 benches, syn200 kernel table (last)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-sp6}
mkdir -p $OUT
cd $R
timeout -k 10 200 python3 scripts/sparse_bench.py > $OUT/sbench.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse_replay.py tests/test_gpu_explore_pmask.py tests/test_gpu_ops.py -k "sparse or explore or pmask" -x -v --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1 || exit 1
SKIP_TESTS=1 TAG=${TAG:-sp6} PROF=${PROF:-1} bash scripts/gpurun/r5_sparse.sh
