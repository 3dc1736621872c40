#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_mlp.py $R/tests/test_gpu_learner.py $R/tests/test_gpu_graphs.py -x -q --timeout 200 --timeout-method thread > $OUT/epi_tests.log 2>&1 &&
timeout -k 10 120 python $R/scripts/gemm_epi_bench.py > $OUT/epi.txt 2>&1 &&
timeout -k 10 120 python $R/scripts/mlp_bench.py >> $OUT/epi.txt 2>&1 &&
for i in 1 2; do timeout -k 10 200 python $R/bench.py --steps 40 --warmup 5 2>/dev/null | grep -o '"value": [0-9.]*' >> $OUT/epi.txt || exit 1; done
