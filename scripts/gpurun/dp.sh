#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest $R/tests/test_gpu_dp.py -x -v -s --timeout 150 --timeout-method thread > $OUT/dp_test.log 2>&1 &&
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_learner.py $R/tests/test_gpu_mlp.py -x -q --timeout 200 --timeout-method thread > $OUT/quick_tests.log 2>&1 &&
timeout -k 10 120 python $R/scripts/gemm_epi_bench.py > $OUT/gemm_epi.txt 2>&1 &&
bash $R/scripts/gpurun/simcus_sweep.sh
