#!/bin/bash
# native learner: GEMM tests + whole-update tests vs the fp32 reference
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_learner.py -v -s --timeout 200 --timeout-method thread > $OUT/learner_tests.log 2>&1
