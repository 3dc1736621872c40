#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/bk.txt
for b in 32 64; do
  GSC_GEMM_BK=$b timeout -k 10 120 python $R/scripts/gemm_epi_bench.py 2>&1 | grep -v amdgpu | sed "s/^/bk=$b /" >> $OUT/bk.txt || exit 1
  GSC_GEMM_BK=$b timeout -k 10 120 python $R/scripts/mlp_bench.py 2>&1 | grep -v amdgpu | sed "s/^/bk=$b /" >> $OUT/bk.txt || exit 1
done
for b in 32 64 32 64; do
  GSC_GEMM_BK=$b timeout -k 10 200 python $R/bench.py --steps 40 --warmup 5 2>/dev/null | grep -o '"value": [0-9.]*' | sed "s/^/bench bk=$b /" >> $OUT/bk.txt || exit 1
done
GSC_GEMM_BK=64 timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_mlp.py $R/tests/test_gpu_learner.py -x -q --timeout 200 --timeout-method thread >> $OUT/bk.txt 2>&1
