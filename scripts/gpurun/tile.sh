#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/tile.txt
for t in small large small large; do
  GSC_GEMM_TILE=$t timeout -k 10 200 python $R/bench.py --steps 40 --warmup 5 2>/dev/null | grep -o '"value": [0-9.]*' | sed "s/^/tile=$t /" >> $OUT/tile.txt || exit 1
done
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_mlp.py $R/tests/test_gpu_learner.py -x -q --timeout 200 --timeout-method thread >> $OUT/tile.txt 2>&1
