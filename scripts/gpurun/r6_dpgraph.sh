#!/bin/bash
# DP update with its all-reduces captured in the one update graph: the world-size-1 RCCL tests, then the
# headline bench plain / forced-RCCL (one graph) / forced-RCCL with GSC_DP_GRAPH=0 (five graphs, eager collectives)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/dpgraph
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 5 > $OUT/plain_$i.json 2> $OUT/plain_$i.err || exit $?
  GSC_DIST_FORCE=1 timeout -k 10 300 python bench.py --steps 50 --warmup 5 > $OUT/dp_$i.json 2> $OUT/dp_$i.err || exit $?
  GSC_DIST_FORCE=1 GSC_DP_GRAPH=0 timeout -k 10 300 python bench.py --steps 50 --warmup 5 > $OUT/dpeager_$i.json 2> $OUT/dpeager_$i.err || exit $?
done
