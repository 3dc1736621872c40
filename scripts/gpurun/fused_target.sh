#!/bin/bash
# Fused target projection: kernel + learner numerics, then the abilene headline and syn200 benches with
# the fused path off / on (GSC_FUSE_TARGET).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread $R/tests/test_gpu_ops.py::test_actor_proj_matches_reference \
  $R/tests/test_gpu_learner.py > $OUT/fused_tests.txt 2>&1 &&
for f in 0 1; do
  GSC_FUSE_TARGET=$f timeout -k 10 300 python $R/bench.py --steps 100 --warmup 10 > $OUT/bench_abilene_fuse$f.json 2>/dev/null || exit 1
  GSC_FUSE_TARGET=$f timeout -k 10 300 python $R/bench.py --preset syn200 --steps 25 --warmup 5 > $OUT/bench_syn200_fuse$f.json 2>/dev/null || exit 1
done
