#!/bin/bash
# 200-node layer-wise GATv2: numerics tests, micro-benchmark (B = 2048 graphs) and per-kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
rm -rf $OUT/prof_gnn200
NET=configs/networks/synthetic/syn200-in16-cap1-3-s0.graphml
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread $R/tests/test_gpu_gnn_lw.py > $OUT/lw_tests.txt 2>&1 &&
timeout -k 10 200 python -u $R/scripts/gnn_bench.py --network $NET --n-pad 200 --batch 2048 > $OUT/gnn200.txt 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_gnn200 -o run -- python3 $R/scripts/gnn_bench.py --network $R/$NET --n-pad 200 --batch 2048 > $OUT/prof_gnn200.log 2>&1
