#!/bin/bash
# Layer-wise GATv2 (200-node graphs): numerics tests, then the syn200 bench with its timed-window
# kernel table (rocprof last: its finalizer may crash after the database is written).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread $R/tests/test_gpu_gnn_lw.py \
  $R/tests/test_large_topologies.py > $OUT/lw_tests.txt 2>&1 &&
bash $R/scripts/gpurun/preset_prof.sh syn200 25 5
