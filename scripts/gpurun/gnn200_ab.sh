#!/bin/bash
# 200-node layer-wise GNN: numerics (tests/test_gpu_gnn_lw.py), then fwd / fwd+bwd timing at the config-5
# learner batch for the variants in VARIANTS ("<GSC_LW_MFMA>:<GSC_LW_STREAM_GRADS>")
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/gnn200_ab.txt
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_gnn_lw.py -x -v --timeout 120 --timeout-method thread > $OUT/gnn_lw.log 2>&1 || exit $?
echo "gnn_lw: $(tail -1 $OUT/gnn_lw.log)" >> $OUT/gnn200_ab.txt
for v in ${VARIANTS:-1:1 1:0}; do
  GSC_LW_MFMA=${v%%:*} GSC_LW_STREAM_GRADS=${v##*:} timeout -k 10 300 python $R/scripts/gnn_bench.py --network $R/configs/networks/synthetic/syn200-in16-cap1-3-s0.graphml --n-pad 200 --batch 25600 --iters 5 > $OUT/gnn200_v.txt 2>&1 || exit $?
  echo "$v $(grep layer-wise $OUT/gnn200_v.txt)" >> $OUT/gnn200_ab.txt
done
