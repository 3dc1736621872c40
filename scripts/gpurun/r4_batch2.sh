#!/bin/bash
# round-4 batch 2: 200-node GNN (MFMA linears / input gradients / weight gradients) checks + benches, then
# batch 1 (A/B of native builds, DP + ops + learner tests, config-5 timed-window profile)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/scripts/gpurun/gnn200_check.sh && bash $R/scripts/gpurun/r4_batch1.sh
