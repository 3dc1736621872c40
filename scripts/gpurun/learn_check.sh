#!/bin/bash
# Learning check: composed vs materialised actor loss, fp32 learner + fp32 reference embedder,
# 3 seeds each, 10 lockstep episodes of 256 envs; plus the reference update ratio (E updates of 100).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/learn
mkdir -p $OUT
EP=${EP:-10}
for seed in 0 1 2; do
  GSC_GNN_NATIVE=0 timeout -k 10 200 python -u $R/scripts/train_curve.py --fp32 --episodes $EP --seed $seed --tag "compose s$seed" >> $OUT/compose.txt 2>&1 || exit 1
  GSC_COMPOSE=0 GSC_GNN_NATIVE=0 timeout -k 10 200 python -u $R/scripts/train_curve.py --fp32 --episodes $EP --seed $seed --tag "material s$seed" >> $OUT/material.txt 2>&1 || exit 1
done
timeout -k 10 400 python -u $R/scripts/train_curve.py --episodes $EP --envs 32 --ref-ratio --tag "refratio" >> $OUT/refratio.txt 2>&1
