#!/bin/bash
# Learning check, default (native bf16) learner: composed vs materialised actor loss, 3 seeds; and the
# reference update ratio (E updates of batch 100 per step) with the sigmoid-bounded actor.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/learn
mkdir -p $OUT
EP=${EP:-10}
for seed in 0 1 2; do
  timeout -k 10 200 python -u $R/scripts/train_curve.py --episodes $EP --seed $seed --tag "bf16-compose s$seed" >> $OUT/bf16_compose.txt 2>&1 || exit 1
  GSC_COMPOSE=0 timeout -k 10 200 python -u $R/scripts/train_curve.py --episodes $EP --seed $seed --tag "bf16-material s$seed" >> $OUT/bf16_material.txt 2>&1 || exit 1
done
timeout -k 10 400 python -u $R/scripts/train_curve.py --episodes $EP --envs 32 --ref-ratio --agent configs/config/agent/sample_agent_sigmoid.yaml --tag "refratio-sigmoid" >> $OUT/refratio_sigmoid.txt 2>&1
