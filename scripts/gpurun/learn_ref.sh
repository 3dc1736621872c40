#!/bin/bash
# Learning under the reference update rule: GPU learner, one env with one batch-100
# update per env-step (the reference's ratio; the CPU oracle runs SimpleDDPG's 200 updates at every
# episode end), bounded (sigmoid) and reference (unbounded) actors; plus 32 envs x 32 updates (reference
# ratio) and the batched rule (one batch-25,600 update per step of 256 envs), sigmoid actor.  3 seeds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/learn
mkdir -p $OUT
EP=${EP:-20}
for seed in 0 1 2; do
  for ag in sample_agent_sigmoid sample_agent; do
    timeout -k 10 300 python -u $R/scripts/train_curve.py --episodes $EP --envs 1 --ref-ratio --seed $seed \
      --agent configs/config/agent/$ag.yaml --tag "e1-refratio $ag s$seed" >> $OUT/e1_$ag.txt 2>&1 || exit 1
  done
  timeout -k 10 400 python -u $R/scripts/train_curve.py --episodes $EP --envs 32 --ref-ratio --seed $seed \
    --agent configs/config/agent/sample_agent_sigmoid.yaml --tag "e32-refratio sigmoid s$seed" >> $OUT/e32_sigmoid.txt 2>&1 || exit 1
  timeout -k 10 300 python -u $R/scripts/train_curve.py --episodes $EP --envs 256 --seed $seed \
    --agent configs/config/agent/sample_agent_sigmoid.yaml --tag "e256-batched sigmoid s$seed" >> $OUT/e256_sigmoid.txt 2>&1 || exit 1
done
