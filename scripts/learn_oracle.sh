#!/bin/bash
# CPU oracle learning curves for profiles/learning_curves.md: backend "oracle" = the event-driven host
# simulator plus SimpleDDPG on the CPU with the reference's update schedule (200 updates of batch 100 at
# every episode end).  20 episodes, 3 seeds, bounded (sigmoid) and reference (unbounded) actors.
#   OUT=/tmp/lc bash scripts/learn_oracle.sh      (~50 min on 8 CPUs)
cd "$(dirname "$0")/.."
OUT=${OUT:-/tmp/lc}
mkdir -p "$OUT"
run() {
  OMP_NUM_THREADS=2 timeout 3000 python main.py configs/config/agent/$1.yaml \
    configs/networks/abilene/abilene-in4-rand-cap1-2.graphml configs/service_functions/abc.yaml \
    configs/config/simulator/sample_config.yaml configs/config/scheduler.yaml 20 --backend oracle --device cpu \
    --no-test --seed $2 --results-root "$OUT/$1_s$2" > "$OUT/$1_s$2.log" 2>&1
}
run sample_agent_sigmoid 0 & run sample_agent_sigmoid 1 & run sample_agent_sigmoid 2 & wait
run sample_agent 0 & run sample_agent 1 & run sample_agent 2 & wait
