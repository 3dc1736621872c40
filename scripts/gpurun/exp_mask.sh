#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/exp_mask.txt
for m in 0 1 0 1; do
  GSC_LEARNER_MASK=$m timeout -k 10 200 python $R/bench.py --steps 40 --warmup 5 2>/dev/null | grep -o '"value": [0-9.]*' | sed "s/^/learner_mask=$m /" >> $OUT/exp_mask.txt || exit 1
done
timeout -k 10 100 python -c "
import sys; sys.path.insert(0, '$R')
import os; os.chdir('$R')
import torch, yaml
from gsc_amd.sim.batched import load_batched_from_paths
cfg = yaml.safe_load(open('configs/config/agent/sample_agent.yaml'))
s = load_batched_from_paths(['configs/networks/abilene/abilene-in4-rand-cap1-2.graphml'], 'configs/service_functions/abc.yaml', 'configs/config/simulator/sample_config.yaml', cfg, 256, device='cuda')
s.reset(); a = torch.rand(256, s.action_dim, device='cuda')
from gsc_amd.envs import threshold_normalize
for _ in range(60): o = s.step(a)
torch.cuda.synchronize()
print('max_events', float(o.stats[:, 13].max()), 'max_procs', float(o.stats[:, 14].max()), 'max_flows', float(o.stats[:, 15].max()))
" >> $OUT/exp_mask.txt 2>&1
