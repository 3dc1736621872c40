#!/bin/bash
# Bounded (sigmoid) actor on the native learner: learner tests vs the fp32 CPU learner, the headline
# bench with sample_agent_sigmoid.yaml, and a timed-window kernel table of it (no hipBLASLt / autograd
# kernels expected)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
AG=$R/configs/config/agent/sample_agent_sigmoid.yaml
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_learner.py $R/tests/test_gpu_mlp.py -x -v --timeout 200 --timeout-method thread > $OUT/learner_tests.log 2>&1 &&
timeout -k 10 300 python $R/bench.py --agent-config $AG --steps 40 --warmup 5 > $OUT/bench_sigmoid.json 2> $OUT/bench_sigmoid.err &&
timeout -k 10 300 python $R/bench.py --steps 40 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err &&
cd /tmp && export TMPDIR=/tmp && export GSC_PROF_WINDOW=1 && rm -rf $OUT/prof_sigmoid &&
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --stats -d $OUT/prof_sigmoid -o run -- python3 $R/bench.py --agent-config $AG --steps 20 --warmup 5 > $OUT/prof_sigmoid.log 2>&1
