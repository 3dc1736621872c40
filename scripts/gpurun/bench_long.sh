#!/bin/bash
# headline bench over 201 timed steps (crosses an episode boundary: all 256 envs reset in one step)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python $R/bench.py --steps 201 --warmup 5 > $OUT/bench_201.json 2> $OUT/bench_201.err
