#!/bin/bash
# simulator changes: device == host tests, benches (non-profiling kernels), then the per-preset
# cycle profiles (profiling variant) last
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_sim.py $R/tests/test_gpu_replay.py $R/tests/test_faults.py -x -v --timeout 120 --timeout-method thread > $OUT/sim_tests.log 2>&1 &&
timeout -k 10 120 python $R/scripts/sim_throughput.py --steps 100 > $OUT/sim_tp.txt 2>&1 &&
timeout -k 10 300 python $R/bench.py --steps 40 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 300 python $R/bench.py --preset syn50 --steps 10 --warmup 3 > $OUT/bench_syn50.json 2> $OUT/bench_syn50.err &&
timeout -k 10 400 python $R/bench.py --preset syn200 --steps 25 --warmup 5 > $OUT/bench_syn200.json 2> $OUT/bench_syn200.err &&
bash $R/scripts/gpurun/syn50_partition.sh &&
timeout -k 10 200 python $R/scripts/sim_throughput.py --preset syn50 --steps 10 --profile > $OUT/sim_prof_syn50.txt 2>&1
