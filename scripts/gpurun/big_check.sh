#!/bin/bash
# Large-topology simulator (action block read in place, pmask pre-kernel, lazy WRR resets) + row-indexed
# replay reads: device == host tests, GEMM / learner tests, standalone simulator, config-4/5 benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_sim.py $R/tests/test_gpu_mlp.py $R/tests/test_gpu_learner.py -x -v --timeout 200 --timeout-method thread > $OUT/big_tests.log 2>&1 &&
timeout -k 10 200 python $R/scripts/sim_throughput.py --preset syn200 --steps 30 > $OUT/sim_tp_syn200.txt 2>&1 &&
timeout -k 10 200 python $R/scripts/sim_throughput.py --preset syn200 --steps 30 --profile > $OUT/sim_prof_syn200.txt 2>&1 &&
timeout -k 10 200 python $R/scripts/sim_throughput.py --preset syn50 --steps 30 > $OUT/sim_tp_syn50.txt 2>&1 &&
timeout -k 10 300 python $R/bench.py --steps 40 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 300 python $R/bench.py --preset syn50 --steps 10 --warmup 3 > $OUT/bench_syn50.json 2> $OUT/bench_syn50.err &&
timeout -k 10 400 python $R/bench.py --preset syn200 --steps 25 --warmup 5 > $OUT/bench_syn200.json 2> $OUT/bench_syn200.err &&
timeout -k 10 400 python $R/bench.py --preset syn200 --envs 256 --steps 25 --warmup 5 > $OUT/bench_syn200_e256.json 2> $OUT/bench_syn200_e256.err &&
timeout -k 10 600 python $R/bench.py --preset syn200 --envs 256 --batch-size 25600 --steps 5 --warmup 3 > $OUT/bench_syn200_full.json 2> $OUT/bench_syn200_full.err
