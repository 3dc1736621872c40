#!/bin/bash
# headline bench over different timed windows: within one episode (190 steps) vs across the boundary;
# the config-5 preset (scheduler switches) after
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/bench_windows.txt
for sw in "190 5" "201 5"; do
  set -- $sw
  timeout -k 10 300 python $R/bench.py --steps $1 --warmup $2 > $OUT/p.json 2> $OUT/p.err || exit $?
  echo "steps=$1 warmup=$2 $(cat $OUT/p.json)" >> $OUT/bench_windows.txt
done
timeout -k 10 400 python $R/bench.py --preset syn200 --steps 25 --warmup 5 > $OUT/bench_syn200.json 2> $OUT/bench_syn200.err &&
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_cli.py -x -q --timeout 120 --timeout-method thread > $OUT/cli_tests.log 2>&1
