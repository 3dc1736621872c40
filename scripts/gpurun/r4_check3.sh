#!/bin/bash
# restored LDS-resident kernel layout: simulator on 64 / 128 / 256 CUs, headline bench x2, then the full GPU
# suite and smoke
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/r4c3.txt
for cus in 64 128 0; do
  timeout -k 10 120 python $R/scripts/sim_throughput.py --steps 100 --cus $cus > $OUT/ab_sim.txt 2>&1 || exit $?
  echo "sim: $(grep cus= $OUT/ab_sim.txt)" >> $OUT/r4c3.txt
done
for k in 1 2; do
  timeout -k 10 300 python $R/bench.py --steps 40 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit $?
  echo "bench: $(cut -c1-160 $OUT/bench.json)" >> $OUT/r4c3.txt
done
timeout -k 10 1000 python -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
