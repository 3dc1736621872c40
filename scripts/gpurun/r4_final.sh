#!/bin/bash
# round-end evidence at HEAD: full GPU suite, smoke, DP rehearsal record, 200-node GNN timing, the three preset
# benches, then the syn200 timed-window trace last (the profiled process can segfault in the tool finalizer)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/final.txt
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
echo "gpu tests: $(tail -1 $OUT/gpu_tests.log)" >> $OUT/final.txt
timeout -k 10 300 python -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
echo "smoke: $(tail -1 $OUT/smoke.log | cut -c1-80)" >> $OUT/final.txt
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_dp.py -v -s --timeout 150 --timeout-method thread > $OUT/gpu_dp_rehearsal.txt 2>&1 || exit $?
VARIANTS="1:1" bash $R/scripts/gpurun/gnn200_ab.sh || exit $?
cat $OUT/gnn200_ab.txt >> $OUT/final.txt
for p in abilene syn50 syn200; do
  timeout -k 10 400 python $R/bench.py --preset $p --steps 40 --warmup 5 > $OUT/bench_$p.json 2> $OUT/bench_$p.err || exit $?
  echo "$p: $(grep -o '"value": [0-9.]*' $OUT/bench_$p.json)" >> $OUT/final.txt
done
PRESET=syn200 STEPS=20 bash $R/scripts/gpurun/prof_preset.sh
