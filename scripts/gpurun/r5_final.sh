#!/bin/bash
# evidence at HEAD: full GPU suite, smoke, the headline bench, then 100-episode Abilene learning curves
# (bounded actor, three seeds) with the per-episode return
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT/lc
: > $OUT/final.txt
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
echo "gpu tests: $(tail -1 $OUT/gpu_tests.log)" >> $OUT/final.txt
timeout -k 10 300 python -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
echo "smoke: $(tail -1 $OUT/smoke.log | cut -c1-80)" >> $OUT/final.txt
timeout -k 10 400 python $R/bench.py --steps 40 --warmup 5 > $OUT/bench_abilene.json 2> $OUT/bench_abilene.err || exit $?
echo "abilene: $(grep -o '"value": [0-9.]*' $OUT/bench_abilene.json)" >> $OUT/final.txt
for s in ${SEEDS:-0 1 2}; do
  timeout -k 10 330 python3 -u $R/scripts/train_curve.py --episodes ${EPISODES:-100} --seed $s \
    --agent $R/configs/config/agent/sample_agent_sigmoid.yaml --tag s$s > $OUT/lc/s$s.txt 2>&1 || exit $?
  echo "curve s$s: $(tail -1 $OUT/lc/s$s.txt)" >> $OUT/final.txt
done
