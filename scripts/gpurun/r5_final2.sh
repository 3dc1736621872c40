#!/bin/bash
# evidence at HEAD: full GPU suite, smoke, the three preset benches (headline at the driver's 20 steps and at 50)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/final2
mkdir -p $OUT
: > $OUT/final.txt
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
echo "gpu tests: $(tail -1 $OUT/gpu_tests.log)" >> $OUT/final.txt
timeout -k 10 300 python -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
echo "smoke: $(tail -1 $OUT/smoke.log | cut -c1-80)" >> $OUT/final.txt
timeout -k 10 300 python $R/bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit $?
timeout -k 10 300 python $R/bench.py --steps 50 --warmup 5 > $OUT/bench_abilene.json 2> $OUT/bench_abilene.err || exit $?
timeout -k 10 400 python $R/bench.py --preset syn50 --steps 40 --warmup 5 > $OUT/bench_syn50.json 2> $OUT/bench_syn50.err || exit $?
timeout -k 10 400 python $R/bench.py --preset syn200 --steps 20 --warmup 5 > $OUT/bench_syn200.json 2> $OUT/bench_syn200.err || exit $?
for f in default abilene syn50 syn200; do echo "$f: $(grep -o '"value": [0-9.]*' $OUT/bench_$f.json)" >> $OUT/final.txt; done
