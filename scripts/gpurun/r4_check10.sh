#!/bin/bash
# full GPU suite + smoke, the three preset benches, then the Abilene timed-window trace (last: the profiled
# process can segfault in the tool finalizer)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/r4c10.txt
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
echo "gpu tests: $(tail -1 $OUT/gpu_tests.log)" >> $OUT/r4c10.txt
timeout -k 10 300 python -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
echo "smoke: $(tail -1 $OUT/smoke.log | cut -c1-100)" >> $OUT/r4c10.txt
for p in syn200 abilene syn50; do
  timeout -k 10 400 python $R/bench.py --preset $p --steps ${STEPS:-30} --warmup 5 > $OUT/bench_$p.json 2> $OUT/bench_$p.err || exit $?
  echo "$p: $(cut -c1-250 $OUT/bench_$p.json)" >> $OUT/r4c10.txt
done
PRESET=abilene STEPS=20 bash $R/scripts/gpurun/prof_preset.sh
