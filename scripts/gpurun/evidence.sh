#!/bin/bash
# Round evidence: GPU tests, smoke, the headline bench and the config-4/5 presets (JSON), then a
# rocprofv3 kernel table of the headline's TIMED steps only (GSC_PROF_WINDOW=1 + --marker-trace; cut by
# scripts/prof_summary.py; last: the profiled process may crash in the tool's finalizer).
# Usage: evidence.sh [tests|notests] [abilene|syn50|syn200 (profiled preset)]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
if [ "${1:-tests}" = tests ]; then
  timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
  timeout -k 10 300 python -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
fi
P=${2:-abilene}
timeout -k 10 300 python $R/bench.py --steps 40 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 300 python $R/bench.py --preset syn50 --steps 10 --warmup 3 > $OUT/bench_syn50.json 2> $OUT/bench_syn50.err &&
timeout -k 10 400 python $R/bench.py --preset syn200 --steps 25 --warmup 5 > $OUT/bench_syn200.json 2> $OUT/bench_syn200.err &&
cd /tmp && export TMPDIR=/tmp && export GSC_PROF_WINDOW=1 && rm -rf $OUT/prof_$P &&
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --stats -d $OUT/prof_$P -o run -- python3 $R/bench.py --preset $P --steps 20 --warmup 5 > $OUT/prof_$P.log 2>&1
