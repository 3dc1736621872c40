#!/bin/bash
# Round evidence in one call: GPU tests, smoke, headline bench (JSON), BASELINE config 4/5 presets,
# then the rocprofv3 kernel table of the headline step (last: the profiled process can crash in the
# tool's finalizer after the database is written).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 python $R/bench.py --steps 40 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 300 python $R/bench.py --preset syn50 --steps 10 --warmup 3 > $OUT/bench_syn50.json 2> $OUT/bench_syn50.err &&
timeout -k 10 400 python $R/bench.py --preset syn200 --steps 5 --warmup 2 > $OUT/bench_syn200.json 2> $OUT/bench_syn200.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python $R/bench.py --steps 10 --warmup 3 > $OUT/prof.log 2>&1
