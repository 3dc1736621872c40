#!/bin/bash
# One PMC pass (counters only, no trace domains) over a short bench.py run: PASS=<name> PMC="<counters>"
# [PRESET=abilene|syn50|syn200] (bench.py's profiled process can segfault at exit inside the tool's
# finalizer after the csv is written, so each pass is its own gpurun call)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/bench_pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 150 rocprofv3 --pmc $PMC --output-format csv -d $OUT/$PASS -o run -- python3 $R/bench.py --preset ${PRESET:-abilene} --steps 3 --warmup 2 > $OUT/$PASS.log 2>&1
