#!/bin/bash
# One PMC pass over a short bench run (counters only; no trace domains). PMC="<counters>" PASS=<name>.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_${PASS}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 120 rocprofv3 --pmc $PMC --output-format csv -d $OUT -o run -- python3 $R/bench.py --steps 3 --warmup 2 > $OUT/log.txt 2>&1
