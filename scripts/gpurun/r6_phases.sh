#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 200 python -u $R/scripts/diag/lg_phases.py > $OUT/lg_phases.txt 2>&1 &&
LG_MODES=1 LG_ITERS=1,2 timeout -k 10 200 python -u $R/scripts/diag/lg_err.py 6 8 9 10 11 12 > $OUT/lg_err2.txt 2>&1
