#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u $R/scripts/diag/lg_err.py 8 12 16 22 > $OUT/lg_err.txt 2>&1
