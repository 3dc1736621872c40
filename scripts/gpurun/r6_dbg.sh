#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/lg_dbg.txt
for nl in 4 2; do
  echo "NL=$nl" >> $OUT/lg_dbg.txt
  GSC_LG_PROF=1 GSC_LG_BWD_NL=$nl timeout -k 10 120 python -u $R/scripts/diag/lg_dbg.py 64 >> $OUT/lg_dbg.txt 2>&1 || exit $?
done
