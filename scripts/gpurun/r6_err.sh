#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/lg_err.txt
for nl in ${NLS:-4 2}; do
  echo "GSC_LG_BWD_NL=$nl" >> $OUT/lg_err.txt
  GSC_LG_BWD_NL=$nl LG_MODES=1 timeout -k 10 200 python -u $R/scripts/diag/lg_err.py ${ERR:-22} >> $OUT/lg_err.txt 2>&1 || exit $?
done
