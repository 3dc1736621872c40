#!/bin/bash
# gnn_lg gradient determinism at HEAD and at the builds under ab/lgbis/<commit> (each in its own process)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/lgbis
SO=gsc_amd/_native.cpython-310-x86_64-linux-gnu.so
mkdir -p $OUT
: > $OUT/res.txt
cp $R/$SO /tmp/head_native.so || exit 1
echo "HEAD: $(timeout -k 10 120 python $R/scripts/diag/lg_determinism.py 6 2>&1 | tail -1)" >> $OUT/res.txt || exit $?
for c in ${COMMITS:-a0a9be9 7785607 f308f7e}; do
  cp $R/ab/lgbis/$c/$SO $R/$SO || exit 1
  echo "$c: $(timeout -k 10 120 python $R/scripts/diag/lg_determinism.py 6 2>&1 | tail -1)" >> $OUT/res.txt || exit $?
done
cp /tmp/head_native.so $R/$SO
cat $OUT/res.txt
