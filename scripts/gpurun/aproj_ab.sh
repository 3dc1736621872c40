#!/bin/bash
# actor_proj microbenchmark: the in-tree build vs the A/B builds named in VARIANTS (ab/_native_<v>.so)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/aproj_ab.txt
for v in new ${VARIANTS:-aprojold}; do
  if [ $v = new ]; then unset GSC_NATIVE_SO; else export GSC_NATIVE_SO=$R/ab/_native_$v.cpython-310-x86_64-linux-gnu.so; fi
  timeout -k 10 120 python $R/scripts/aproj_bench.py $ARGS > $OUT/aproj_v.txt 2>&1 || exit $?
  echo "$v $(grep actor_proj $OUT/aproj_v.txt)" >> $OUT/aproj_ab.txt
done
