#!/bin/bash
# per-kernel mean times of the headline bench for ab/head and this tree (rocprofv3 --kernel-trace --stats, no markers)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/abp
SO=gsc_amd/_native.cpython-310-x86_64-linux-gnu.so
PY=gsc_amd/ops/explore.py
mkdir -p $OUT
cd $R
cp $SO /tmp/new.so && cp $PY /tmp/new_explore.py || exit 1
cp ab/head/$SO $SO && cp ab/head/$PY $PY || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/head -o run -- python3 $R/bench.py --steps 40 --warmup 5 > $OUT/head.log 2>&1 || exit $?
cp /tmp/new.so $R/$SO && cp /tmp/new_explore.py $R/$PY || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/new -o run -- python3 $R/bench.py --steps 40 --warmup 5 > $OUT/new.log 2>&1
