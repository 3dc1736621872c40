#!/bin/bash
# fused Adam: ab/head vs this tree at the config-5 actor size (interleaved), then the learner / DP tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/adam
SO=gsc_amd/_native.cpython-310-x86_64-linux-gnu.so
mkdir -p $OUT
cd $R
cp $SO /tmp/new.so || exit 1
: > $OUT/ab.txt
for i in 1 2; do
  cp ab/head/$SO $SO && echo "head $(timeout -k 10 120 python scripts/adam_bench.py 2>&1 | tail -1)" >> $OUT/ab.txt || exit 1
  cp /tmp/new.so $SO && echo "new  $(timeout -k 10 120 python scripts/adam_bench.py 2>&1 | tail -1)" >> $OUT/ab.txt || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_learner.py tests/test_gpu_dp.py tests/test_gpu_ops.py -k "adam or learner or dp or rccl" -x -v --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1 || exit $?
cat $OUT/ab.txt
