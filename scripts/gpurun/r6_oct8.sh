#!/bin/bash
# octet exploration kernel: this tree vs ab/oct8 (amdgpu_waves_per_eu(8, 8)), interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/oct8
SO=gsc_amd/_native.cpython-310-x86_64-linux-gnu.so
mkdir -p $OUT
cd $R
cp $SO /tmp/base.so || exit 1
: > $OUT/ab.txt
for i in 1 2; do
  cp /tmp/base.so $SO && echo "base $(timeout -k 10 120 python scripts/explore_bench.py --n-pad 200 --pmask 2>&1 | grep explore | tr '\n' ' ')" >> $OUT/ab.txt || exit 1
  cp ab/oct8/$SO $SO && echo "oct8 $(timeout -k 10 120 python scripts/explore_bench.py --n-pad 200 --pmask 2>&1 | grep explore | tr '\n' ' ')" >> $OUT/ab.txt || exit 1
done
cp /tmp/base.so $SO
cat $OUT/ab.txt
