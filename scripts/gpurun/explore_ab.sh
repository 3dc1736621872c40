#!/bin/bash
# exploration kernel A/B: GPU explore tests, timing at 200 / 50 nodes with this tree's extension and with the
# one under ab/explore_old (if present), then one PMC pass of this tree's kernel (last: the profiled process can
# segfault in the tool's finalizer after the csv is written)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ex
SO=gsc_amd/_native.cpython-310-x86_64-linux-gnu.so
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_ops.py -k explore $R/tests/test_gpu_explore_pmask.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1 || exit $?
for P in 200 50; do timeout -k 10 120 python $R/scripts/explore_bench.py --n-pad $P --pmask >> $OUT/new.txt 2>&1 || exit $?; done
if [ -f $R/ab/explore_old/$SO ]; then
  cp $R/$SO /tmp/new_native.so && cp $R/ab/explore_old/$SO $R/$SO || exit 1
  for P in 200 50; do timeout -k 10 120 python $R/scripts/explore_bench.py --n-pad $P --pmask >> $OUT/old.txt 2>&1 || exit $?; done
  cp /tmp/new_native.so $R/$SO || exit 1
fi
cd /tmp && export TMPDIR=/tmp && rm -rf $OUT/pmc &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc -o run -- python3 $R/scripts/explore_bench.py --n-pad 200 --pmask --iters 3 > $OUT/pmc.log 2>&1
