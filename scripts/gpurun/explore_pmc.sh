#!/bin/bash
# exploration kernel: timing at one slice per wave vs grid-stride grids, then one PMC pass (last GPU step:
# the profiled process can segfault in the tool's finalizer after the csv is written)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ex
mkdir -p $OUT
for b in 0 4 16; do
  GSC_EXPLORE_BLOCKS_PER_CU=$b timeout -k 10 120 python $R/scripts/explore_bench.py --n-pad 200 --pmask > $OUT/grid_$b.txt 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp && rm -rf $OUT/pmc &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc -o run -- python3 $R/scripts/explore_bench.py --n-pad 200 --pmask --iters 3 > $OUT/pmc.log 2>&1
