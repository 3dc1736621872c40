#!/bin/bash
# one PMC pass (counters only) over a short bench run of PRESET (default syn200), counters in PMC; the
# profiled process can segfault in the tool's finalizer after the csv is written (last GPU step)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
P=${PRESET:-syn200}
cd /tmp && export TMPDIR=/tmp && rm -rf $OUT/pmc_$P &&
timeout -s KILL 200 rocprofv3 --pmc ${PMC:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_ANY TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE} --output-format csv -d $OUT/pmc_$P -o run -- python3 $R/bench.py --preset $P --steps 3 --warmup 2 > $OUT/pmc_$P.log 2>&1
