#!/bin/bash
# one PMC pass over the sparse critic products at config-5 shapes (PMC="<counters>", PASS=<name>)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
P=${PASS:-a}
cd /tmp && export TMPDIR=/tmp && rm -rf $OUT/sppmc_$P &&
timeout -s KILL 120 rocprofv3 --pmc ${PMC:-SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE} --output-format csv -d $OUT/sppmc_$P -o run -- python3 $R/scripts/sparse_bench.py --B 25600 --R 1800 --P 200 --iters 2 > $OUT/sppmc_$P.log 2>&1
