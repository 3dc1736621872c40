#!/bin/bash
# one PMC pass over the GNN micro-benchmark at config-5 shapes (PMC="<counters>", PASS=<name>)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
P=${PASS:-a}
cd /tmp && export TMPDIR=/tmp && rm -rf $OUT/lgpmc_$P &&
timeout -s KILL 120 rocprofv3 --pmc ${PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE} --output-format csv -d $OUT/lgpmc_$P -o run -- python3 $R/scripts/gnn_bench.py --network configs/networks/synthetic/syn200-in16-cap1-3-s0.graphml --n-pad 200 --batch 25600 --iters 2 > $OUT/lgpmc_$P.log 2>&1
