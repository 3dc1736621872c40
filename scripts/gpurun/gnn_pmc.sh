#!/bin/bash
# One PMC pass (counters only, no trace domains) over the GNN micro-benchmark: PASS=<name> PMC="<counters>"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/gnn_pmc
mkdir -p $OUT
PMC=${PMC:-SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES}
PASS=${PASS:-p}
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 90 rocprofv3 --pmc $PMC --output-format csv -d $OUT/$PASS -o run -- python3 $R/scripts/gnn_bench.py --iters 3 > $OUT/$PASS.log 2>&1
