#!/bin/bash
# PMC passes (counters only, no trace domains) over the GNN micro-benchmark
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/gnn_pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES --output-format csv -d $OUT/p1 -o run -- python3 $R/scripts/gnn_bench.py --iters 3 > $OUT/p1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/p2 -o run -- python3 $R/scripts/gnn_bench.py --iters 3 > $OUT/p2.log 2>&1
