#!/bin/bash
# large-graph fused GATv2: numerics, micro-benchmark (lg vs layer-wise), one PMC pass over the micro-benchmark
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/lgperf.txt
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_gnn_lg.py -x -v --timeout 120 --timeout-method thread > $OUT/lg_tests.log 2>&1 || { echo "lg tests failed" >> $OUT/lgperf.txt; exit 1; }
echo "lg tests: $(tail -1 $OUT/lg_tests.log)" >> $OUT/lgperf.txt
timeout -k 10 200 python -u $R/scripts/diag/lg_err.py 8 22 >> $OUT/lgperf.txt 2>&1 || exit $?
for lg in 1 0; do
  GSC_GNN_LG=$lg timeout -k 10 200 python $R/scripts/gnn_bench.py --network configs/networks/synthetic/syn200-in16-cap1-3-s0.graphml --n-pad 200 --batch 25600 --iters 5 > $OUT/gb.txt 2>&1 || exit $?
  echo "GSC_GNN_LG=$lg $(tail -1 $OUT/gb.txt)" >> $OUT/lgperf.txt
done
cd /tmp && export TMPDIR=/tmp && rm -rf $OUT/lg_pmc &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/lg_pmc -o run -- python3 $R/scripts/gnn_bench.py --network configs/networks/synthetic/syn200-in16-cap1-3-s0.graphml --n-pad 200 --batch 25600 --iters 2 > $OUT/lg_pmc.log 2>&1
