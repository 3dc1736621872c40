#!/bin/bash
# one iteration on the large-graph kernels: numerics, phase profile, micro-benchmark (both backward lane groupings)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/lgiter.txt
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_gnn_lg.py -x -v --timeout 120 --timeout-method thread > $OUT/lg_tests.log 2>&1 || { echo "lg tests failed" >> $OUT/lgiter.txt; exit 1; }
echo "lg tests: $(tail -1 $OUT/lg_tests.log)" >> $OUT/lgiter.txt
for nl in ${NLS:-4 2}; do
  GSC_LG_BWD_NL=$nl timeout -k 10 200 python $R/scripts/gnn_bench.py --network configs/networks/synthetic/syn200-in16-cap1-3-s0.graphml --n-pad 200 --batch 25600 --iters 5 > $OUT/gb.txt 2>&1 || exit $?
  echo "NL=$nl $(tail -1 $OUT/gb.txt)" >> $OUT/lgiter.txt
done
if [ -n "${ERR:-}" ]; then LG_MODES=1 timeout -k 10 200 python -u $R/scripts/diag/lg_err.py $ERR >> $OUT/lgiter.txt 2>&1; fi
if [ -n "${PHASES:-}" ]; then timeout -k 10 200 python -u $R/scripts/diag/lg_phases.py >> $OUT/lgiter.txt 2>&1; fi
