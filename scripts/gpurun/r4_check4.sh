#!/bin/bash
# gnn_mt NVS / row-image sizing (syn50 bench + one PMC pass last: the profiled process may segfault at
# exit), staged (coalesced) 200-node GNN kernels first (numerics), then the restored simulator layout (64 / 128 / all
# CUs, hint variant on 64), the headline bench x2, config-5 bench staged vs VALU lane kernels, smoke
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/r4c4.txt
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_gnn_lw.py -x -v --timeout 120 --timeout-method thread > $OUT/gnn_lw.log 2>&1 || exit $?
echo "gnn_lw: $(tail -1 $OUT/gnn_lw.log)" >> $OUT/r4c4.txt
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_ops.py -x -v -k "gnn" --timeout 120 --timeout-method thread > $OUT/gnn_ops.log 2>&1 || exit $?
echo "gnn_ops: $(tail -1 $OUT/gnn_ops.log)" >> $OUT/r4c4.txt
timeout -k 10 300 python $R/bench.py --preset syn50 --steps 10 --warmup 3 > $OUT/b50.json 2> $OUT/b50.err || exit $?
echo "syn50: $(cut -c1-200 $OUT/b50.json)" >> $OUT/r4c4.txt
for cus in 64 128 0; do
  timeout -k 10 120 python $R/scripts/sim_throughput.py --steps 100 --cus $cus > $OUT/ab_sim.txt 2>&1 || exit $?
  echo "sim: $(grep cus= $OUT/ab_sim.txt)" >> $OUT/r4c4.txt
done
GSC_NATIVE_SO=$R/ab/_native_hint.cpython-310-x86_64-linux-gnu.so timeout -k 10 120 python $R/scripts/sim_throughput.py --steps 100 --cus 64 > $OUT/ab_sim.txt 2>&1 || exit $?
echo "hint sim: $(grep cus= $OUT/ab_sim.txt)" >> $OUT/r4c4.txt
for k in 1 2; do
  timeout -k 10 300 python $R/bench.py --steps 40 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit $?
  echo "bench: $(cut -c1-160 $OUT/bench.json)" >> $OUT/r4c4.txt
done
for mf in 1 0; do
  GSC_LW_MFMA=$mf timeout -k 10 400 python $R/bench.py --preset syn200 --envs 256 --batch-size 25600 --steps 6 --warmup 3 > $OUT/b200.json 2> $OUT/b200.err || exit $?
  echo "syn200 full mf=$mf: $(cut -c1-200 $OUT/b200.json)" >> $OUT/r4c4.txt
done
timeout -k 10 300 python -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc50 -o run -- python3 $R/bench.py --preset syn50 --steps 3 --warmup 2 > $OUT/pmc50.log 2>&1
