#!/bin/bash
# A/B of native builds x event-queue capacity (GSC_SIM_EVENT_CAP): standalone simulator on 64 CUs (the
# bench's partition), the act+sim chain alone (GSC_DIAG_NO_LEARN=1, diagnostic) and the headline bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/ab2.txt
for ev in 128 64; do
  for v in new oldsim; do
    if [ $v = new ]; then unset GSC_NATIVE_SO; else export GSC_NATIVE_SO=$R/ab/_native_$v.cpython-310-x86_64-linux-gnu.so; fi
    export GSC_SIM_EVENT_CAP=$ev
    timeout -k 10 120 python $R/scripts/sim_throughput.py --steps 100 --cus 64 > $OUT/ab_sim.txt 2>&1 || exit $?
    echo "$v ev=$ev sim64: $(grep cus= $OUT/ab_sim.txt)" >> $OUT/ab2.txt
    GSC_DIAG_NO_LEARN=1 timeout -k 10 300 python $R/bench.py --steps 40 --warmup 5 > $OUT/ab_bench.json 2> $OUT/ab_bench.err || exit $?
    echo "$v ev=$ev nolearn: $(cut -c1-120 $OUT/ab_bench.json)" >> $OUT/ab2.txt
    timeout -k 10 300 python $R/bench.py --steps 40 --warmup 5 > $OUT/ab_bench.json 2> $OUT/ab_bench.err || exit $?
    echo "$v ev=$ev bench: $(cut -c1-120 $OUT/ab_bench.json)" >> $OUT/ab2.txt
  done
done
# instruction-cache pressure with 4 simulator waves per CU (64 CUs) vs 1 (all CUs), old vs new build
cd /tmp && export TMPDIR=/tmp
for v in new oldsim; do
  if [ $v = new ]; then unset GSC_NATIVE_SO; else export GSC_NATIVE_SO=$R/ab/_native_$v.cpython-310-x86_64-linux-gnu.so; fi
  export GSC_SIM_EVENT_CAP=128
  for cus in 64 0; do
    rm -rf $OUT/icache_$v_$cus; mkdir -p $OUT/icache_${v}_$cus
    timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $OUT/icache_${v}_$cus -o run -- python3 $R/scripts/sim_throughput.py --steps 10 --cus $cus > $OUT/icache_${v}_$cus/log.txt 2>&1 || exit $?
    python3 $R/scripts/pmc_summary.py $(find $OUT/icache_${v}_$cus -name "*counter_collection.csv" | head -1) > $OUT/icache_${v}_$cus/summary.txt 2>&1
  done
done
