#!/bin/bash
# PMC passes over the simulator-only loop (one counter group per run, no trace domains).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/simpmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1
run() {
  mkdir -p $OUT/$1
  timeout -s KILL 90 rocprofv3 --pmc $2 --output-format csv -d $OUT/$1 -o run -- python3 $R/scripts/sim_throughput.py --steps 10 > $OUT/$1/log.txt 2>&1
  python3 $R/scripts/pmc_summary.py $(find $OUT/$1 -name "*counter_collection.csv" | head -1) 3 > $OUT/$1/summary.txt 2>&1
}
run wait "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_INSTS_VALU SQ_INSTS_SALU"
run icache "SQC_ICACHE_HITS SQC_ICACHE_MISSES"
run lds "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAVES SQ_INSTS_BRANCH"
exit 0
