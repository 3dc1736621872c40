#!/bin/bash
# instruction-cache counters of the simulator kernel, all CUs vs a 96-CU stream (counters only)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/sim_icache
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp &&
for c in 0 96; do
  timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAIT_INST_ANY SQ_IFETCH SQ_WAVE_CYCLES --output-format csv -d $OUT/c$c -o run -- python3 $R/scripts/sim_throughput.py --steps 20 --cus $c > $OUT/c$c.log 2>&1 || exit 1
done
