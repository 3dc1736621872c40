#!/bin/bash
# Simulator baseline at HEAD: standalone ms/step on 64 CUs and all CUs, the cycle-counting variant, one PMC
# pass of instruction counts per event (one counter group, no trace domains), then the headline bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-simbase}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/scripts/sim_throughput.py --steps 100 --cus 64 > $OUT/sim.txt 2>&1 &&
timeout -k 10 120 python3 $R/scripts/sim_throughput.py --steps 100 >> $OUT/sim.txt 2>&1 &&
timeout -k 10 120 python3 $R/scripts/sim_throughput.py --steps 30 --profile >> $OUT/sim.txt 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM --output-format csv -d $OUT/pmc -o run -- python3 $R/scripts/sim_throughput.py --steps 10 > $OUT/pmc_log.txt 2>&1 &&
python3 $R/scripts/pmc_summary.py $(find $OUT/pmc -name "*counter_collection.csv" | head -1) > $OUT/pmc_summary.txt 2>&1 &&
timeout -k 10 200 python3 $R/bench.py --steps 40 --warmup 5 > $OUT/bench.txt 2>&1
