#!/bin/bash
# Simulator iteration check: device == host bit-exact tests, standalone ms/step (64 CUs = the bench's
# partition, and all CUs), one PMC pass of instructions per event, then the headline bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-simab}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_sim.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 120 python3 $R/scripts/sim_throughput.py --steps 100 --cus 64 > $OUT/sim.txt 2>&1 &&
timeout -k 10 120 python3 $R/scripts/sim_throughput.py --steps 100 >> $OUT/sim.txt 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM --output-format csv -d $OUT/pmc -o run -- python3 $R/scripts/sim_throughput.py --steps 10 > $OUT/pmc_log.txt 2>&1 &&
python3 $R/scripts/pmc_summary.py $(find $OUT/pmc -name "*counter_collection.csv" | head -1) > $OUT/pmc_summary.txt 2>&1 &&
timeout -k 10 200 python3 $R/bench.py --steps 40 --warmup 5 > $OUT/bench.txt 2>&1
