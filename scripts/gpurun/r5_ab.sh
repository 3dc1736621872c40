#!/bin/bash
# A/B of simulator builds / runtime knobs: CFGS="name:VAR=val,VAR2=val name2:..." (empty assignment list =
# defaults).  Two interleaved rounds of standalone ms/step on the bench's 64-CU partition (and on all CUs
# when ALL=1); optional device==host tests first (TESTS=1) and one PMC pass of the first config last (PMC=1:
# the profiler's finalizer may crash after writing its csv, so nothing runs after it).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-ab}
mkdir -p $OUT
if [ "${TESTS:-0}" = 1 ]; then
  (cd $R && timeout -k 10 300 python -u -m pytest tests/test_gpu_sim.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1) || exit 1
fi
cd /tmp && export TMPDIR=/tmp
for round in 1 2; do
  for c in $CFGS; do
    name=${c%%:*}; assigns=${c#*:}
    envs=$(echo "$assigns" | tr ',' ' ')
    echo "== $name round $round" >> $OUT/sim.txt
    env $envs timeout -k 10 120 python3 $R/scripts/sim_throughput.py --steps 100 --cus 64 ${SIMARGS} >> $OUT/sim.txt 2>&1 || exit 1
    if [ "${ALL:-0}" = 1 ]; then
      env $envs timeout -k 10 120 python3 $R/scripts/sim_throughput.py --steps 100 ${SIMARGS} >> $OUT/sim.txt 2>&1 || exit 1
    fi
  done
done
if [ "${BENCH:-0}" = 1 ]; then
  for c in $CFGS; do
    name=${c%%:*}; envs=$(echo "${c#*:}" | tr ',' ' ')
    echo "== bench $name" >> $OUT/bench.txt
    env $envs timeout -k 10 200 python3 $R/bench.py --steps 40 --warmup 5 >> $OUT/bench.txt 2>&1 || exit 1
  done
fi
if [ "${PMC:-0}" = 1 ]; then
  c=${CFGS%% *}; envs=$(echo "${c#*:}" | tr ',' ' ')
  env $envs timeout -s KILL 90 rocprofv3 --pmc ${PMCS:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_IFETCH} --output-format csv -d $OUT/pmc -o run -- python3 $R/scripts/sim_throughput.py --steps 10 --cus 64 ${SIMARGS} > $OUT/pmc_log.txt 2>&1
  python3 $R/scripts/pmc_summary.py $(find $OUT/pmc -name "*counter_collection.csv" | head -1) > $OUT/pmc_summary.txt 2>&1
fi
exit 0
