#!/bin/bash
# simulator layout variants on the bench's 64-CU partition (GSC_NATIVE_SO builds under ab/), then the
# config-5 (equal learner work) timed-window kernel table
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/ab4.txt
for k in 1 2; do
  for v in ${VARIANTS:-new hint oldsim}; do
    if [ $v = new ]; then unset GSC_NATIVE_SO; else export GSC_NATIVE_SO=$R/ab/_native_$v.cpython-310-x86_64-linux-gnu.so; fi
    timeout -k 10 120 python $R/scripts/sim_throughput.py --steps 100 --cus 64 > $OUT/ab_sim.txt 2>&1 || exit $?
    echo "$v sim64: $(grep cus= $OUT/ab_sim.txt)" >> $OUT/ab4.txt
    if [ $k = 1 ]; then
      timeout -k 10 300 python $R/bench.py --steps 40 --warmup 5 > $OUT/ab_bench.json 2> $OUT/ab_bench.err || exit $?
      echo "$v bench: $(cut -c1-130 $OUT/ab_bench.json)" >> $OUT/ab4.txt
    fi
  done
done
unset GSC_NATIVE_SO
cd /tmp && export TMPDIR=/tmp && export GSC_PROF_WINDOW=1 && rm -rf $OUT/prof_syn200full &&
timeout -k 10 500 rocprofv3 --kernel-trace --marker-trace --stats -d $OUT/prof_syn200full -o run -- python3 $R/bench.py --preset syn200 --envs 256 --batch-size 25600 --steps 4 --warmup 3 > $OUT/prof_syn200full.log 2>&1
