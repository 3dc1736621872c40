#!/bin/bash
# preset benches at HEAD (abilene / syn50 / syn200 at 256 envs x 100 samples per env-step), then the syn200
# timed-window kernel table last (the profiled process can segfault in the tool's finalizer after the
# database is written)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
: > $OUT/r4c6.txt
for p in abilene syn50 syn200; do
  timeout -k 10 400 python $R/bench.py --preset $p --steps ${STEPS:-40} --warmup 5 > $OUT/bench_$p.json 2> $OUT/bench_$p.err || exit $?
  echo "$p: $(cut -c1-400 $OUT/bench_$p.json)" >> $OUT/r4c6.txt
done
cd /tmp && export TMPDIR=/tmp && export GSC_PROF_WINDOW=1 && rm -rf $OUT/prof_syn200 &&
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats -d $OUT/prof_syn200 -o run -- python3 $R/bench.py --preset syn200 --steps 25 --warmup 3 > $OUT/prof_syn200.log 2>&1
